// ipt_knobs.h — the path kernel's build-time parameters. Every switch below
// selects between EXACT forms (bit-identical results; the parity tests pass
// with either value); the defaults are the measured best. A
// build that overrides any of them must say so with -DIPT_AB_BUILD (A/B
// measurement builds, scripts/variants*.sh), so that a stray -D cannot slip
// into the product library unnoticed.
#pragma once

#if !defined(IPT_AB_BUILD) &&                                                                           \
    (defined(IPT_BLOCK) || defined(IPT_RES_BLOCK) || defined(IPT_RESUME) || defined(IPT_RESUME_LIGHTS) || defined(IPT_SPHERE_GRID) || \
     defined(IPT_GRID_BUDGET) || defined(IPT_GRID_LDS) || defined(IPT_GRID_LDS_BLOCK) || defined(IPT_GRID_INLINE) || defined(IPT_GRID_C4) || defined(IPT_GRID_ITEMS) || defined(IPT_GRID_PIPE) || defined(IPT_GRID_WAVE) || defined(IPT_GRID_WAVE_PIPE) || defined(IPT_GRID_WAVE_UNC) || defined(IPT_GRID_WAVE_FLOOR) || defined(IPT_GRID_WAVE_FLOOR_IT) ||                   \
     defined(IPT_WALK_BUDGET) || defined(IPT_LWALK_BUDGET) || defined(IPT_WAVES_PER_SIMD) ||           \
     defined(IPT_RES_WAVES) || defined(IPT_RES_HOLD) || defined(IPT_LIGHT_HOLD) || defined(IPT_RESL_WAVES) || defined(IPT_BOXDIV) || defined(IPT_LPF) || defined(IPT_LPF_CALC) || defined(IPT_LTR_CALC) || defined(IPT_FRAME_PF) || defined(IPT_FRAME_FB_PF) ||      \
     defined(IPT_LIGHT_INR) || defined(IPT_LIGHT_AXIS) || defined(IPT_LIGHT_GRID) || defined(IPT_CDF_LO) || defined(IPT_CDF_POW2) || defined(IPT_PICK_INT) || defined(IPT_PICK_INT_CDF) || defined(IPT_CDF_EXACT) || defined(IPT_LIGHT_AX_REC) || defined(IPT_LAX_LDS) || \
     defined(IPT_RAYGEN) || defined(IPT_FRAME_TAB) || defined(IPT_FRAME_TAB_LISTS) || defined(IPT_C2_ONLY) || defined(IPT_C2_LMODE) ||  \
     defined(IPT_BVH_LEAF) || defined(IPT_LBVH_LEAF) || defined(IPT_GRID_CELLS_PER_SPHERE) || defined(IPT_GRID_SPHERE_REG) || \
     defined(IPT_COSB_TAB) || defined(IPT_SKIP_AHEAD) || defined(IPT_PRE_SKIP))
#error "an ipt_knobs.h parameter is overridden: A/B builds must define IPT_AB_BUILD"
#endif

// ---- launch shape
#ifndef IPT_BLOCK
#define IPT_BLOCK 256  // threads per workgroup (4 waves; 128 / 512 measured -2 % / -7 %)
#endif
#ifndef IPT_RES_BLOCK
#define IPT_RES_BLOCK 64  // threads per workgroup of the sphere-list instances (C3: 64 / 128 / 256 -> 15.13 / 14.90 / 14.80)
#endif
#ifndef IPT_WAVES_PER_SIMD
#define IPT_WAVES_PER_SIMD 4  // __launch_bounds__ occupancy of the non-resumable instances
#endif
#ifndef IPT_RES_WAVES
#define IPT_RES_WAVES 4  // ... of the resumable sphere-list instances (C3: 3 -> 4 waves +12 %)
#endif
#ifndef IPT_RESL_WAVES
#define IPT_RESL_WAVES 3  // ... of the resumable many-light (light BVH) instances
#endif
#ifndef IPT_LIGHT_HOLD
#define IPT_LIGHT_HOLD 1  // the single light held in VGPRs (vgpr_hold) by the non-resumable instances (+3.5 % C2)
#endif
#ifndef IPT_RES_HOLD
#define IPT_RES_HOLD 0  // sphere-list instances hold the single light and the grid parameters in
                        // VGPRs (+5 % at 3 waves; at 4 waves the registers are needed, -30 %)
#endif

// ---- structure (each also has a runtime or scene condition)
#ifndef IPT_RAYGEN
#define IPT_RAYGEN 1  // new paths' camera ray + Philox block 0 precomputed by raygen_kernel (+4.8 % C2)
#endif
#ifndef IPT_FRAME_TAB
#define IPT_FRAME_TAB 1  // RotateDdf angle (sin, cos) from the exact 1 GiB frame table (+8.6 % C2)
#endif
#ifndef IPT_FRAME_TAB_LISTS
#define IPT_FRAME_TAB_LISTS 0  // ... for the sphere-list (C3) frames too
#endif
#ifndef IPT_FRAME_PF
#define IPT_FRAME_PF 3  // 3: the next step's frame-table entry gathered at the end of the step
                        // (0: in the frame pass; gathering it right after the geometry trace,
                        // or at the step's end with a predicted node, measured slower)
#endif
#ifndef IPT_FRAME_FB_PF
#define IPT_FRAME_FB_PF 0  // IPT_FRAME_PF == 3: the out-of-table angle (|to.z| < 2^-8) computed in the
                           // end-of-step prefetch too (the frame phase then reads it unconditionally)
#endif
#ifndef IPT_BOXDIV
#define IPT_BOXDIV 1  // box planes' divisions without range handling (origins within 2^39)
#endif
#ifndef IPT_LIGHT_AXIS
#define IPT_LIGHT_AXIS 1  // axis-aligned single-light instances (kLightsOneA10/A01, +1.7 % C2)
#endif
#ifndef IPT_LIGHT_INR
#define IPT_LIGHT_INR 1  // ... with the range-free roots / quotients of light_ranges_box (+4.9 % C2)
#endif
#ifndef IPT_LIGHT_GRID
#define IPT_LIGHT_GRID 1  // coplanar light lattices by cell lookup (kLightsGridA10/A01; C5 3x)
#endif
#ifndef IPT_SKIP_AHEAD
#define IPT_SKIP_AHEAD 1  // single axis-aligned light: a certain light-sample skip and the next pick in one step
#endif
#ifndef IPT_PRE_SKIP
#define IPT_PRE_SKIP 1  // skip-ahead instances with the end-of-step pop: the next iteration's certain skip
                        // taken at the end of the step (before the pop)
#endif
#ifndef IPT_COSB_TAB
#define IPT_COSB_TAB 0  // non-resumable instances: CosineDdf's (cos phi, sin phi) gathered from the 128 MiB table
                        // (C2 358 -> 256, C5 296 -> 256 Mpaths/s: the second random table line per cosine
                        // iteration, round 5)
#endif
#ifndef IPT_LPF
#define IPT_LPF 1  // lattice instances: the picked light's sample fields gathered in the prologue (C5 +2 %)
#endif
#ifndef IPT_LPF_CALC
#define IPT_LPF_CALC 0  // ... computed from the light index where every light matches the lattice formula
                        // (C5 327.9 -> 323.1 Mpaths/s: the LDS read is cheaper than the formula, round 6)
#endif
#ifndef IPT_LTR_CALC
#define IPT_LTR_CALC 0  // ... and the light tests' records and cell lookup too (only the weight is read)
                        // (C5 -> 310.9 Mpaths/s with IPT_LPF_CALC, round 6)
#endif
#ifndef IPT_LIGHT_AX_REC
#define IPT_LIGHT_AX_REC 1  // lattice lights read from 48-byte compact records (three 16-byte loads)
#endif
#ifndef IPT_LAX_LDS
#define IPT_LAX_LDS 1  // lattice lights' records in LDS, one 1024-thread workgroup per CU (C5 +5 %)
#endif
#ifndef IPT_GRID_C4
#define IPT_GRID_C4 1  // pipelined grid walk: items as packed 16-byte records, indices apart (C3 +1.5 %)
#endif
#ifndef IPT_CDF_LO
#define IPT_CDF_LO 1  // many lights: the pick's scan started from a 256-bucket table (+7 % C5)
#endif
#ifndef IPT_PICK_INT
#define IPT_PICK_INT 1  // the single light's pick and the pre-skip's light test on the raw draw words
#endif
#ifndef IPT_PICK_INT_CDF
#define IPT_PICK_INT_CDF 1  // the near-uniform many-light pick (IPT_CDF_POW2) on the draw's 24-bit integer
#endif
#ifndef IPT_CDF_EXACT
#define IPT_CDF_EXACT 1  // ... and when every light's integer threshold is exactly (i+1) 2^(24-e): no cdf read
#endif
#ifndef IPT_CDF_POW2
#define IPT_CDF_POW2 1  // many lights whose cdf is within 2^-e/2 of (i+1) 2^-e: the pick from floor(r 2^e)
                        // and two cdf entries (no bucket table read)
#endif
#ifndef IPT_SPHERE_GRID
#define IPT_SPHERE_GRID 1  // uniform grid instead of the BVH for large sphere lists inside the box
#endif
#ifndef IPT_RESUME
#define IPT_RESUME 1  // sphere-list walks bounded per step and resumed in later steps
#endif
#ifndef IPT_RESUME_LIGHTS
#define IPT_RESUME_LIGHTS 1  // light-BVH walks bounded per step and resumed (many-light scenes)
#endif
#ifndef IPT_GRID_PIPE
#define IPT_GRID_PIPE 1  // resumable grid walk pipelined: next cell's range + IPT_GRID_ITEMS loads in flight (C3 +11 %)
#endif

#ifndef IPT_GRID_WAVE
#define IPT_GRID_WAVE 1  // resumable grid walk with the item tests spread over the wave's lanes (C3 +14 %)
#endif
#ifndef IPT_GRID_WAVE_UNC
#define IPT_GRID_WAVE_UNC 1  // ... every lane loads an item per round, waited for outside the test's branch
#endif
#ifndef IPT_GRID_WAVE_PIPE
#define IPT_GRID_WAVE_PIPE 0  // ... with the first two rounds' item loads issued together
#endif
#ifndef IPT_GRID_WAVE_FLOOR
#define IPT_GRID_WAVE_FLOOR 0  // ... ended early once fewer lanes than this walk
#endif
#ifndef IPT_GRID_WAVE_FLOOR_IT
#define IPT_GRID_WAVE_FLOOR_IT 0  // ... but not before this many cell iterations
#endif
// the two-cell wave walk reads the packed items and their separate index array
static_assert(IPT_GRID_WAVE != 2 || IPT_GRID_C4, "IPT_GRID_WAVE=2 needs IPT_GRID_C4 (kp.grid_c4 / grid_idx)");

// ---- walk budgets and acceleration-structure parameters
#ifndef IPT_GRID_LDS
#define IPT_GRID_LDS 0  // sphere-list instances: the grid's cell ranges packed and staged in LDS, one
                        // IPT_GRID_LDS_BLOCK-thread workgroup per CU sharing them
#endif
#ifndef IPT_GRID_LDS_BLOCK
#define IPT_GRID_LDS_BLOCK 896
#endif
#ifndef IPT_GRID_INLINE
#define IPT_GRID_INLINE 0  // 1: the grid walk over 64-byte cell records (range + first 3 items inline): C3 -9 %
#endif
#ifndef IPT_GRID_BUDGET
#define IPT_GRID_BUDGET 8  // grid cells per lane per step of a resumable walk (wave walk: 6-32 measured;
                           // the per-lane walk: 4-16, best 5)
#endif
#ifndef IPT_GRID_ITEMS
#define IPT_GRID_ITEMS 3  // item loads issued together per inner iteration of the pipelined grid walk (1-4)
#endif
#ifndef IPT_WALK_BUDGET
#define IPT_WALK_BUDGET 48  // sphere-BVH node visits per lane per step of a resumable walk
#endif
#ifndef IPT_LWALK_BUDGET
#define IPT_LWALK_BUDGET 16  // light-BVH nodes per lane per step of a resumable walk
#endif
#ifndef IPT_BVH_LEAF
#define IPT_BVH_LEAF 16  // sphere BVH: median split down to this many spheres (ipt_bvh.h)
#endif
#ifndef IPT_LBVH_LEAF
#define IPT_LBVH_LEAF 2  // light BVH leaf size
#endif
#ifndef IPT_GRID_CELLS_PER_SPHERE
#define IPT_GRID_CELLS_PER_SPHERE 1.5  // C3 sweep: 0.75-12, best 1.5 with a 5-cell budget
#endif

#ifndef IPT_GRID_SPHERE_REG
#define IPT_GRID_SPHERE_REG 1  // grid cells register a sphere only where its padded ball reaches them
#endif

// ---- experiment builds: -DIPT_AB_BUILD -DIPT_C2_ONLY=1 instantiates the
// sample_scenes[0] kernel alone (seconds to compile); other scenes fail loudly
#ifndef IPT_C2_ONLY
#define IPT_C2_ONLY 0
#endif
#ifndef IPT_C2_LMODE
#define IPT_C2_LMODE kLightsOneA10
#endif
