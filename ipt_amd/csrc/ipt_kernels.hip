// ipt_kernels.hip — gfx950 kernels and the C-ABI (include/ipt_capi.h) of the
// ipt path-tracing inner loop.
//
// Kernels
//   path_kernel        persistent megakernel: one lane = one path (camera
//                      sample) at a time; the reference's recursive branching
//                      estimator (main.cpp:98-184) runs as an explicit DFS
//                      with the suspended ancestors in LDS and the current
//                      node in registers; lanes refill from a wave-local pool
//                      of work units fed by one global atomic per 256 units.
//                      Writes the per-sample radiance + GridRenderPlane drift
//                      code of every (pass, source pixel).
//   accumulate_kernel  one thread per destination pixel: replays
//                      GridRenderPlane::addRay (GridRenderPlane.cpp:61-75) for
//                      all passes in render_sample order — coalesced reads of
//                      the radiance buffer, HBM-bound.
// Build: see __graft_entry__.py (hipcc --offload-arch=gfx950 -O3
//        -ffp-contract=off, no fast-math).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/ipt_capi.h"
#include "ipt_bvh.h"
#include "ipt_internal.h"
#include "ipt_path.h"
#include "ipt_knobs.h"
#include "ipt_diag.h"

using namespace ipt;

namespace {

constexpr int kBlock = IPT_BLOCK;  // threads per workgroup (4 waves; ipt_knobs.h)
template <typename T>
__device__ __forceinline__ void keep_alive(const T& v) {
    const float* p = reinterpret_cast<const float*>(&v);
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) asm volatile("" ::"v"(p[i]));
}
constexpr int kStackFields = 6;   // pos3, res, mult, meta(i | kind<<8)
constexpr int kPoolChunk = 256;   // work units per global atomic
constexpr int kNumCounters = 15;

struct KParams {
    int W, H, spp, spp_offset, n_rays, depth_max;
    int meta_shift;  // a suspended level's meta word: ti | kind << meta_shift (8, or 16 for n_rays > 255)
    uint32_t key0, key1;
    int n_cand;              // candidate source rows
    const int* __restrict__ cand_rows;    // [n_cand] source row index
    int tile_rows, n_shards, shard_id;
    unsigned long long total_units;
    unsigned long long* unit_counter;
    // the launch's pool-drained flag (signal memory, hipStreamWaitValue64's
    // operand): the wave that takes the last chunk stores drain_seq there
    unsigned long long* drained;
    unsigned long long drain_seq;
#if IPT_RAYLOG
    RayLogRec* raylog;               // [raylog_cap]
    unsigned long long* raylog_n;    // finished traces seen
    unsigned long long raylog_cap;
    unsigned raylog_every;
#endif
    float* __restrict__ values;           // [spp][n_cand][W]
    uint8_t* __restrict__ codes;          // [spp][n_cand][W]
    uint8_t* __restrict__ flags;          // [H][W]
    unsigned long long* counters;
    int geometry_kind;
    int n_lights;
    const LightDev* __restrict__ lights;  // [n_lights]
    const float* __restrict__ weights;    // [n_lights+1]
    const float* __restrict__ cdf;        // [n_lights+1] sequential prefix sums of weights
    const Frame* __restrict__ wall_frames;  // [5]
    vec3 cam_pos, cam_dir, cam_right, cam_up;
    int n_spheres;
    const float4* __restrict__ spheres;   // (c.xyz, r)
    float bvh_tmargin;                    // sphere BVH / grid: additive pruning margin (1e-3 D, ipt_bvh.h)
    int n_grid;                           // > 0: uniform sphere grid (ipt_bvh.h SphereGrid) instead of the BVH
    float grid_g0[3], grid_h[3], grid_inv_h[3], grid_m;
    float grid_g1[3];                     // g0 + (float)n * h, the grid's far corner (host-computed)
    int grid_n[3];
    const int* __restrict__ grid_start;   // [cells + 1]
    // IPT_GRID_LDS: grid_start packed for LDS staging -- [grid_packed_nb] u32
    // bases of 8-entry blocks, then [cells + 1] u8 offsets from them
    const int* __restrict__ grid_packed;
    int grid_packed_words, grid_packed_nb;
    const GridCell* __restrict__ grid_cells;  // [cells] range + first three items (IPT_GRID_INLINE)
    const BvhSphere* __restrict__ grid_items;
    // the same items packed for the pipelined walk (IPT_GRID_C4): centre and
    // radius as one float4 per item (16-byte stride: a cell's items share
    // lines), original indices in a separate array
    const float4* __restrict__ grid_c4;
    const int* __restrict__ grid_idx;
    const BvhNode* __restrict__ bvh_nodes;     // n_nodes > 0: sphere BVH (ipt_bvh.h)
    const BvhSphere* __restrict__ bvh_prims;
    int n_nodes;
    const BvhNode* __restrict__ light_nodes;   // n_light_nodes > 0: light BVH over index ranges
    int n_light_nodes;
    int lnodes_lds;                       // light BVH staged in LDS (kLightsGlobal)
    // kLightsGridA10/A01: coplanar axis-aligned lights on a lattice (LightGrid)
    const int* __restrict__ lgrid;        // [lg_nu * lg_nv] light index per cell, -1 = none
    const float4* __restrict__ lax;       // [n_lights][3] LightAx records (IPT_LIGHT_AX_REC)
    int lg_nu, lg_nv;
    float lg_u0, lg_v0, lg_icw, lg_ich;   // cell coordinates: (q - u0) * icw
    float lg_e;                           // candidate margin in cells (LightGrid::e)
    // skip-ahead (prologue): every light sample's point lies on the plane z =
    // sa_pz and the light normal is (+-0, +-0, sa_nz): light picks at nodes
    // with sa_nz * (sa_pz - z) >= 0 are certain skips (sa_on, host-checked)
    // u01(w) < c  <=>  w < (ceil(c 2^24) << 8) (clamped to [0, 2^32]) for the
    // draw word w: the single light's cdf[0], cdf[1] (pk_u0, pk_u1) and sa_cl
    // (sa_u) as word thresholds (host: word_threshold)
    unsigned long long pk_u0, pk_u1, sa_u;
    int sa_on;
    float sa_pz, sa_nz;
    // a pick r < sa_cl is a light pick (one light: cdf[0]; a lattice with a
    // non-decreasing cdf: cdf[nl - 1]; else 0, never)
    float sa_cl;
    float lg_pn, lg_nn;                   // the lights' shared plane: P[na], n[na]
    int cdf_bsearch;                      // cdf non-decreasing: pick by binary search
    // |cdf[i] - (i+1) 2^-e| < 2^-e/2 for every light i and a non-decreasing
    // cdf (host-checked): the pick is floor(r 2^e) - 1, + 0 or + 1 by two cdf
    // entries, then cdf[nl] decides past the lights (cdf_p2s = 2^e)
    int cdf_p2;  // 1: near-uniform as above; 2: every threshold exact (KParams::cdf_p2e)
    float cdf_p2s, cdf_end;
    // the same pick on the draw's 24-bit integer g = w >> 8 (IPT_PICK_INT_CDF):
    // floor(r 2^e) = g >> (24 - e) and r < c <=> g < ceil(c 2^24); the staged
    // cdf then holds those integer thresholds (cdf_end_t: cdf[nl]'s)
    int cdf_p2e;
    uint32_t cdf_end_t;
    // IPT_LPF_CALC: the lattice lights' sample fields are a formula of the
    // light index i (host-checked for every light): P.x = lc_x0 + (float)(i &
    // (2^lc_shift - 1)) * lc_dx, P.y = lc_y0 + (float)(i >> lc_shift) * lc_dy,
    // x[XA] = lc_ax, y[YA] = lc_ay (C5's 16 x 16 split light, built that way)
    int lpf_calc, lc_shift;
    float lc_x0, lc_y0, lc_dx, lc_dy, lc_ax, lc_ay;
    // IPT_LTR_CALC (with lpf_calc): every lattice light's inverse entries,
    // area and power are the same (lc_ix .. lc_spow), so a light test reads
    // only the light's weight; lg_ident 1 / 2: cell (i, j) holds light
    // i + nu j / j + nv i (every cell, host-checked), no cell read
    int ltr_calc, lg_ident;
    float lc_ix, lc_iy, lc_area, lc_spow;
    const int* __restrict__ cdf_lo;       // [kCdfBuckets] or null: first c with cdf[c] > b/256
    double inv_per_pass, inv_w;           // 1/(n_cand*W), 1/W (exact 32-bit unit decomposition)
    uint32_t per_pass32;                  // n_cand*W (< 2^32)
    int box_inrange;                      // camera and sphere list within 2^39 (box_plane_t<true>)
    const float* __restrict__ cos_a;      // [2^24] CosineDdf table by u1's 24 bits: sin(acos(sqrt(u1)))
    const float2* __restrict__ cos_b;     // [2^24] by u2's 24 bits: (cos phi, sin phi)
    const float2* __restrict__ frame_sc;  // frame_table_kernel: RotateDdf angle (sin, cos) by to.z
    const uint4* __restrict__ rg;         // IPT_RAYGEN: [total_units][2] raygen_kernel records
    int count;                            // raygen_kernel: accumulate the drift counter
};

// floor(n / d) for 32-bit n, d >= 1 from a double reciprocal: the estimate's
// error is below (n/d) * 2^-51 < 1/d (n < 2^32), i.e. below the distance of a
// non-integer n/d from the next integer, so it truncates to the quotient or,
// when n/d is an integer approached from below, to one less (fixed up).
__host__ __device__ inline uint32_t udiv_exact(uint32_t n, uint32_t d, double inv_d) {
    uint32_t q = (uint32_t)((double)n * inv_d);
    if (n - q * d >= d) ++q;
    return q;
}
// length(a) > length(b) (glm length = sqrtf(dot), func_geometric.inl:8-14) for
// a, b with squares x, y: sqrtf is monotone, so x <= y gives false, and
// x > y(1+2^-20) (y normal) separates the two correctly rounded roots by more
// than their rounding; only the rare near-ties (or NaN/tiny) take the roots.
__device__ __forceinline__ bool longer_sq(float x, float y) {
    const bool far_gt = x > y * 1.000001907f && y >= 1e-30f;  // 1 + 2^-19
    const bool le = x <= y;
    const bool tie = !far_gt && !le;
    bool r = far_gt;
    if (__builtin_expect(__any(tie), 0))
        if (tie) r = sqrt_(x) > sqrt_(y);
    return r;
}
__device__ __forceinline__ bool longer(vec3 a, vec3 b) { return longer_sq(dot(a, a), dot(b, b)); }

// A uniform value kept in a VGPR (the asm output counts as divergent), so
// that its uses read it directly instead of from an SGPR spilled to a VGPR
// lane (v_readlane + hazard nops per use).
__device__ __forceinline__ void vgpr_hold(float& f) { asm volatile("" : "+v"(f)); }
__device__ __forceinline__ void vgpr_hold(vec3& v) { vgpr_hold(v.x); vgpr_hold(v.y); vgpr_hold(v.z); }
__device__ __forceinline__ void vgpr_hold(int& i) { asm volatile("" : "+v"(i)); }

// The RotateDdf angle's (sin, cos) are functions of to.z alone: an exact
// table over every float with |to.z| in [2^-8, 1] (frame_table_kernel, 1 GiB),
// entry ((bits(|z|) - bits(2^-8)) << 1 | sign); other z (|z| < 2^-8, NaN) are
// computed. Replaces the f64 acos + sincos of most frame builds by one gather.
constexpr uint32_t kFrameTabLo = 0x3b800000u;    // 2^-8
constexpr uint32_t kFrameTabSpan = 0x04000000u;  // bits(1.0) - bits(2^-8)
constexpr size_t kFrameTabEntries = 2 * ((size_t)kFrameTabSpan + 1);
__device__ __forceinline__ void frame_sc_lookup(const float2* __restrict__ tab, vec3 to, float& s, float& c) {
    const uint32_t u = f2u(to.z), m = u & 0x7fffffffu;
    const bool in = m - kFrameTabLo <= kFrameTabSpan;
    if (in) {
        const float2 e = tab[((m - kFrameTabLo) << 1) | (u >> 31)];
        s = e.x;
        c = e.y;
    }
    if (__builtin_expect(__any(!in), 0))
        if (!in) frame_angle_sc(to, &s, &c);
}

__device__ __forceinline__ bool owned_row(const KParams& kp, int yi) {
    if (kp.n_shards <= 1 || kp.tile_rows <= 0) return true;
    return ((yi / kp.tile_rows) % kp.n_shards) == kp.shard_id;
}

// 8-word RNG window (blocks blk and blk+1 of the path's Philox stream) in
// named registers; draws are picked with selects (a runtime-indexed array
// would be placed in scratch).
struct Win8 {
    uint32_t a0, a1, a2, a3, b0, b1, b2, b3;
};

// w_j, w_(j+1), w_(j+2) for j in [0,4) (the prologue shifts the window as soon
// as k leaves block blk, and a step consumes at most 3 draws): three 4-way
// selects on j's two bits instead of three 6-way chains
__device__ __forceinline__ uint32_t sel4(uint32_t j, uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
    const bool b0 = (j & 1u) != 0u, b1 = (j & 2u) != 0u;
    const uint32_t lo = b0 ? x1 : x0, hi = b0 ? x3 : x2;
    return b1 ? hi : lo;
}

// ceil(c 2^24) clamped to [0, 2^24] (0 for c <= 0 or NaN): u01(w) < c <=>
// (w >> 8) < cdf_threshold24(c), both sides exact (host: word_threshold)
__device__ __forceinline__ uint32_t cdf_threshold24(float c) {
    const float x = c * 16777216.0f;
    return !(x > 0.0f) ? 0u : (x >= 16777216.0f ? 16777216u : (uint32_t)__builtin_ceilf(x));
}

__device__ __forceinline__ void philox_fill(uint32_t& d0, uint32_t& d1, uint32_t& d2, uint32_t& d3,
                                            uint32_t blk, uint32_t pass, uint32_t pix, uint32_t k0,
                                            uint32_t k1) {
    u32x4 o = philox4x32_10(blk, pass, pix, 0u, k0, k1);
    d0 = o.v[0];
    d1 = o.v[1];
    d2 = o.v[2];
    d3 = o.v[3];
}

// Conservative slab test (entry distance or +inf). Approximate reciprocals
// are fine here: only whether a subtree can contain the scan's winner is
// decided, with margins; the winner itself comes from the exact sphere_t().
__device__ __forceinline__ float bvh_box_entry(const BvhNode& b, vec3 o, vec3 inv) {
    const float tx0 = (b.bmin[0] - o.x) * inv.x, tx1 = (b.bmax[0] - o.x) * inv.x;
    const float ty0 = (b.bmin[1] - o.y) * inv.y, ty1 = (b.bmax[1] - o.y) * inv.y;
    const float tz0 = (b.bmin[2] - o.z) * inv.z, tz1 = (b.bmax[2] - o.z) * inv.z;
    const float tnear = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tfar = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    return tnear <= tfar * 1.0001f + 1e-5f ? tnear : inf_();
}
__device__ __forceinline__ float safe_rcp(float d) {
    return d == 0.0f ? (f2u(d) >> 31 ? -1e30f : 1e30f) : __builtin_amdgcn_rcpf(d);
}

// Stackless walk of the sphere BVH (ipt_bvh.h) from node i for at most
// `budget` node visits; i == kp.n_nodes when the walk is complete. best/bidx
// carry the nearest accepted hit (FractalSpheres.cpp:75-84's rule: minimal t,
// lowest original index on ties, never replacing an equal plane hit).
template <bool COUNT>
__device__ __forceinline__ void sphere_bvh_walk(const KParams& kp, vec3 o, vec3 d, int& i, float& best, int& bidx,
                                                int budget, uint32_t& c_nodes, uint32_t& c_tests) {
    const vec3 inv = v3(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
    // near-child-first linearisation for this direction octant (ipt_bvh.h)
    const int oct = (int)(f2u(d.x) >> 31) | (int)(f2u(d.y) >> 31) << 1 | (int)(f2u(d.z) >> 31) << 2;
    const BvhNode* __restrict__ nodes = kp.bvh_nodes + (size_t)oct * kp.n_nodes;
    // while-while (Aila & Laine 2009): the inner loop only walks nodes until
    // each lane stands on an entered leaf (or is done), so the leaf's sphere
    // tests run with all such lanes together instead of once per wave-iteration
    while (i < kp.n_nodes && budget > 0) {
        int leaf = -1;
        while (i < kp.n_nodes && budget > 0) {
            --budget;
            const BvhNode nd = nodes[i];
            if (COUNT) ++c_nodes;
            const float te = bvh_box_entry(nd, o, inv);
            // te == inf is a miss; it must not pass when best is inf too (open floor)
            const bool enter = te != inf_() && te <= best * 1.0001f + 1e-5f + kp.bvh_tmargin;
            if (enter && nd.leaf >= 0) {
                leaf = nd.leaf;
                i = nd.skip;
                break;
            }
            i = enter ? i + 1 : nd.skip;
        }
        if (leaf >= 0) {
            const int first = leaf & 0xffffff, cnt = leaf >> 24;
            if (COUNT) c_tests += (uint32_t)cnt;
            for (int k2 = 0; k2 < cnt; ++k2) {
                const BvhSphere sp = kp.bvh_prims[first + k2];
                const float t = sphere_t(sp.r, o - v3(sp.c[0], sp.c[1], sp.c[2]), d);
                if (isfinite_(t) && gt_1em6(fabs_(t)) &&
                    (t < best || (t == best && bidx >= 0 && sp.index < bidx))) {
                    best = t;
                    bidx = sp.index;
                }
            }
        }
    }
}

// Uniform-grid walk (ipt_bvh.h SphereGrid; exactness argument there). The
// resumable state is the current cell (x | y << 8 | z << 16, -1 when done) and
// the t of the next cell boundary per axis.
__device__ __forceinline__ void sphere_grid_init(const KParams& kp, vec3 o, vec3 d, int& cell, vec3& tmx) {
    const vec3 inv = v3(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
    const float dv[3] = {d.x, d.y, d.z}, ov[3] = {o.x, o.y, o.z}, iv[3] = {inv.x, inv.y, inv.z};
    float tn = 0.0f, tf = inf_();
    for (int a = 0; a < 3; ++a) {
        const float g1 = kp.grid_g1[a];  // g0 + (float)n * h
        if (dv[a] == 0.0f) {
            if (ov[a] < kp.grid_g0[a] || ov[a] > g1) tf = -1.0f;  // parallel and outside
            continue;
        }
        const float t0 = (kp.grid_g0[a] - ov[a]) * iv[a], t1 = (g1 - ov[a]) * iv[a];
        tn = fmaxf(tn, fminf(t0, t1));
        tf = fminf(tf, fmaxf(t0, t1));
    }
    if (!(tn <= tf * 1.0001f + 1e-5f)) {
        cell = -1;
        return;
    }
    int ia[3];
    float tm[3];
    for (int a = 0; a < 3; ++a) {
        const float pa = ov[a] + dv[a] * tn;
        int c = (int)floorf((pa - kp.grid_g0[a]) * kp.grid_inv_h[a]);
        c = c < 0 ? 0 : (c >= kp.grid_n[a] ? kp.grid_n[a] - 1 : c);
        ia[a] = c;
        tm[a] = dv[a] > 0.0f   ? ((kp.grid_g0[a] + (float)(c + 1) * kp.grid_h[a]) - ov[a]) * iv[a]
                : dv[a] < 0.0f ? ((kp.grid_g0[a] + (float)c * kp.grid_h[a]) - ov[a]) * iv[a]
                               : inf_();
    }
    cell = ia[0] | ia[1] << 8 | ia[2] << 16;
    tmx = v3(tm[0], tm[1], tm[2]);
}
__device__ __forceinline__ float4 grid_item(const KParams& kp, int k) {
    if constexpr (IPT_GRID_C4) return kp.grid_c4[k];
    return *reinterpret_cast<const float4*>(kp.grid_items[k].c);
}
__device__ __forceinline__ int grid_item_index(const KParams& kp, int k) {
    if constexpr (IPT_GRID_C4) return kp.grid_idx[k];
    return kp.grid_items[k].index;
}
// POS (the pipelined walk of the resumable instances, IPT_GRID_PIPE): bidx is
// the best item's position in grid_items instead of its original index, so an
// item is one 16-byte load and its index is read only on a tie (the caller
// converts when the walk is done); IPT_GRID_ITEMS item loads are issued before
// their tests, and the next cell's item range is fetched with them.
template <bool COUNT, bool POS = false>
__device__ __forceinline__ void sphere_grid_walk(const KParams& kp, vec3 o, vec3 d, int& cell, vec3& tmx, float& best,
                                                 int& bidx, int budget, uint32_t& c_nodes,
                                                 uint32_t& c_tests IPT_DIAG_PARAMS) {
    const vec3 inv = v3(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
    auto accept = [&](float t, int k2) {  // FractalSpheres.cpp:75-84's rule on item positions
        if (isfinite_(t) && gt_1em6(fabs_(t))) {
            if (t < best)
                bidx = k2;
            else if (t == best && bidx >= 0 && kp.grid_items[k2].index < kp.grid_items[bidx].index)
                bidx = k2;
            best = t < best ? t : best;
        }
    };
    if constexpr (POS && IPT_GRID_INLINE) {
        // cells as 64-byte records (GridCell: the item range and the first
        // three items): the next cell follows from tmx alone, so its record is
        // fetched while the current cell's items are tested -- one round trip
        // per cell, overlapped, instead of a range load and then item loads.
        // Same cells, items, tests and exit decisions as the walk below.
        if (cell < 0 || budget <= 0) return;
        auto lin_of = [&](int c) {
            return (c & 0xff) + kp.grid_n[0] * (((c >> 8) & 0xff) + kp.grid_n[1] * (c >> 16));
        };
        auto load = [&](int l, int& a, int& b, float4* it) {
            const uint4* r = reinterpret_cast<const uint4*>(kp.grid_cells + l);
            const uint4 h = r[0];
            it[0] = __builtin_bit_cast(float4, r[1]);
            it[1] = __builtin_bit_cast(float4, r[2]);
            it[2] = __builtin_bit_cast(float4, r[3]);
            a = (int)h.x;
            b = (int)h.y;
        };
        int lin = lin_of(cell);
        int s0, s1;
        float4 it[3];
        load(lin, s0, s1, it);
        for (;;) {
            const int ix = cell & 0xff, iy = (cell >> 8) & 0xff, iz = cell >> 16;
            int ncell;
            vec3 ntm = tmx;
            bool nvalid;
            if (tmx.x <= tmx.y && tmx.x <= tmx.z) {
                const int nx = d.x > 0.0f ? ix + 1 : ix - 1;
                nvalid = !(nx < 0 || nx >= kp.grid_n[0]);
                ncell = (cell & ~0xff) | (nx & 0xff);
                ntm.x = ((kp.grid_g0[0] + (float)(d.x > 0.0f ? nx + 1 : nx) * kp.grid_h[0]) - o.x) * inv.x;
            } else if (tmx.y <= tmx.z) {
                const int ny = d.y > 0.0f ? iy + 1 : iy - 1;
                nvalid = !(ny < 0 || ny >= kp.grid_n[1]);
                ncell = (cell & ~0xff00) | (ny & 0xff) << 8;
                ntm.y = ((kp.grid_g0[1] + (float)(d.y > 0.0f ? ny + 1 : ny) * kp.grid_h[1]) - o.y) * inv.y;
            } else {
                const int nz = d.z > 0.0f ? iz + 1 : iz - 1;
                nvalid = !(nz < 0 || nz >= kp.grid_n[2]);
                ncell = (cell & 0xffff) | (nz & 0xff) << 16;
                ntm.z = ((kp.grid_g0[2] + (float)(d.z > 0.0f ? nz + 1 : nz) * kp.grid_h[2]) - o.z) * inv.z;
            }
            // the next record, unconditionally (this cell's again when there is none)
            const int nlin = nvalid ? lin_of(ncell) : lin;
            int n0, n1;
            float4 nit[3];
            load(nlin, n0, n1, nit);
            if (COUNT) {
                ++c_nodes;
                c_tests += (uint32_t)(s1 - s0);
            }
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (s0 + q < s1) accept(sphere_t(it[q].w, o - v3(it[q].x, it[q].y, it[q].z), d), s0 + q);
            // items beyond the record (IPT_GRID_ITEMS loads in flight)
            constexpr int X = IPT_GRID_ITEMS;
            for (int k2 = s0 + 3; k2 < s1; k2 += X) {
                float4 c4[X];
#pragma unroll
                for (int q = 0; q < X; ++q)
                    c4[q] = *reinterpret_cast<const float4*>(kp.grid_items[k2 + q < s1 ? k2 + q : k2].c);
#pragma unroll
                for (int q = 0; q < X; ++q)
                    if (k2 + q < s1) accept(sphere_t(c4[q].w, o - v3(c4[q].x, c4[q].y, c4[q].z), d), k2 + q);
            }
            --budget;
            const float texit = fminf(fminf(tmx.x, tmx.y), tmx.z);
            if (texit > (best * 1.0001f + 1e-5f + kp.bvh_tmargin + kp.grid_m) * 1.00001f + 1e-5f || !nvalid) {
                cell = -1;
                return;
            }
            cell = ncell;
            tmx = ntm;
            if (budget <= 0) return;
            lin = nlin;
            s0 = n0;
            s1 = n1;
#pragma unroll
            for (int q = 0; q < 3; ++q) it[q] = nit[q];
        }
    } else if constexpr (POS) {
        // the next cell (it depends on tmx alone) and its item range are
        // fetched before the current cell's items are tested, so the range
        // load overlaps the item loads; the exit test (on best) then decides
        // whether the walk moves there. Same cells, items and tests.
        if (cell < 0 || budget <= 0) return;
        auto lin_of = [&](int c) {
            return (c & 0xff) + kp.grid_n[0] * (((c >> 8) & 0xff) + kp.grid_n[1] * (c >> 16));
        };
        int lin = lin_of(cell);
        int s0 = kp.grid_start[lin], s1 = kp.grid_start[lin + 1];
        for (;;) {
#if IPT_PROF
            if (prof_w) { IPT_PHASE(6); }  // one cell of the pipelined walk
#endif
            const int ix = cell & 0xff, iy = (cell >> 8) & 0xff, iz = cell >> 16;
            int ncell;
            vec3 ntm = tmx;
            bool nvalid;
            if (tmx.x <= tmx.y && tmx.x <= tmx.z) {
                const int nx = d.x > 0.0f ? ix + 1 : ix - 1;
                nvalid = !(nx < 0 || nx >= kp.grid_n[0]);
                ncell = (cell & ~0xff) | (nx & 0xff);
                ntm.x = ((kp.grid_g0[0] + (float)(d.x > 0.0f ? nx + 1 : nx) * kp.grid_h[0]) - o.x) * inv.x;
            } else if (tmx.y <= tmx.z) {
                const int ny = d.y > 0.0f ? iy + 1 : iy - 1;
                nvalid = !(ny < 0 || ny >= kp.grid_n[1]);
                ncell = (cell & ~0xff00) | (ny & 0xff) << 8;
                ntm.y = ((kp.grid_g0[1] + (float)(d.y > 0.0f ? ny + 1 : ny) * kp.grid_h[1]) - o.y) * inv.y;
            } else {
                const int nz = d.z > 0.0f ? iz + 1 : iz - 1;
                nvalid = !(nz < 0 || nz >= kp.grid_n[2]);
                ncell = (cell & 0xffff) | (nz & 0xff) << 16;
                ntm.z = ((kp.grid_g0[2] + (float)(d.z > 0.0f ? nz + 1 : nz) * kp.grid_h[2]) - o.z) * inv.z;
            }
            // unconditional load (the current cell's range when there is no next)
            const int nlin = nvalid ? lin_of(ncell) : lin;
            const int n0 = kp.grid_start[nlin], n1 = kp.grid_start[nlin + 1];
            if (COUNT) {
                ++c_nodes;
                c_tests += (uint32_t)(s1 - s0);
            }
            auto test = [&](float4 c4, int k2) {
                const float t = sphere_t(c4.w, o - v3(c4.x, c4.y, c4.z), d);
                if (isfinite_(t) && gt_1em6(fabs_(t))) {
                    if (t < best)
                        bidx = k2;
                    else if (t == best && bidx >= 0 && grid_item_index(kp, k2) < grid_item_index(kp, bidx))
                        bidx = k2;
                    best = t < best ? t : best;
                }
            };
            constexpr int X = IPT_GRID_ITEMS;
                for (int k2 = s0; k2 < s1; k2 += X) {
                    float4 c4[X];
#pragma unroll
                    for (int q = 0; q < X; ++q)
                        c4[q] = grid_item(kp, k2 + q < s1 ? k2 + q : k2);
                    test(c4[0], k2);
#pragma unroll
                    for (int q = 1; q < X; ++q)
                        if (k2 + q < s1) test(c4[q], k2 + q);
                }
            --budget;
            const float texit = fminf(fminf(tmx.x, tmx.y), tmx.z);
            if (texit > (best * 1.0001f + 1e-5f + kp.bvh_tmargin + kp.grid_m) * 1.00001f + 1e-5f || !nvalid) {
                cell = -1;
                return;
            }
            cell = ncell;
            tmx = ntm;
            if (budget <= 0) return;
            lin = nlin;
            s0 = n0;
            s1 = n1;
        }
    }
    while (cell >= 0 && budget-- > 0) {
        const int ix = cell & 0xff, iy = (cell >> 8) & 0xff, iz = cell >> 16;
        const int lin = ix + kp.grid_n[0] * (iy + kp.grid_n[1] * iz);
        const int s0 = kp.grid_start[lin], s1 = kp.grid_start[lin + 1];
        if (COUNT) {
            ++c_nodes;
            c_tests += (uint32_t)(s1 - s0);
        }
        for (int k2 = s0; k2 < s1; ++k2) {
            const BvhSphere sp = kp.grid_items[k2];
            const float t = sphere_t(sp.r, o - v3(sp.c[0], sp.c[1], sp.c[2]), d);
            if (isfinite_(t) && gt_1em6(fabs_(t)) && (t < best || (t == best && bidx >= 0 && sp.index < bidx))) {
                best = t;
                bidx = sp.index;
            }
        }
        const float texit = fminf(fminf(tmx.x, tmx.y), tmx.z);
        if (texit > (best * 1.0001f + 1e-5f + kp.bvh_tmargin + kp.grid_m) * 1.00001f + 1e-5f) {
            cell = -1;
            break;
        }
        // step across the nearest boundary (x, then y, then z on ties)
        if (tmx.x <= tmx.y && tmx.x <= tmx.z) {
            const int nx = d.x > 0.0f ? ix + 1 : ix - 1;
            if (nx < 0 || nx >= kp.grid_n[0]) { cell = -1; break; }
            cell = (cell & ~0xff) | nx;
            tmx.x = ((kp.grid_g0[0] + (float)(d.x > 0.0f ? nx + 1 : nx) * kp.grid_h[0]) - o.x) * inv.x;
        } else if (tmx.y <= tmx.z) {
            const int ny = d.y > 0.0f ? iy + 1 : iy - 1;
            if (ny < 0 || ny >= kp.grid_n[1]) { cell = -1; break; }
            cell = (cell & ~0xff00) | ny << 8;
            tmx.y = ((kp.grid_g0[1] + (float)(d.y > 0.0f ? ny + 1 : ny) * kp.grid_h[1]) - o.y) * inv.y;
        } else {
            const int nz = d.z > 0.0f ? iz + 1 : iz - 1;
            if (nz < 0 || nz >= kp.grid_n[2]) { cell = -1; break; }
            cell = (cell & 0xffff) | nz << 16;
            tmx.z = ((kp.grid_g0[2] + (float)(d.z > 0.0f ? nz + 1 : nz) * kp.grid_h[2]) - o.z) * inv.z;
        }
    }
}

// Wave-wide inclusive scans over the 64 lanes (DPP: row shifts within each
// 16-lane row, then rows 1/3 from lane 15 of the row before and rows 2/3 from
// lane 31). Called with every lane of the wave active.
__device__ __forceinline__ int wave_scan_add(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}
__device__ __forceinline__ int wave_scan_max(int v) {  // v >= 0
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));
    return v;
}

// Orders one wave's LDS accesses across its lanes for the compiler (the
// hardware runs a wave's LDS instructions in order): without it a lane's load
// of a word it stored itself would be forwarded from that store, missing the
// other lanes' stores in between.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The resumable grid walk with the item tests spread over the whole wave
// (IPT_GRID_WAVE). Per wave iteration every walking lane steps one cell: the
// (lane, item) pairs of the cells the lanes stand on are numbered by a wave
// prefix sum and tested 64 at a time, one pair per lane (the lane that owns
// pair p is found by a ds_permute of the segment starts and a max-scan; its
// ray is read with ds_bpermute), and each accepted t goes to its owner's
// LDS slot as an atomic minimum of (t bits << 32 | item position). Within a
// cell the positions are in original-index order (grid_build_spheres fills
// each cell in index order) and accepted t are positive, so the slot ends as
// the cell's (t, index) minimum; the owner merges it with `accept`, the
// per-lane walk's rule (FractalSpheres.cpp:75-84: strict '<', lowest index on
// equal t, a plane never loses a tie). The tests run at full lane
// utilisation instead of once per lane per item slot. Same cells, same tests
// (sphere_t on the same operands), same exit decisions: the (t, index) minimum
// does not depend on the order of the tests. Every lane of the wave calls it.
// grid_start[lin] from global memory, or (IPT_GRID_LDS) from the packed copy
// staged in LDS (gl): an 8-entry block's base plus the entry's byte offset
__device__ __forceinline__ int grid_start_at(const KParams& kp, const int* gl, int lin) {
    if constexpr (IPT_GRID_LDS != 0) {
        const uint8_t* off = reinterpret_cast<const uint8_t*>(gl + kp.grid_packed_nb);
        return gl[lin >> 3] + (int)off[lin];
    }
    return kp.grid_start[lin];
}

template <bool COUNT>
__device__ __forceinline__ void sphere_grid_walk_wave(const KParams& kp, bool walking, vec3 o, vec3 d, int& cell,
                                                      vec3& tmx, float& best, int& bidx, int budget,
                                                      unsigned long long* slots, int lane, const int* gl,
                                                      uint32_t& c_nodes, uint32_t& c_tests IPT_DIAG_PARAMS) {
    const vec3 inv = v3(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
    auto lin_of = [&](int c) {
        return (c & 0xff) + kp.grid_n[0] * (((c >> 8) & 0xff) + kp.grid_n[1] * (c >> 16));
    };
    bool act = walking && cell >= 0 && budget > 0;
    int s0 = 0, s1 = 0;
    if (act) {
        const int lin = lin_of(cell);
        s0 = grid_start_at(kp, gl, lin);
        s1 = grid_start_at(kp, gl, lin + 1);
    }
    for (int it = 0;; ++it) {
        // (after IPT_GRID_WAVE_FLOOR_IT iterations the wave stops once fewer than
        // IPT_GRID_WAVE_FLOOR lanes walk; they resume in the next step)
        const uint64_t am = __ballot(act);
        if (!am || (it >= IPT_GRID_WAVE_FLOOR_IT && __popcll(am) < IPT_GRID_WAVE_FLOOR)) break;
#if IPT_PROF
        // phase 6 (walk cell): one wave iteration, its walking lanes (every
        // lane of the wave runs this loop, so lane 0 counts)
        if (prof_w && lane == 0) {
            prof_w[6] += 1u;
            prof_l[6] += (uint32_t)__popcll(am);
        }
#endif
        // the next cell (from tmx alone) and its range, in flight during the tests
        int ncell = 0, n0 = 0, n1 = 0;
        vec3 ntm = tmx;
        bool nvalid = false;
        if (act) {
            const int ix = cell & 0xff, iy = (cell >> 8) & 0xff, iz = cell >> 16;
            if (tmx.x <= tmx.y && tmx.x <= tmx.z) {
                const int nx = d.x > 0.0f ? ix + 1 : ix - 1;
                nvalid = !(nx < 0 || nx >= kp.grid_n[0]);
                ncell = (cell & ~0xff) | (nx & 0xff);
                ntm.x = ((kp.grid_g0[0] + (float)(d.x > 0.0f ? nx + 1 : nx) * kp.grid_h[0]) - o.x) * inv.x;
            } else if (tmx.y <= tmx.z) {
                const int ny = d.y > 0.0f ? iy + 1 : iy - 1;
                nvalid = !(ny < 0 || ny >= kp.grid_n[1]);
                ncell = (cell & ~0xff00) | (ny & 0xff) << 8;
                ntm.y = ((kp.grid_g0[1] + (float)(d.y > 0.0f ? ny + 1 : ny) * kp.grid_h[1]) - o.y) * inv.y;
            } else {
                const int nz = d.z > 0.0f ? iz + 1 : iz - 1;
                nvalid = !(nz < 0 || nz >= kp.grid_n[2]);
                ncell = (cell & 0xffff) | (nz & 0xff) << 16;
                ntm.z = ((kp.grid_g0[2] + (float)(d.z > 0.0f ? nz + 1 : nz) * kp.grid_h[2]) - o.z) * inv.z;
            }
            ncell = nvalid ? ncell : -1;
            // (no next cell: cell 0's range, unused)
            const int nlin = nvalid ? lin_of(ncell) : 0;
            n0 = grid_start_at(kp, gl, nlin);
            n1 = grid_start_at(kp, gl, nlin + 1);
        }
        const int cnt = act ? s1 - s0 : 0;
        if (COUNT && act) {
            ++c_nodes;
            c_tests += (uint32_t)cnt;
        }
        const int incl = wave_scan_add(cnt);
        const int total = __builtin_amdgcn_readlane(incl, 63);
        const int excl = incl - cnt;
        if (total > 0) {
            if (cnt > 0) slots[lane] = ~0ull;
            wave_lds_sync();  // the clears before any lane's atomic minimum
            const int dk = s0 - excl;  // pair p of this lane tests item p + dk
            // one round: pairs base .. base + 63 (owner, its ray, the item)
            struct Pair {
                vec3 o, d;
                float4 c4;
                int k, src;
                bool valid;
            };
            auto setup = [&](int base, Pair& q) {
                // the owner of pair base + lane, in one ds_permute (no LDS
                // round trip): every lane whose segment starts before the
                // round's end sends lane + 1 to its start (clamped to 0); of
                // lanes sharing a start only the highest-numbered can own
                // pairs (excl[L] == excl[L+1] means cnt[L] == 0), and the
                // highest-numbered source is the one ds_permute keeps. The
                // lanes starting beyond the round (a suffix: excl does not
                // decrease) send to position 63, which then takes the last
                // sender; a max-scan carries each start to the pairs after it.
                const bool snd = excl < base + 64;
                int r = __builtin_amdgcn_ds_permute((snd ? (excl > base ? excl - base : 0) : 63) << 2, lane + 1);
                const uint64_t sm = __ballot(snd);
                if (~sm && lane == 63) r = __popcll(sm);
                q.src = wave_scan_max(r) - 1;
                const int p = base + lane;
                q.valid = p < total;
                const int sl = q.valid ? q.src : lane;
                q.o = v3(__shfl(o.x, sl), __shfl(o.y, sl), __shfl(o.z, sl));
                q.d = v3(__shfl(d.x, sl), __shfl(d.y, sl), __shfl(d.z, sl));
                q.k = p + __shfl(dk, sl);
                if (IPT_GRID_WAVE_UNC)
                    q.c4 = grid_item(kp, q.valid ? q.k : 0);
                else if (q.valid)
                    q.c4 = grid_item(kp, q.k);
            };
            auto test = [&](const Pair& q) {
                // IPT_GRID_WAVE_UNC: every lane loads (item 0 for lanes without a
                // pair) and the wave waits for the item here, outside the branch:
                // otherwise a load left pending on the path that skips the test
                // made the next round's load wait for every outstanding load,
                // the next cell's range prefetch included (vmcnt(0))
                if (IPT_GRID_WAVE_UNC) keep_alive(q.c4);
                if (q.valid) {
                    const float t = sphere_t(q.c4.w, q.o - v3(q.c4.x, q.c4.y, q.c4.z), q.d);
                    if (isfinite_(t) && gt_1em6(fabs_(t)))
                        __hip_atomic_fetch_min(slots + q.src,
                                               (unsigned long long)__float_as_uint(t) << 32 | (uint32_t)q.k,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                }
            };
            int base = 0;
            if constexpr (IPT_GRID_WAVE_PIPE) {
                // the first two rounds' items fetched together
                Pair q0, q1;
                setup(0, q0);
                const bool two = total > 64;
                if (two) setup(64, q1);
                test(q0);
                if (two) test(q1);
                base = 128;
            }
            for (; base < total; base += 64) {
                Pair q;
                setup(base, q);
                test(q);
            }
            wave_lds_sync();
            if (cnt > 0) {
                const unsigned long long key = slots[lane];
                if (key != ~0ull) {
                    const float t = __uint_as_float((uint32_t)(key >> 32));
                    const int k2 = (int)(uint32_t)key;
                    if (t < best)
                        bidx = k2;
                    else if (t == best && bidx >= 0 && grid_item_index(kp, k2) < grid_item_index(kp, bidx))
                        bidx = k2;
                    best = t < best ? t : best;
                }
            }
        }
        if (act) {
            --budget;
            const float texit = fminf(fminf(tmx.x, tmx.y), tmx.z);
            if (texit > (best * 1.0001f + 1e-5f + kp.bvh_tmargin + kp.grid_m) * 1.00001f + 1e-5f || ncell < 0) {
                cell = -1;
                act = false;
            } else {
                cell = ncell;
                tmx = ntm;
                s0 = n0;
                s1 = n1;
                act = budget > 0;
            }
        }
    }
}

// IPT_GRID_WAVE == 2: the same with two cells per lane per wave iteration --
// the cell the lane stands on (A) and the next one (B), whose range was
// fetched in the previous iteration; the two cells after them are located and
// their ranges fetched while A's and B's items are tested -- and the slots
// keyed by (t bits << 32 | original index) (the index is loaded with the
// item), so bidx holds the original index and the minimum over two cells'
// items is the scan's (t, index) rule directly. Exit tests after A and after
// B as in the per-cell walk; B's items are tested even when the walk ends
// after A, which is harmless (any sphere's t is a valid candidate of the
// scan, and the exit bound only shrinks with best). Two cells of budget per
// iteration.
template <bool COUNT>
__device__ __forceinline__ void sphere_grid_walk_wave2(const KParams& kp, bool walking, vec3 o, vec3 d, int& cell,
                                                       vec3& tmx, float& best, int& bidx, int budget,
                                                       unsigned long long* slots, uint8_t* own, int lane,
                                                       uint32_t& c_nodes, uint32_t& c_tests) {
    const vec3 inv = v3(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z));
    auto lin_of = [&](int c) {
        return (c & 0xff) + kp.grid_n[0] * (((c >> 8) & 0xff) + kp.grid_n[1] * (c >> 16));
    };
    // one DDA step from cell c with boundary t's tm (ties: x, then y, then z)
    auto step = [&](int c, vec3 tm, int& nc, vec3& ntm, bool& nv) {
        const int ix = c & 0xff, iy = (c >> 8) & 0xff, iz = c >> 16;
        ntm = tm;
        if (tm.x <= tm.y && tm.x <= tm.z) {
            const int nx = d.x > 0.0f ? ix + 1 : ix - 1;
            nv = !(nx < 0 || nx >= kp.grid_n[0]);
            nc = (c & ~0xff) | (nx & 0xff);
            ntm.x = ((kp.grid_g0[0] + (float)(d.x > 0.0f ? nx + 1 : nx) * kp.grid_h[0]) - o.x) * inv.x;
        } else if (tm.y <= tm.z) {
            const int ny = d.y > 0.0f ? iy + 1 : iy - 1;
            nv = !(ny < 0 || ny >= kp.grid_n[1]);
            nc = (c & ~0xff00) | (ny & 0xff) << 8;
            ntm.y = ((kp.grid_g0[1] + (float)(d.y > 0.0f ? ny + 1 : ny) * kp.grid_h[1]) - o.y) * inv.y;
        } else {
            const int nz = d.z > 0.0f ? iz + 1 : iz - 1;
            nv = !(nz < 0 || nz >= kp.grid_n[2]);
            nc = (c & 0xffff) | (nz & 0xff) << 16;
            ntm.z = ((kp.grid_g0[2] + (float)(d.z > 0.0f ? nz + 1 : nz) * kp.grid_h[2]) - o.z) * inv.z;
        }
    };
    bool act = walking && cell >= 0 && budget > 0;
    int s0 = 0, s1 = 0, cb = 0, a0 = 0, a1 = 0;
    vec3 tmb = tmx;
    bool bval = false;
    if (act) {
        const int l = lin_of(cell);
        s0 = kp.grid_start[l];
        s1 = kp.grid_start[l + 1];
        step(cell, tmx, cb, tmb, bval);
        if (bval) {
            const int lb = lin_of(cb);
            a0 = kp.grid_start[lb];
            a1 = kp.grid_start[lb + 1];
        }
    }
    while (__ballot(act)) {
        // cells C and D after A, B and their ranges, in flight during the tests
        int cc = 0, cd = 0, c0 = 0, c1 = 0, d0 = 0, d1 = 0;
        vec3 tmc = tmb, tmd = tmb;
        bool cval = false, dval = false;
        if (act && bval) {
            step(cb, tmb, cc, tmc, cval);
            if (cval) {
                const int lc = lin_of(cc);
                c0 = kp.grid_start[lc];
                c1 = kp.grid_start[lc + 1];
                step(cc, tmc, cd, tmd, dval);
                if (dval) {
                    const int ld = lin_of(cd);
                    d0 = kp.grid_start[ld];
                    d1 = kp.grid_start[ld + 1];
                }
            }
        }
        const int cnta = act ? s1 - s0 : 0;
        const int cnt = cnta + ((act && bval) ? a1 - a0 : 0);
        if (COUNT && act) {
            c_nodes += bval ? 2u : 1u;
            c_tests += (uint32_t)cnt;
        }
        const int incl = wave_scan_add(cnt);
        const int total = __builtin_amdgcn_readlane(incl, 63);
        const int excl = incl - cnt;
        if (total > 0) {
            if (cnt > 0) slots[lane] = ~0ull;
            // pair p of this lane: item p + da (p < ea, cell A) or p + db (cell B)
            const int ea = excl + cnta, da = s0 - excl, db = a0 - ea;
            for (int base = 0; base < total; base += 64) {
                own[lane] = 0;
                if (cnt > 0 && excl < base + 64 && incl > base) own[excl > base ? excl - base : 0] = (uint8_t)(lane + 1);
                wave_lds_sync();
                const int src = wave_scan_max((int)own[lane]) - 1;
                const int p = base + lane;
                const bool valid = p < total;
                const int sl = valid ? src : lane;
                const float ox = __shfl(o.x, sl), oy = __shfl(o.y, sl), oz = __shfl(o.z, sl);
                const float dx = __shfl(d.x, sl), dy = __shfl(d.y, sl), dz = __shfl(d.z, sl);
                const int eao = __shfl(ea, sl), dao = __shfl(da, sl), dbo = __shfl(db, sl);
                if (valid) {
                    const int k = p < eao ? p + dao : p + dbo;
                    const float4 c4 = kp.grid_c4[k];
                    const int idx = kp.grid_idx[k];
                    const float t = sphere_t(c4.w, v3(ox, oy, oz) - v3(c4.x, c4.y, c4.z), v3(dx, dy, dz));
                    if (isfinite_(t) && gt_1em6(fabs_(t)))
                        __hip_atomic_fetch_min(slots + src,
                                               (unsigned long long)__float_as_uint(t) << 32 | (uint32_t)idx,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                }
            }
            wave_lds_sync();
            if (cnt > 0) {
                const unsigned long long key = slots[lane];
                if (key != ~0ull) {
                    const float t = __uint_as_float((uint32_t)(key >> 32));
                    const int idx = (int)(uint32_t)key;
                    if (t < best || (t == best && bidx >= 0 && idx < bidx)) bidx = idx;
                    best = t < best ? t : best;
                }
            }
        }
        if (act) {
            budget -= 2;
            const float bound = (best * 1.0001f + 1e-5f + kp.bvh_tmargin + kp.grid_m) * 1.00001f + 1e-5f;
            if (fminf(fminf(tmx.x, tmx.y), tmx.z) > bound || !bval || fminf(fminf(tmb.x, tmb.y), tmb.z) > bound ||
                !cval) {
                cell = -1;
                act = false;
            } else {
                cell = cc;
                tmx = tmc;
                s0 = c0;
                s1 = c1;
                cb = cd;
                tmb = tmd;
                bval = dval;
                a0 = d0;
                a1 = d1;
                act = budget > 0;
            }
        }
    }
}

// Nearest geometry hit for both geometry kinds. prim: 0..4 plane, 5 the
// r=0.5 sphere, 6+i extra sphere i (original index), -1 miss.
template <bool COUNT, int GEOM>
__device__ __forceinline__ float trace_geometry(const KParams& kp, vec3 o, vec3 d, int* prim, uint32_t& c_nodes,
                                                uint32_t& c_tests) {
    // kp.box_inrange: every ray origin (camera, wall/floor hits, listed spheres)
    // lies within 2^39, so the planes' divisions take the range-free sequence
    if (GEOM == IPT_GEOM_SPHERE_IN_BOX)
        return (IPT_BOXDIV && kp.box_inrange) ? trace_box<true>(o, d, prim) : trace_box<false>(o, d, prim);
    if (GEOM == IPT_GEOM_FLOOR) {  // GeometryFloor.cpp:11-13
        const float t = box_plane_t(o.z, d.z, -1.0f, o, d);
        *prim = t == inf_() ? -1 : 0;
        return t;
    }
    if (GEOM == IPT_GEOM_CORNER) {  // GeometryCorner.cpp:11-28: tx, then ty, tz with strict <
        float t = box_plane_t(o.x, d.x, -1.0f, o, d);
        int p = 0;
        const float ty = box_plane_t(o.y, d.y, -1.0f, o, d);
        if (ty < t) { t = ty; p = 1; }
        const float tz = box_plane_t(o.z, d.z, -1.0f, o, d);
        if (tz < t) { t = tz; p = 2; }
        *prim = t == inf_() ? -1 : p;
        return t;
    }
    if (GEOM == IPT_GEOM_SMALLPT) {  // GeometrySmallPt.cpp:14-47, double precision
        double min_t = (double)inf_();
        int mi = -1;
        for (int i = 0; i < kp.n_spheres; ++i) {
            const float4 sp = kp.spheres[i];
            const vec3 op = v3(sp.x, sp.y, sp.z) - o;  // p - ro (float)
            const double rad = (double)sp.w;
            const double b = (double)dot(op, d);
            double det = b * b - (double)dot(op, op) + rad * rad;
            double t = 0.0;
            if (!(det < 0.0)) {
                det = sqrtd_(det);
                t = b - det;
                if (!(t > 1e-4)) {
                    t = b + det;
                    if (!(t > 1e-4)) t = 0.0;
                }
            }
            if (COUNT) ++c_tests;
            if (t != 0.0 && t < min_t) {
                min_t = t;
                mi = i;
            }
        }
        *prim = mi >= 0 ? 6 + mi : -1;
        return mi >= 0 ? (float)min_t : inf_();
    }
    // planes as GeometrySphereInBox, then spheres with FractalSpheres' rule
    // (FractalSpheres.cpp:75-84): strict '<' in index order == minimal t,
    // lowest index among equal t, and a sphere never wins a tie with a plane.
    int p = -1;
    float best = inf_();  // FractalSpheres: no walls
    if (GEOM == IPT_GEOM_SPHERES_IN_BOX)
        best = (IPT_BOXDIV && kp.box_inrange) ? trace_box_planes_only<true>(o, d, &p) : trace_box_planes_only<false>(o, d, &p);
    int bidx = -1;
    if (kp.n_grid > 0) {
        int cell;
        vec3 tmx;
        sphere_grid_init(kp, o, d, cell, tmx);
        sphere_grid_walk<COUNT>(kp, o, d, cell, tmx, best, bidx, 0x7fffffff, c_nodes, c_tests IPT_DIAG_NULL_ARGS);
    } else if (kp.n_nodes > 0) {
        int i = 0;
        sphere_bvh_walk<COUNT>(kp, o, d, i, best, bidx, 0x7fffffff, c_nodes, c_tests);
    } else {
        if (COUNT) c_tests += (uint32_t)kp.n_spheres;
        for (int i = 0; i < kp.n_spheres; ++i) {
            float4 s = kp.spheres[i];
            vec3 c = v3(s.x, s.y, s.z);
            float t = sphere_t(s.w, o - c, d);
            if (isfinite_(t) && gt_1em6(fabs_(t)) && t < best) {
                best = t;
                bidx = i;
            }
        }
    }
    *prim = bidx >= 0 ? 6 + bidx : p;
    return best;
}

// Scene data staged once per workgroup (never re-read from HBM/L2 inside the
// step loop): wall frames, lights (<= kLdsLights), mixture weights + CDF and
// the candidate-row table live in LDS after the DFS stack.
constexpr int kLdsLights = 16;
constexpr int kLightWords = (int)(sizeof(LightDev) / 4);
// LDS after the DFS stack: frames, [LMODE 2: lights, weights, cdf],
// [sharded: candidate rows], [LMODE 3: weights, cdf, light BVH].
// Frames live in LDS, [12][kFrameStride]: column tid is the lane's current
// sphere-node frame, columns kBlock..kBlock+4 the five wall frames.
// CosineDdf samples come from exact tables (cos_table_kernel).
// Column stride: single-light instances use kBlock + 64 words (a multiple of
// 64 dwords, so a column's 12 words pair into ds_read2st64/ds_write2st64;
// 2.7 KiB more, still 4 workgroups/CU); the others keep kBlock + 8 so that
// their light data fits 4 workgroups as well.
// Threads per workgroup of a path-kernel instance: kBlock, or one 1024-thread
// workgroup per CU for the light lattices with their records in LDS
// (kLightsGridA10L/A01L: the per-lane LDS is the same, the shared tables and
// records are held once per CU instead of once per 256-thread workgroup).
constexpr int kLatticeBlock = 1024;
__host__ __device__ constexpr bool resumable_geom(int geom);
// The sphere-list (resumable) instances run 64-thread workgroups: a persistent
// launch's tail frees a CU slot per finished wave instead of per finished
// 4-wave workgroup, so the next launch fills it sooner (C3 +2.2 %, 16-spp
// progressive calls 0.964 -> 0.985 of one call); C2 keeps 256 (its frame
// columns' ds_read2st64 stride, -1.2 % at 64).
__host__ __device__ constexpr int block_of(int lmode, int geom) {
    return (lmode == 9 || lmode == 10) ? kLatticeBlock
                                       : (resumable_geom(geom) ? (IPT_GRID_LDS ? IPT_GRID_LDS_BLOCK : IPT_RES_BLOCK) : kBlock);
}
// the wave-spread grid walk's per-lane LDS (IPT_GRID_WAVE): an 8-byte slot
__host__ __device__ constexpr int walk_lds_words(int lmode, int geom) {
    // (the two-cell walk keeps its 64-byte owner table per wave)
    return (IPT_GRID_WAVE && resumable_geom(geom)) ? 2 * block_of(lmode, geom) + (IPT_GRID_WAVE == 2 ? block_of(lmode, geom) / 4 : 0)
                                                   : 0;
}
__host__ __device__ constexpr int frame_stride(int lmode, int geom) {
    return ((lmode == 1 || lmode == 5 || lmode == 6) && walk_lds_words(lmode, geom) == 0 && block_of(lmode, geom) >= 256)
               ? block_of(lmode, geom) + 64
               : block_of(lmode, geom) + 8;
}
__host__ __device__ constexpr size_t scene_lds_words(int lmode, int geom) {
    return (size_t)walk_lds_words(lmode, geom) + 12 * (size_t)frame_stride(lmode, geom) +
           (lmode == 2 ? (size_t)kLdsLights * kLightWords + 2 * (kLdsLights + 1) : 0);
}
// kLightsGlobal: mixture weights + CDF (and, when small, the light BVH) are
// staged in LDS after the fixed layout: their global copies would be evicted
// from L2 by the CosineDdf gathers, and the pick / walk are chains of
// dependent loads.
constexpr int kLdsLightNodesMax = 512;
// [weights | cdf | cdf bucket starts (kCdfBuckets)] then the light BVH nodes or
// the lattice cells, 16-byte aligned
constexpr int kCdfBuckets = 256;
// The lattice instances leave the weights in global memory (read once per hit
// light) so that C5's 256 emitters fit 4 workgroups per CU: [cdf | buckets].
__host__ __device__ inline int global_light_prefix_words(int nl, bool grid = false) {
    return ((grid ? 1 : 2) * (nl + 1) + kCdfBuckets + 3) & ~3;
}
__host__ __device__ inline size_t global_light_lds_words(int nl, int n_nodes_lds, bool grid = false) {
    return (size_t)global_light_prefix_words(nl, grid) + 8 * (size_t)n_nodes_lds;
}

// Where the lights live during the step loop (compile time, so that no
// generic/flat pointer is ever formed: a flat load would make the compiler
// wait for every outstanding radiance store).
enum { kLightsOne = 1, kLightsLds = 2, kLightsGlobal = 3, kLightsAny = 4, kLightsOneA10 = 5, kLightsOneA01 = 6,
       kLightsGridA10 = 7, kLightsGridA01 = 8, kLightsGridA10L = 9, kLightsGridA01L = 10 };
// kLightsGridA10 / A01: many AreaLights, all axis-aligned with the same axis
// pattern, sharing their plane and lying on a lattice, one per cell
// (light_grid_build): a ray's lights are found by its plane point's cell(s)
// instead of the light BVH walk; weights and CDF staged as kLightsGlobal.
// kLightsGridA10L / A01L: the same with the 48-byte records in LDS, one
// 1024-thread workgroup per CU (block_of), chosen when the LDS fits (+5 % C5)
__host__ __device__ constexpr bool grid_lights(int lm) { return lm >= kLightsGridA10 && lm <= kLightsGridA01L; }
__host__ __device__ constexpr bool lattice_a10(int lm) { return lm == kLightsGridA10 || lm == kLightsGridA10L; }
__host__ __device__ constexpr bool lax_in_lds(int lm) { return lm == kLightsGridA10L || lm == kLightsGridA01L; }
__host__ __device__ constexpr bool global_lights(int lm) { return lm == kLightsGlobal || grid_lights(lm); }
// kLightsOneA10 / A01: the single light is an axis-aligned AreaLight
// (axis_aligned_light, ipt_path.h) with x_axis along y and y_axis along x
// (A10, sample_scenes[0]'s light) or along x and y (A01), normal along z
__host__ __device__ constexpr bool one_light(int lm) { return lm == kLightsOne || lm == kLightsOneA10 || lm == kLightsOneA01; }
// kLightsAny: global-memory lights of any type (sphere, point, outer lights
// present); the other modes are AreaLight-only.

template <int LMODE>
struct LightSet {
    const LightDev* lds;
    const LightDev* __restrict__ glob;
    const float* wl;  // weights in LDS
    const float* cl;  // cdf in LDS
    const float* __restrict__ wg;
    const float* __restrict__ cg;
    LightDev one;
    float w0, c0, c1;
    __device__ __forceinline__ const LightDev& light(int i) const {
        if (one_light(LMODE)) return one;
        if (LMODE == kLightsLds) return lds[i];
        return glob[i];  // kLightsGlobal, kLightsAny
    }
    __device__ __forceinline__ float weight(int i) const {
        if (one_light(LMODE)) return w0;
        if (grid_lights(LMODE)) return wg[i];
        if (LMODE == kLightsLds || global_lights(LMODE)) return wl[i];
        return wg[i];
    }
    __device__ __forceinline__ float cdf(int i) const {
        if (one_light(LMODE)) return i == 0 ? c0 : c1;
        if (LMODE == kLightsLds || global_lights(LMODE)) return cl[i];
        return cg[i];
    }
};

// GEOM (IPT_GEOM_*) is a template parameter so that the box instance carries
// neither the sphere-list code nor its pointers (SGPR pressure).
// Sphere-list instances carry the resumable walk's state (IPT_RESUME): they
// are given 3 waves per SIMD of registers (their LDS allows 3 workgroups).
__host__ __device__ constexpr bool resumable_geom(int geom) {
    return IPT_RESUME && (geom == IPT_GEOM_SPHERES_IN_BOX || geom == IPT_GEOM_SPHERES);
}
// many-light instances without a sphere list resume their light-BVH walk the same way
__host__ __device__ constexpr bool resumable_lights(int lmode, int geom) {
    return IPT_RESUME_LIGHTS && lmode == 3 /* kLightsGlobal */ && !resumable_geom(geom);
}
__host__ __device__ constexpr int waves_per_simd(int geom, int lmode) {
    return resumable_geom(geom) ? IPT_RES_WAVES : (resumable_lights(lmode, geom) ? IPT_RESL_WAVES : IPT_WAVES_PER_SIMD);
}
// render_sample's per-sample work before ray_power (main.cpp:192-211) for
// work unit `unit` (pass-major, then candidate row, then column): the absolute
// pass and source pixel (the Philox counter), the two jitter draws, the
// GridRenderPlane drift code (and the flags of drifted samples), the camera
// ray. A unit whose sample lands outside the image or in another shard's row
// gets its value (0) and code stored here and is not traced.
struct RayGen {
    vec3 rd;
    uint32_t a0, a1, a2, a3, rpass, rpix;
    bool valid, drift;
};
__device__ __forceinline__ RayGen new_path_setup(const KParams& kp, unsigned long long unit, bool sharded,
                                                 const int* cand_rows) {
    RayGen g;
    // 32-bit arithmetic with double reciprocals (udiv_exact; units < 2^32)
    const uint32_t u32 = (uint32_t)unit;
    const uint32_t s = udiv_exact(u32, kp.per_pass32, kp.inv_per_pass);
    const uint32_t rem = u32 - s * kp.per_pass32;
    const int cand = (int)udiv_exact(rem, (uint32_t)kp.W, kp.inv_w);
    const int ix = (int)(rem - (uint32_t)cand * (uint32_t)kp.W);
    const int iy = sharded ? cand_rows[cand] : cand;
    g.rpass = (uint32_t)(kp.spp_offset + (int)s);
    g.rpix = (uint32_t)(iy * kp.W + ix);
    philox_fill(g.a0, g.a1, g.a2, g.a3, 0u, g.rpass, g.rpix, kp.key0, kp.key1);
    const float x = jitter_coord(ix, u01(g.a0), kp.W);
    const float y = jitter_coord(iy, u01(g.a1), kp.H);
    int xi, yi;
    grid_index(x, y, kp.W, kp.H, &xi, &yi);
    const int yn = nominal_row(iy, kp.H);
    const int dx = xi - ix, dy = yi - yn;
    uint8_t code = 0xff;
    if (dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1 && xi < kp.W && yi < kp.H)
        code = (uint8_t)((dx + 1) | ((dy + 1) << 2));
    g.drift = code != 0x05 && code != 0xff;
    if (g.drift) {
        kp.flags[(size_t)yn * kp.W + ix] = 1;
        kp.flags[(size_t)yi * kp.W + xi] = 1;
    }
    g.valid = !(code == 0xff || !owned_row(kp, yi));
    g.rd = v3(0, 0, 0);
    if (!g.valid) {
        // not ours (halo row of another shard) or out of range
        kp.values[unit] = 0.0f;
        kp.codes[unit] = code == 0xff ? code : (uint8_t)0xfe;
    } else {
        kp.codes[unit] = code;
        g.rd = camera_dir(kp.cam_right, kp.cam_up, kp.cam_dir, x, y);
    }
    return g;
}

// One thread per work unit of the launch: new_path_setup at full lane
// utilisation (inside the persistent path kernel a refill serves ~2 lanes of a
// wave), written as two 16-byte records {rd.xyz, valid} {a2, a3, pass, pixel}
// that the path kernel's refill reads.
__global__ __launch_bounds__(256) void raygen_kernel(const KParams kp) {
    const unsigned long long unit = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (unit >= kp.total_units) return;
    const bool sharded = !(kp.n_shards <= 1 || kp.tile_rows <= 0);
    const RayGen g = new_path_setup(kp, unit, sharded, kp.cand_rows);
    uint4* out = const_cast<uint4*>(kp.rg) + 2 * unit;
    out[0] = make_uint4(__float_as_uint(g.rd.x), __float_as_uint(g.rd.y), __float_as_uint(g.rd.z), g.valid ? 1u : 0u);
    out[1] = make_uint4(g.a2, g.a3, g.rpass, g.rpix);
    if (kp.count) {
        const uint64_t m = __ballot(g.drift);
        if (m && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)m) - 1))
            atomicAdd(&kp.counters[10], (unsigned long long)__popcll(m));
    }
}

template <int MAXSUSP, bool COUNT, int LMODE, int GEOM>
__global__ __launch_bounds__(block_of(LMODE, GEOM), waves_per_simd(GEOM, LMODE)) void path_kernel(const KParams kp) {
    constexpr int kBlock = block_of(LMODE, GEOM);  // this instance's workgroup size
    extern __shared__ float lds[];
    // IPT_GRID_WAVE (resumable sphere-list instances): a 64-bit test slot and a
    // segment-start byte per lane in front of the stack
    unsigned long long* wslots = reinterpret_cast<unsigned long long*>(lds);
    uint8_t* wown = reinterpret_cast<uint8_t*>(lds + 2 * kBlock);
    float* stk = lds + walk_lds_words(LMODE, GEOM);           // [MAXSUSP][F][kBlock]
    constexpr int kFrameStride = frame_stride(LMODE, GEOM);
    float* lfr = stk + MAXSUSP * kStackFields * kBlock;       // [12][kFrameStride] lane + wall frames
    // IPT_GRID_LDS: the packed grid ranges after the frames
    constexpr bool kGridLds = IPT_GRID_LDS && resumable_geom(GEOM);
    int* grid_lds = reinterpret_cast<int*>(lfr + 12 * kFrameStride);
    LightDev* lights_lds = reinterpret_cast<LightDev*>(lfr + 12 * kFrameStride + (kGridLds ? kp.grid_packed_words : 0));
    float* weights_lds = reinterpret_cast<float*>(lights_lds) + kLdsLights * kLightWords;
    float* cdf_lds = weights_lds + (kLdsLights + 1);
    // kLightsGlobal: [weights | cdf | light BVH nodes] after the frames
    float* gl_lds = reinterpret_cast<float*>(lights_lds) +
                    (LMODE == kLightsLds ? kLdsLights * kLightWords + 2 * (kLdsLights + 1) : 0);
    constexpr bool kGridL = grid_lights(LMODE);
    BvhNode* lnodes_lds = reinterpret_cast<BvhNode*>(gl_lds + global_light_prefix_words(kp.n_lights, kGridL));
    float* cdf_gl = gl_lds + (kGridL ? 0 : kp.n_lights + 1);
    // kLightsGridA10L/A01L: the lattice lights' records after the cells (16-byte aligned)
    constexpr bool kLaxLds = lax_in_lds(LMODE);
    float4* lax_lds = reinterpret_cast<float4*>(reinterpret_cast<int*>(lnodes_lds) + ((kp.lg_nu * kp.lg_nv + 3) & ~3));
    int* cdf_lo_lds = reinterpret_cast<int*>(cdf_gl + kp.n_lights + 1);
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const bool sharded = !(kp.n_shards <= 1 || kp.tile_rows <= 0);
    if (tid < 60) lfr[(tid % 12) * kFrameStride + kBlock + tid / 12] = reinterpret_cast<const float*>(kp.wall_frames)[tid];
    if (kGridLds)
        for (int i = tid; i < kp.grid_packed_words; i += kBlock) grid_lds[i] = kp.grid_packed[i];
    if (LMODE == kLightsLds) {
        const float* src = reinterpret_cast<const float*>(kp.lights);
        float* dst = reinterpret_cast<float*>(lights_lds);
        for (int i = tid; i < kp.n_lights * kLightWords; i += kBlock) dst[i] = src[i];
        for (int i = tid; i <= kp.n_lights; i += kBlock) {
            weights_lds[i] = kp.weights[i];
            cdf_lds[i] = kp.cdf[i];
        }
    }
    if (global_lights(LMODE)) {
        const bool int_cdf = IPT_PICK_INT_CDF && IPT_CDF_POW2 && kp.cdf_p2;
        for (int i = tid; i <= kp.n_lights; i += kBlock) {
            if (!kGridL) gl_lds[i] = kp.weights[i];
            cdf_gl[i] = int_cdf ? __uint_as_float(cdf_threshold24(kp.cdf[i])) : kp.cdf[i];
        }
        if (kp.cdf_lo)
            for (int i = tid; i < kCdfBuckets; i += kBlock) cdf_lo_lds[i] = kp.cdf_lo[i];
        if (grid_lights(LMODE))
            for (int i = tid; i < kp.lg_nu * kp.lg_nv; i += kBlock) reinterpret_cast<int*>(lnodes_lds)[i] = kp.lgrid[i];
        if (kLaxLds)
            for (int i = tid; i < 3 * kp.n_lights; i += kBlock) lax_lds[i] = kp.lax[i];
        if (LMODE == kLightsGlobal && kp.lnodes_lds) {
            const float4* src = reinterpret_cast<const float4*>(kp.light_nodes);
            float4* dst = reinterpret_cast<float4*>(lnodes_lds);
            for (int i = tid; i < 2 * kp.n_light_nodes; i += kBlock) dst[i] = src[i];
        }
    }
    __syncthreads();
    LightSet<LMODE> LS;
    LS.lds = lights_lds;
    LS.glob = kp.lights;
    LS.wl = global_lights(LMODE) ? gl_lds : weights_lds;
    LS.cl = global_lights(LMODE) ? cdf_gl : cdf_lds;
    LS.wg = kp.weights;
    LS.cg = kp.cdf;
    if (one_light(LMODE)) {
        LS.one = kp.lights[0];
        // held in VGPRs (+3.5 % C2; area and spow stay uniform)
        if (IPT_LIGHT_HOLD && (IPT_RES_HOLD || !resumable_geom(GEOM))) {
            vgpr_hold(LS.one.P); vgpr_hold(LS.one.x); vgpr_hold(LS.one.y);
            vgpr_hold(LS.one.n); vgpr_hold(LS.one.inv.c[0]); vgpr_hold(LS.one.inv.c[1]); vgpr_hold(LS.one.inv.c[2]);
        }
        LS.w0 = kp.weights[0];
        LS.c0 = kp.cdf[0];
        LS.c1 = kp.cdf[1];
    }

    // this instance's light functions (axis-aligned single light: the reduced
    // forms of ipt_path.h, exact where observed)
    auto ltrace = [&](const LightDev& L, vec3 o, vec3 d, vec3* hp, vec3* hn) -> bool {
        if constexpr (LMODE == kLightsOneA10) return light_trace_ax<1, 0, IPT_LIGHT_INR>(L, o, d, hp, hn);
        else if constexpr (LMODE == kLightsOneA01) return light_trace_ax<0, 1, IPT_LIGHT_INR>(L, o, d, hp, hn);
        else if constexpr (grid_lights(LMODE) && lattice_a10(LMODE)) return light_trace_ax<1, 0, IPT_LIGHT_INR>(L, o, d, hp, hn);
        else if constexpr (grid_lights(LMODE)) return light_trace_ax<0, 1, IPT_LIGHT_INR>(L, o, d, hp, hn);
        else return light_trace<LMODE == kLightsAny>(L, o, d, hp, hn);
    };
    auto lpdf = [&](const LightDev& L, vec3 o, bool h, vec3 hp, vec3 hn) -> float {
        if constexpr (LMODE == kLightsOneA10 || LMODE == kLightsOneA01) return light_pdf_ax<2, IPT_LIGHT_INR>(L, o, h, hp, hn);
        else if constexpr (grid_lights(LMODE)) return light_pdf_ax<2, IPT_LIGHT_INR>(L, o, h, hp, hn);
        else return light_pdf(L, o, h, hp, hn);
    };
    auto lsample = [&](const LightDev& L, vec3 o, float a, float b) -> vec3 {
        if constexpr (LMODE == kLightsOneA10) return light_sample_dir_ax<1, 0, IPT_LIGHT_INR>(L, o, a, b);
        else if constexpr (LMODE == kLightsOneA01) return light_sample_dir_ax<0, 1, IPT_LIGHT_INR>(L, o, a, b);
        else if constexpr (grid_lights(LMODE) && lattice_a10(LMODE)) return light_sample_dir_ax<1, 0, IPT_LIGHT_INR>(L, o, a, b);
        else if constexpr (grid_lights(LMODE)) return light_sample_dir_ax<0, 1, IPT_LIGHT_INR>(L, o, a, b);
        else return light_sample_dir<LMODE == kLightsAny>(L, o, a, b);
    };

    // the sphere grid walk's parameters (kRes instances), held in VGPRs (+5 % C3)
    KParams kg = kp;
    if (IPT_RES_HOLD && resumable_geom(GEOM)) {
        for (int a = 0; a < 3; ++a) {
            vgpr_hold(kg.grid_g0[a]);
            vgpr_hold(kg.grid_h[a]);
            vgpr_hold(kg.grid_n[a]);
        }
        vgpr_hold(kg.grid_m);
        vgpr_hold(kg.bvh_tmargin);
    }
    const int lane = tid & 63;
    const uint64_t lanemask_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int nl = one_light(LMODE) ? 1 : kp.n_lights;  // a compile-time 1 for one light
    const float w_sdf = kp.weights[nl];
    const unsigned long long per_pass = (unsigned long long)kp.n_cand * (unsigned long long)kp.W;
    // n at every depth is n_rays >> d; when n_rays is a power of two, res/n ==
    // res * 2^-e exactly (both round the same exact quotient)
    const bool n_pow2 = kp.n_rays > 0 && (kp.n_rays & (kp.n_rays - 1)) == 0;
    const int n_log2 = n_pow2 ? 31 - __clz(kp.n_rays) : 0;

    // the setup's vector loads (the single light, weights) complete here, so
    // the step loop's waits never drain them (a conservative vmcnt(0) inside
    // the loop would also drain the step's young table gathers)
    __builtin_amdgcn_s_waitcnt(0);

    // wave-local unit pool (uniform)
    unsigned long long pool_next = 0, pool_end = 0;

    // lane state. The current node lives in registers; suspended ancestors in
    // LDS as {pos.xyz, res, pending multiplier, meta = i | kind<<8}. Frames are
    // never stored: walls load theirs from the LDS table, sphere nodes rebuild
    // theirs (make_frame) in the frame phase of the step after a push or pop.
    bool active = true, has_path = false, fresh = false, need_frame = false, need_b = false;
    // the iteration's pick and draws (prologue) and CosineDdf factors (gathers)
    int pick = -1;
    float u1 = 0.0f, u2 = 0.0f, tr = 0.0f, cs_c = 0.0f, cs_s = 0.0f;
    // IPT_FRAME_PF == 3: the frame-table entry (sin, cos) of the node the lane
    // builds a frame for in the next step, gathered at the end of this step,
    // with its `to` (pfok: `to` inside the table's range)
    float pfs = 0.0f, pfc = 0.0f;
    vec3 pto = v3(0, 0, 0);
    bool pfok = false;
    uint32_t unit = 0;  // < 2^32 per launch (checked by the host)
    uint32_t rpass = 0, rpix = 0, k = 0, blk = 0;
    Win8 w;
    vec3 tpos = v3(0, 0, 0);
    int fdepth = -1;  // depth of the sphere node whose frame is in the lane's column
    uint32_t finm = 0;  // bit l = the node suspended at level l has run all its iterations
    // Resumable sphere-BVH walks (sphere-list scenes): a lane whose walk is not
    // done within IPT_WALK_BUDGET node visits keeps its ray and light results
    // and resumes the walk in the next steps (doing nothing else meanwhile), so
    // a step costs the budget, not the longest walk of the workgroup.
    constexpr bool kRes = resumable_geom(GEOM);
    constexpr bool kResL = resumable_lights(LMODE, GEOM);
    // the frame-entry prefetch pays where every lane iterates every step; in the
    // resumable instances (lanes parked in walks) it measured -5 % on C5
    constexpr int kFramePf = (kRes || kResL) ? 0 : IPT_FRAME_PF;
    // certain light-sample skips taken within the step (the prologue below):
    // the axis-aligned single-light instances, whose ranges are proven
    constexpr bool kSkipAhead = IPT_SKIP_AHEAD && (one_light(LMODE) || grid_lights(LMODE)) && !kResL;
    // ... and the next iteration's certain skip taken at the end of the step,
    // before its pop (the instances that pop at the end of the step)
    constexpr bool kPreSkip = kSkipAhead && IPT_PRE_SKIP && kFramePf == 3;
    bool tracing = false;  // a resumable walk (sphere list or light BVH) is in progress
    float xlmix = 0.0f;    // light walk: the running UnionDdf light sum
    vec3 xro = v3(0, 0, 0), xrd = v3(0, 0, 0), xli_pos = v3(0, 0, 0);
    int xrdepth = 0, xi = 0, xbidx = -1;
    // sphere-list walks (kRes) keep |li_pos - origin|^2 instead of li_pos
    // (resolve's only use of it), and neither the origin nor the depth: the
    // lane's node does not change while it walks, so they are (is_iter ?
    // tpos : camera) and (is_iter ? tdepth + 1 : 0); the plane hit rides in
    // xbidx as -2 - plane (-1: none), negative until a sphere wins (-7 VGPRs:
    // the C3 instance fits 128 without spills)
    float xli_y = 0.0f;
    bool xis_iter = false, xhas_li = false;
    float xmult = 0.0f, xli_pow = 0.0f, xbest = 0.0f;
    vec3 xtm = v3(0, 0, 0);  // grid walk: t of the next cell boundaries
    float tres = 0.0f;
    int ti = 0, tdepth = 0, tkind = 0;  // kind: 0..4 wall plane, 5 box sphere, 6+i extra sphere i
    uint32_t c_paths = 0, c_traced = 0, c_surf = 0, c_light = 0, c_exp = 0, c_iter = 0,
             c_lsamp = 0, c_skip = 0, c_sframe = 0, c_ltr = 0, c_drift = 0, c_nodes = 0, c_tests = 0,
             c_lnode = 0, c_ltest = 0;
    IPT_DIAG_STATE  // diagnostic builds only (ipt_diag.h)

    for (;;) {
        IPT_STAMP_AT(0);  // previous step's tail (resolve, push, stores)
        // -------------------------------------------------- unit refill
        const bool need = active && !has_path;
        const uint64_t needmask = __ballot(need);
        if (needmask) {
            const int cnt = __popcll(needmask);
            const int rank = __popcll(needmask & lanemask_lt);
            unsigned long long avail = pool_end - pool_next;
            unsigned long long my = 0;
            if ((unsigned long long)cnt > avail) {
                unsigned long long base = 0;
                if (lane == __ffsll((long long)needmask) - 1) {
                    base = atomicAdd(kp.unit_counter, (unsigned long long)kPoolChunk);
                    // every unit handed out: release the successor launch's
                    // gate (a plain vector store of this launch's sequence
                    // number; every wave that gets here stores the same value)
                    if (kp.drained && base + kPoolChunk >= kp.total_units)
                        __hip_atomic_store(kp.drained, kp.drain_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                base = __shfl(base, __ffsll((long long)needmask) - 1);
                if ((unsigned long long)rank < avail)
                    my = pool_next + rank;
                else
                    my = base + (rank - avail);
                pool_next = base + (cnt - avail);
                pool_end = base + kPoolChunk;
            } else {
                my = pool_next + rank;
                pool_next += cnt;
            }
            if (need) {
                if (my >= kp.total_units) {
                    active = false;
                } else {
                    unit = (uint32_t)my;
                    has_path = true;
                    fresh = true;
                }
            }
        }

        IPT_STAMP_AT(1);  // refill
        if (active) { IPT_PHASE(0); }
        // ------------------------------- phase 1: finalize + pop (main.cpp:177-183)
        // (IPT_FRAME_PF == 3: at the end of the previous step instead -- the
        // same operations on the same state, nothing changes it in between but
        // the refill of lanes without a path)
        auto pop_node = [&]() {
        if (active && has_path && !fresh && !((kRes || kResL) && tracing) && ti >= (kp.n_rays >> tdepth)) {
            // the node is done: unwind every suspended level whose node has run
            // all its iterations too (finm, set at push) in one pass -- only
            // their res/multiplier are read -- then resume the first level
            // with iterations left (or store the path's value)
            IPT_PHASE(1);
            auto fin_v = [&](float r, int d) {
                float v = 0.0f;
                if (isfinite_(r))
                    v = n_pow2 ? r * __builtin_amdgcn_ldexpf(1.0f, -(n_log2 - d)) : r / (float)(kp.n_rays >> d);
                return v;
            };
            const uint32_t m = ~finm & ((1u << tdepth) - 1u);
            const int stop = m ? 31 - (int)__clz(m) : -1;
            // every LDS read of the unwind issued before the first use -- the
            // resumed level's six fields and the res/multiplier of the first
            // two finished levels (addresses clamped to level 0 where a level
            // does not exist; those values are not used) -- so that their
            // latencies overlap instead of forming a chain; the outcomes as
            // selects so that the loads have unconditional consumers
            auto lvl = [&](int l) { return stk + (size_t)(l < 0 ? 0 : l) * kStackFields * kBlock + tid; };
            const float* bs = lvl(stop);
            const float s0 = bs[0 * kBlock], s1 = bs[1 * kBlock], s2 = bs[2 * kBlock];
            const float s3 = bs[3 * kBlock], s4 = bs[4 * kBlock], s5 = bs[5 * kBlock];
            const float* b1 = lvl(tdepth - 1);
            const float r1 = b1[3 * kBlock], m1 = b1[4 * kBlock];
            const float* b2 = lvl(tdepth - 2);
            const float r2 = b2[3 * kBlock], m2 = b2[4 * kBlock];
            auto fin_s = [&](float r, int d) {
                const float q = n_pow2 ? r * __builtin_amdgcn_ldexpf(1.0f, -(n_log2 - d))
                                       : r / (float)(kp.n_rays >> (d < 0 ? 0 : d));
                return isfinite_(r) ? q : 0.0f;
            };
            float v = fin_s(tres, tdepth);
            const float v1 = fin_s(r1 + (m1 * 1.0f) * v, tdepth - 1);
            v = tdepth - 1 > stop ? v1 : v;
            const float v2 = fin_s(r2 + (m2 * 1.0f) * v, tdepth - 2);
            v = tdepth - 2 > stop ? v2 : v;
            for (int l = tdepth - 3; l > stop; --l) {
                const float* b = lvl(l);
                v = fin_v(b[3 * kBlock] + (b[4 * kBlock] * 1.0f) * v, l);
            }
            const bool resume = stop >= 0;
            const int meta = __float_as_int(s5);
            tpos = resume ? v3(s0, s1, s2) : tpos;
            tres = resume ? s3 + (s4 * 1.0f) * v : tres;  // res += multiplier*albedo*ray_power
            // (unsigned: with n_rays > 255 a kind of 6 + sphere index >= 32768
            // sets bit 31 of the word, which must not sign-extend)
            const int mkind = (int)((uint32_t)meta >> kp.meta_shift);
            ti = resume ? meta & ((1 << kp.meta_shift) - 1) : ti;
            tkind = resume ? mkind : tkind;
            need_frame = resume ? mkind >= 5 && fdepth != stop : need_frame;
            tdepth = resume ? stop : tdepth;
            if (!resume) {
                kp.values[unit] = v >= 0.0f ? v : 0.0f;  // main.cpp:214
                has_path = false;
            }
        }
        };
        if (kFramePf != 3) pop_node();

        IPT_STAMP_AT(2);  // finalize + pop
        // the current node's frame normal (frame build below)
        auto frame_normal = [&]() -> vec3 {
            vec3 nrm;
            if (GEOM == IPT_GEOM_SPHERE_IN_BOX || tkind == 5) {
                nrm = tpos;  // normalize(position), GeometrySphereInBox.cpp:67
            } else {
                const float4 sp = kp.spheres[tkind - 6];
                nrm = tpos - v3(sp.x, sp.y, sp.z);  // FractalSpheres.cpp:91
                // GeometrySmallPt.cpp:41: -normalize(v) for the room spheres;
                // normalize(-v) is the same bits (negation is exact)
                if (GEOM == IPT_GEOM_SMALLPT && !((double)sp.w < 100.0)) nrm = -nrm;
            }
            return nrm;
        };
        constexpr bool kFrameInrange = GEOM == IPT_GEOM_SPHERE_IN_BOX;  // range-free frame roots / quotients (+1.4 % C2)
        const bool fneed = need_frame && has_path && !fresh && !((kRes || kResL) && tracing);
        IPT_STAMP_AT(3);  // (new path: later in the step)
        // iteration prologue: RNG window, UnionDdf pick (ddf.cpp:142-153) and,
        // for a cosine pick, the CosineDdf table gathers (running it one step
        // ahead, right after the direction phase, measured -2.7 %: DESIGN.md 4.3)
        const bool iter_lane = active && has_path && !fresh && !((kRes || kResL) && tracing);
        if constexpr (kRes) {
            // the iteration's pick, draws and CosineDdf factors live within the
            // step (set by the prologue / gathers, used by the direction phase):
            // overwritten here, they are not carried across the step loop's back
            // edge (-13 VGPRs: the sphere-list instances fit 4 waves per SIMD;
            // the others measured 1 % slower this way)
            pick = -1;
            u1 = u2 = tr = cs_c = cs_s = 0.0f;
        }
        // the cosine pick's table indices; the gathers are issued by the whole
        // wave after the prologue (index 0 for the other lanes) so that the
        // number of loads between a gather and its wait is the same on every
        // path and the compiler's waits drain only what they wait for
        uint32_t gi_a = 0, gi_b = 0;
        bool gcos = false;
        // kPreSkip: the word after the iteration's draws (the next pick) and
        // whether the end of the step may take it (set by the prologue)
        uint32_t pre_w = 0u;
        bool pre_ok = false;
        // IPT_LPF (lattice instances): the picked light's sample fields are
        // gathered with the CosineDdf gathers (whole wave, index 0 for lanes
        // without a light pick) instead of read in the direction phase
        vec3 lpP = v3(0, 0, 0);
        float lpx = 0.0f, lpy = 0.0f, lpn = 0.0f;
        int lptype = 0;
        // (`ran`: the lane ran the prologue in this step. In the resumable
        // instances a lane keeps its prepared iteration while its walk goes on,
        // so there the gathers stay per lane.)
        auto gathers = [&](bool ran) {
            if constexpr (kRes || kResL) {
                if (ran && gcos) {
                    tr = kp.cos_a[gi_a];
                    float sp, cp;
                    sincosf_small_(two_pi_times_u24(gi_b), &sp, &cp);
                    cs_c = cp;
                    cs_s = sp;
                }
            } else {
                if constexpr (grid_lights(LMODE) && IPT_LPF && IPT_LIGHT_AX_REC) {
                    // the compact record's first 16 bytes: P.xy, x[XA], y[YA]
                    // (P.z, n.z: the lattice plane; lattice lights are diamonds)
                    const int pk = (ran && pick >= 0 && pick < nl) ? pick : 0;
                    if (IPT_LPF_CALC && kp.lpf_calc) {
                        // the same floats from the lattice's formula (no LDS
                        // read on the pick -> light sample chain)
                        lpP = v3(kp.lc_x0 + (float)(pk & ((1 << kp.lc_shift) - 1)) * kp.lc_dx,
                                 kp.lc_y0 + (float)(pk >> kp.lc_shift) * kp.lc_dy, kp.lg_pn);
                        lpx = kp.lc_ax;
                        lpy = kp.lc_ay;
                    } else {
                        const float4 a = kLaxLds ? lax_lds[3 * pk] : kp.lax[3 * pk];
                        lpP = v3(a.x, a.y, kp.lg_pn);
                        lpx = a.z;
                        lpy = a.w;
                    }
                    lpn = kp.lg_nn;
                    lptype = 0;
                } else if constexpr (grid_lights(LMODE) && IPT_LPF) {
                    constexpr int XA = lattice_a10(LMODE) ? 1 : 0, YA = 1 - XA;
                    const LightDev& Ls = kp.lights[(ran && pick >= 0 && pick < nl) ? pick : 0];
                    lpP = Ls.P;
                    lpx = comp<XA>(Ls.x);
                    lpy = comp<YA>(Ls.y);
                    lpn = comp<2>(Ls.n);
                    lptype = Ls.type;
                }
                // (cos phi, sin phi) computed (the table kernel's own code): one
                // table line per cosine sample instead of two (computing r as
                // well, or non-temporal gathers, measured slower: DESIGN.md 4.3)
                tr = kp.cos_a[gcos ? gi_a : 0u];
                if constexpr (IPT_COSB_TAB) {
                    // (cos phi, sin phi) gathered from the exact table as well
                    const float2 cb = kp.cos_b[gcos ? gi_b : 0u];
                    cs_c = cb.x;
                    cs_s = cb.y;
                } else {
                    float sp, cp;
                    sincosf_small_(two_pi_times_u24(gi_b), &sp, &cp);
                    cs_c = cp;
                    cs_s = sp;
                }
            }
        };
        auto prologue = [&]() {
            if ((k >> 2) != blk) {
                w.a0 = w.b0; w.a1 = w.b1; w.a2 = w.b2; w.a3 = w.b3;
                ++blk;
                need_b = true;
            }
            if (need_b) {
                IPT_PHASE(4);
                philox_fill(w.b0, w.b1, w.b2, w.b3, blk + 1, rpass, rpix, kp.key0, kp.key1);
                need_b = false;
            }
            // j = k - 4*blk: the window was shifted above. kPreSkip: a step that
            // took the next pick's skip may end 9 words past blk, so after the
            // one shift j <= 5 (words j .. j+2 are still in the window)
            const uint32_t j = kPreSkip ? k - 4u * blk : k & 3u;
            const uint32_t rw = kPreSkip && j >= 4u ? (j & 1u ? w.b1 : w.b0) : sel4(j & 3u, w.a0, w.a1, w.a2, w.a3);
            const float r = u01(rw);
            // the single light's pick on the raw word: r < cdf[c] as w < pk_u (host-exact)
            auto pick_w = [&](uint32_t wd) {
                return (unsigned long long)wd < kp.pk_u0 ? 0 : ((unsigned long long)wd < kp.pk_u1 ? 1 : 2);
            };
            constexpr bool kPickInt = IPT_PICK_INT && one_light(LMODE);
            // UnionDdf::sample's component: the first c with r < cdf[c] (ddf.cpp:142-153)
            auto pick_of = [&](float r) {
                int c = 0;
                if (one_light(LMODE)) {
                    c = r < LS.c0 ? 0 : (r < LS.c1 ? 1 : 2);
                } else if (global_lights(LMODE) && IPT_CDF_POW2 && kp.cdf_p2) {
                    // (host-checked near-uniform cdf: ce - 1, ce or ce + 1)
                    const int ce = min((int)(r * kp.cdf_p2s), nl);
                    const float fa = LS.cdf(max(ce - 1, 0)), fb = LS.cdf(ce);
                    c = (ce >= 1 && r < fa) ? ce - 1 : (r < fb ? ce : ce + 1);
                    if (c >= nl) c = r < kp.cdf_end ? nl : nl + 1;
                } else if (global_lights(LMODE) && kp.cdf_lo) {
                    // the scan from the first index whose cdf exceeds r's bucket
                    // start floor(256 r)/256 (host table): every earlier entry is
                    // <= that start <= r, so the scan would pass it; a bucket holds
                    // at most 8 entries (else the table is not built)
                    c = cdf_lo_lds[(int)(r * 256.0f)];
                    if (kp.cdf_bsearch) {
                        // non-decreasing cdf: the answer is c plus the number of
                        // the entries from c on that r does not undercut, a
                        // prefix; the first three are read at once (C5: two
                        // lights per bucket), the scan past them is a rare branch
                        const float f0 = LS.cdf(min(c, nl)), f1 = LS.cdf(min(c + 1, nl)), f2 = LS.cdf(min(c + 2, nl));
                        const int n0 = (c <= nl && !(r < f0)) ? 1 : 0;
                        const int n1 = (c + 1 <= nl && !(r < f1)) ? 1 : 0;
                        const int n2 = (c + 2 <= nl && !(r < f2)) ? 1 : 0;
                        const bool more = n2 != 0;
                        c += n0 + n1 + n2;
                        if (__builtin_expect(__any(more), 0))
                            if (more) while (c <= nl && !(r < LS.cdf(c))) ++c;
                    } else {
                        while (c <= nl && !(r < LS.cdf(c))) ++c;
                    }
                } else if ((global_lights(LMODE) || LMODE == kLightsAny) && kp.cdf_bsearch) {
                    // first c with r < cdf[c] (else nl+1): the scan's answer on a
                    // non-decreasing cdf (checked at upload)
                    int hi = nl + 1;
                    while (c < hi) {
                        const int mid = (c + hi) >> 1;
                        if (r < LS.cdf(mid)) hi = mid; else c = mid + 1;
                    }
                } else {
                    while (c <= nl && !(r < LS.cdf(c))) ++c;
                }
                return c;
            };
            // the near-uniform many-light pick on the draw's 24-bit integer
            // (the staged cdf holds ceil(cdf 2^24), KParams::cdf_p2e)
            auto pick_p2w = [&](uint32_t wd) {
                const uint32_t g = wd >> 8;
                const int ce = min((int)(g >> (24 - kp.cdf_p2e)), nl);
                if (kp.cdf_p2 == 2) {
                    // every light's threshold is exactly (i+1) 2^(24-e)
                    // (host-checked): the first i with g < T[i] is ce itself
                    return ce < nl ? ce : (g < kp.cdf_end_t ? nl : nl + 1);
                }
                const uint32_t fa = __float_as_uint(LS.cdf(max(ce - 1, 0))), fb = __float_as_uint(LS.cdf(ce));
                int c = (ce >= 1 && g < fa) ? ce - 1 : (g < fb ? ce : ce + 1);
                if (c >= nl) c = g < kp.cdf_end_t ? nl : nl + 1;
                return c;
            };
            constexpr bool kPickIntCdf = IPT_PICK_INT_CDF && IPT_CDF_POW2 && global_lights(LMODE);
            auto pick_word = [&](uint32_t wd) {
                if constexpr (kPickInt) return pick_w(wd);
                if constexpr (kPickIntCdf)
                    if (kp.cdf_p2) return pick_p2w(wd);
                return pick_of(u01(wd));
            };
            int c = (kPickInt || kPickIntCdf) ? pick_word(rw) : pick_of(r);
            uint32_t jj = j;  // the window offset of the iteration's pick (skip-ahead: j + 3)
            if constexpr (kSkipAhead) {
                // A light pick at a node on the lights' back side is a certain
                // skip: DdfFromLight::sample returns vec3() when cosinus < 1e-5
                // (lighting.cpp:125-134), and for these axis-aligned lights (one,
                // or a coplanar lattice) the sampled point's normal-axis
                // coordinate is P[2] whatever the two draws, so cosinus = n[2] *
                // -RN(RN(P[2] - o[2]) * s) (+ signed zeros, generic light code;
                // s = 1/|pos - o| >= 0: pos.z != o.z and |P[2]| >= 2^-32, so
                // |pos - o|^2 >= 2^-112 does not underflow; an overflow gives
                // s = 0 and cosinus = +-0) is <= 0 whenever n[2] * (P[2] - o[2])
                // > 0 (sa_on: host-checked). Such an iteration does nothing but
                // consume its three draws and count (main.cpp:149-163), so the
                // lane takes the next iteration's pick (word j + 3) in the same
                // step -- when the node has an iteration left and that pick's
                // draws are in the window without a shift (j <= 1: words j+3 ..
                // j+5 <= 6, and k ends below 4*(blk+2)). Same draws, same order,
                // same results; a lane on the back side of the lights spends one
                // step instead of two on the pair. (The draws below are then
                // selected at offset jj = j + 3: one pick computation serves
                // both cases.) (j = 2 as well -- words 5 .. 7, and the next
                // step reading its pick at j = 4 after one shift -- measured
                // +0.2 % on C2, -0.4 % on C5 and C3: not taken.)
                // (o.z - P.z) * n.z < 0: the rounded difference keeps its sign
                // and is zero only when o.z == P.z; an underflowed product is
                // +-0, i.e. not taken (conservative)
                const bool back = (tpos.z - kp.sa_pz) * kp.sa_nz < 0.0f;
                if (kp.sa_on && c < nl && back && j <= 1u && ti + 1 < (kp.n_rays >> tdepth)) {
                    ++ti;
                    if (COUNT) { ++c_iter; ++c_lsamp; ++c_skip; }
                    k += 3;
                    jj = j + 3u;
                    c = pick_word(j == 0u ? w.a3 : w.b0);  // word j + 3
                }
            }
            pick = c;
            if (c <= nl) {
                // words jj+1, jj+2 (jj <= 4 in the skip-ahead instances, <= 5
                // with kPreSkip, else <= 3)
                const bool hi = kSkipAhead && jj >= 4u;
                const uint32_t r1 = hi ? (kPreSkip && (jj & 1u) ? w.b2 : w.b1) : sel4(jj & 3u, w.a1, w.a2, w.a3, w.b0);
                const uint32_t r2 = hi ? (kPreSkip && (jj & 1u) ? w.b3 : w.b2) : sel4(jj & 3u, w.a2, w.a3, w.b0, w.b1);
                if constexpr (kPreSkip) {
                    // the next pick's word jj+3 (taken only at jj <= 3: the step
                    // then ends at most 9 words past blk)
                    pre_w = sel4(jj & 3u, w.a3, w.b0, w.b1, w.b2);
                    pre_ok = jj <= 3u && kp.sa_on;
                }
                u1 = u01(r1);
                u2 = u01(r2);
                if (c == nl) {
                    // CosineDdf::sample (ddf.cpp:223-231) of (u1, u2): (cos_alpha, r) x
                    // (cos phi, sin phi) looked up by the draws' 24 bits
                    // (a non-temporal hint measured slower on C2 and C5)
                    // (cos_alpha = sqrtf(u1) is recomputed in the direction phase)
                    gi_a = r1 >> 8;
                    gi_b = r2 >> 8;
                    gcos = true;
                }
                k += 3;
            } else {
                k += 1;  // fall-through: defined as vec3() (reference UB, ddf.cpp:139)
            }
        };
        if (iter_lane) {
            IPT_PHASE(3);
            prologue();
        }
        gathers(iter_lane);
        // (the frame build sits between the table gathers' issue and their use)
        // ------------- phase 3: the current node's RotateDdf frame when it is a sphere node without one
        // (after a push, or a pop past a sphere descendant): built by the lane
        // itself into its LDS column. Waves share no LDS after the setup, so they
        // run without barriers (a pooled workgroup frame pass with two barriers
        // per step measured 5-13 % slower).
        if (fneed) {
            const vec3 nrm = frame_normal();
            IPT_PHASE(5);
            Frame f;
            // the sphere-in-box node's normal comes from a point on the r = 0.5
            // sphere: every root and quotient of the frame is in the range-free
            // sequences' range (make_frame<true>)
            if (IPT_FRAME_TAB && GEOM == IPT_GEOM_SPHERE_IN_BOX) {
                // (sphere-list scenes: measured slower with the table's
                // gathers in their latency-bound walks)
                vec3 to;
                float fs = 0.0f, fc = 0.0f;
                if (kFramePf == 3) {
                    // `to` and its frame-table entry, prepared at the end of
                    // the previous step (pfok: `to` inside the table's range)
                    to = pto;
                    fs = pfs;
                    fc = pfc;
                    if constexpr (!IPT_FRAME_FB_PF) {
                    if (__builtin_expect(__any(!pfok), 0))
                        if (!pfok) {
                            to = kFrameInrange ? normalize_inrange_(nrm) : normalize(nrm);
                            frame_sc_lookup(kp.frame_sc, to, fs, fc);
                            keep_alive(fs);  // its wait stays in this rare branch
                            keep_alive(fc);
                        }
                    }
                    pfok = false;
                } else {
                    to = kFrameInrange ? normalize_inrange_(nrm) : normalize(nrm);
                    frame_sc_lookup(kp.frame_sc, to, fs, fc);
                }
                if (kFrameInrange) {
                    // without the zero terms; the rare lanes where a term
                    // could decide a zero's sign take the exact build
                    bool ok;
                    f = make_frame_sc_fast(to, fs, fc, ok);
                    if (__builtin_expect(__any(!ok), 0))
                        if (!ok) f = make_frame_sc<kFrameInrange>(to, fs, fc);
                } else {
                    f = make_frame_sc<kFrameInrange>(to, fs, fc);
                }
            } else if (kFrameInrange) {
                f = make_frame<true>(normalize_inrange_(nrm));
            } else {
                // sphere-list scenes: the f64 angle, then the fast build
                // (its own range checks; a normalized `to`), exact fallback
                const vec3 to = normalize(nrm);
                float fs, fc;
                if (IPT_FRAME_TAB && IPT_FRAME_TAB_LISTS && GEOM == IPT_GEOM_SPHERES_IN_BOX)
                    frame_sc_lookup(kp.frame_sc, to, fs, fc);
                else
                    frame_angle_sc(to, &fs, &fc);
                bool ok;
                f = make_frame_sc_fast(to, fs, fc, ok);
                if (__builtin_expect(__any(!ok), 0))
                    if (!ok) f = make_frame_sc<false>(to, fs, fc);
            }
            float* c = lfr + tid;
            c[0 * kFrameStride] = f.m0.x; c[1 * kFrameStride] = f.m0.y; c[2 * kFrameStride] = f.m0.z;
            c[3 * kFrameStride] = f.m1.x; c[4 * kFrameStride] = f.m1.y; c[5 * kFrameStride] = f.m1.z;
            c[6 * kFrameStride] = f.m2.x; c[7 * kFrameStride] = f.m2.y; c[8 * kFrameStride] = f.m2.z;
            c[9 * kFrameStride] = f.iz.x; c[10 * kFrameStride] = f.iz.y; c[11 * kFrameStride] = f.iz.z;
            need_frame = false;
            fdepth = tdepth;
        }
        if (IPT_PROF && wave == 0) { IPT_PHASE(11); }  // workgroup steps (one wave counts)
        IPT_STAMP_AT(4);  // task posting, iteration prologue, Philox
        // the wave's exit test (waves are independent after the setup barrier)
        if (!__ballot(active)) break;
        IPT_STAMP_AT(5);
        // the current node's frame: its wall column or the lane's own column
        const float* frc = lfr + (tkind < 5 ? kBlock + tkind : tid);

        bool have_ray = false, is_iter = false;
        // (written by the new-path or the direction phase wherever have_ray is
        // set and read only then: left uninitialised, no per-step moves)
        vec3 ro, rd;
        int rdepth;
        // ------------- phase 2: new path (render_sample body, main.cpp:192-211), after
        // barrier B so that its camera ray is not live across the worker pass
        if (active && has_path && fresh) {
            IPT_PHASE(2);
            fresh = false;
            if (IPT_RAYGEN) {
                // raygen_kernel ran render_sample's per-sample work for this
                // unit (jitter, drift code and flags, camera ray, Philox block 0)
                // both records load together and are consumed here: no load of
                // this (divergent) phase is left in flight for later waits
                uint4 r0 = kp.rg[2 * unit], r1 = kp.rg[2 * unit + 1];
                keep_alive(r0);
                keep_alive(r1);
                if (r0.w == 0u) {
                    has_path = false;  // not ours / out of range: already stored
                } else {
                    ro = kp.cam_pos;
                    rd = v3(__uint_as_float(r0.x), __uint_as_float(r0.y), __uint_as_float(r0.z));
                    w.a2 = r1.x;
                    w.a3 = r1.y;
                    rpass = r1.z;
                    rpix = r1.w;
                    blk = 0;
                    need_b = true;  // block 1 is produced by the window refill of the next iteration
                    k = 2;
                    rdepth = 0;
                    have_ray = true;
                    if (COUNT) ++c_paths;
                }
            } else {
            const RayGen g = new_path_setup(kp, unit, sharded, kp.cand_rows);
            w.a0 = g.a0;
            w.a1 = g.a1;
            w.a2 = g.a2;
            w.a3 = g.a3;
            rpass = g.rpass;
            rpix = g.rpix;
            blk = 0;
            need_b = true;
            k = 2;
            if (COUNT && g.drift) ++c_drift;
            if (!g.valid) {
                has_path = false;
            } else {
                ro = kp.cam_pos;
                rd = g.rd;
                rdepth = 0;
                have_ray = true;
                if (COUNT) ++c_paths;
            }
            }
        }

        // ------------------------- phase 3b: the iteration's direction (main.cpp:149-163)
        // kLightsOne: both candidate directions are computed by every lane and
        // one is selected (a mixed wave runs both anyway), so the CosineDdf
        // gathers have an unconditional consumer and stay unconditional loads
        vec3 dir_bf = v3(0, 0, 0);
        // (the lattice instances measured 3 % slower this way: their light sample
        // reads the picked light's record, and both directions cost more there)
        constexpr bool kDirBf = one_light(LMODE);
        if constexpr (kDirBf) {
            Frame fm;
            fm.m0 = v3(frc[0 * kFrameStride], frc[1 * kFrameStride], frc[2 * kFrameStride]);
            fm.m1 = v3(frc[3 * kFrameStride], frc[4 * kFrameStride], frc[5 * kFrameStride]);
            fm.m2 = v3(frc[6 * kFrameStride], frc[7 * kFrameStride], frc[8 * kFrameStride]);
            const vec3 cdir = frame_apply(fm, v3(tr * cs_c, tr * cs_s, sqrt_inrange_(u1)));
            const vec3 ldir = lsample(LS.one, tpos, u1, u2);
            const vec3 zero = v3(0, 0, 0);
            dir_bf = pick < nl ? ldir : (pick == nl ? cdir : zero);
        }
        if (iter_lane) {
            vec3 dir = v3(0, 0, 0);
            if (kDirBf) {
                dir = dir_bf;
                if (COUNT && pick < nl) ++c_lsamp;
            } else if (pick < nl) {
                IPT_PHASE(7);
                if constexpr (grid_lights(LMODE) && IPT_LPF) {
                    // the gathered fields are all light_sample_dir_ax reads
                    constexpr int XA = lattice_a10(LMODE) ? 1 : 0, YA = 1 - XA;
                    dir = light_sample_dir_axf<XA, YA, IPT_LIGHT_INR>(lpP, lpx, lpy, lpn, lptype, tpos, u1, u2);
                } else
                dir = lsample(LS.light(pick), tpos, u1, u2);
                if (COUNT) ++c_lsamp;
            } else if (pick == nl) {
                Frame fm;
                fm.m0 = v3(frc[0 * kFrameStride], frc[1 * kFrameStride], frc[2 * kFrameStride]);
                fm.m1 = v3(frc[3 * kFrameStride], frc[4 * kFrameStride], frc[5 * kFrameStride]);
                fm.m2 = v3(frc[6 * kFrameStride], frc[7 * kFrameStride], frc[8 * kFrameStride]);
                // cosine_sample_local from the tables: (r cos phi, r sin phi, cos_alpha)
                // with u2 = r and cos_alpha = sqrtf(u1)
                // u1 is 0 or in [2^-24, 1): the range-free root is sqrtf there
                // (math probe 13 is exhaustive on [2^-96, 2^126); sqrt_inrange_(0) = +0)
                dir = frame_apply(fm, v3(tr * cs_c, tr * cs_s, sqrt_inrange_(u1)));
            }
            ++ti;
            if (COUNT) ++c_iter;
            if (is_zero(dir)) {
                if (COUNT) ++c_skip;
            } else {
                ro = tpos;
                rd = dir;
                rdepth = tdepth + 1;
                have_ray = true;
                is_iter = true;
            }
        }
        IPT_STAMP_AT(8);  // direction
        // --------------------------------------------- phase 4: trace + resolve
        // the child's value (main.cpp:100-143) from its traces, then push it,
        // add it to the current node's sum, or finish the path
        auto resolve = [&](bool traced, float t, int prim, vec3 o, vec3 d, int depth, bool iter, float mult,
                           bool has_li, float li_y, float li_pow) {
            float cv = 0.0f;
            bool push = false;
            vec3 si_pos = v3(0, 0, 0);
            {
                // the reference's hit / light / expand decision (main.cpp:100-143)
                // as selects (the branches only cost exec-mask bookkeeping in
                // waves that mix outcomes: +1 %)
                const bool has_si = prim >= 0;
                if (COUNT && traced) {
                    ++c_traced;
                    c_surf += has_si ? 1u : 0u;
                    c_light += has_li ? 1u : 0u;
                }
                si_pos = o + d * t;
                // y = |li_pos - o|^2, computed by the caller
                const vec3 ea = si_pos - o;
                const float x = dot(ea, ea), y = li_y;
                // longer(si_pos - o, li_pos - o), asked only where both hits exist
                const bool need = has_li && has_si;
                bool lg = x > y * 1.000001907f && y >= 1e-30f;
                const bool tie = need && (!lg && !(x <= y));
                if (__builtin_expect(__any(tie), 0))
                    if (tie) lg = sqrt_(x) > sqrt_(y);
                const bool li_wins = has_li && (!has_si || lg);
                const int nchild = kp.n_rays >> depth;
                const float zero = 0.0f;
                // 0/0 for an expanded node without children: the NaN that
                // poisons the parent (main.cpp:181)
                const float cv_exp = nchild == 0 ? zero / (float)nchild : 0.0f;
                cv = li_wins ? (isfinite_(li_pow) ? li_pow : 1.0f) : (has_si ? cv_exp : 0.0f);
                cv = traced ? cv : 0.0f;
                push = traced && !li_wins && has_si && nchild != 0;
                if (COUNT && traced && !li_wins && has_si) ++c_exp;
            }
            if (push) {
                IPT_PHASE(10);
                if (iter) {
                    finm = (finm & ~(1u << tdepth)) | ((ti >= (kp.n_rays >> tdepth) ? 1u : 0u) << tdepth);
                    float* b = stk + (size_t)tdepth * kStackFields * kBlock + tid;
                    b[0 * kBlock] = tpos.x;
                    b[1 * kBlock] = tpos.y;
                    b[2 * kBlock] = tpos.z;
                    b[3 * kBlock] = tres;
                    b[4 * kBlock] = mult;
                    b[5 * kBlock] = __uint_as_float((uint32_t)ti | ((uint32_t)tkind << kp.meta_shift));
                }
                tpos = si_pos;
                tkind = prim;
                if (prim >= 5) {
                    need_frame = true;  // built by the frame pass of the next step
                    if (COUNT) ++c_sframe;
                }
                tres = 0.0f;
                ti = 0;
                tdepth = depth;
            } else if (iter) {
                tres = tres + (mult * 1.0f) * cv;
            } else {
                // the camera ray itself ended (light, miss, depth_max or n_rays==0)
                kp.values[unit] = cv >= 0.0f ? cv : 0.0f;
                has_path = false;
            }
        };
        if constexpr (kResL) {
            // many lights: the light-BVH walk (same order and arithmetic as the
            // full walk below) is bounded per step and resumed; then the mixture
            // value, the geometry trace and resolve, as below
            if (have_ray) {
                IPT_PHASE(8);
                if (COUNT) c_ltr += (uint32_t)nl * ((is_iter ? 1u : 0u) + ((rdepth < kp.depth_max) ? 1u : 0u));
                xro = ro;
                xrd = rd;
                xrdepth = rdepth;
                xis_iter = is_iter;
                xlmix = 0.0f;
                xhas_li = false;
                xli_pos = v3(0, 0, 0);
                xli_pow = 0.0f;
                xi = 0;
                tracing = true;
            }
            if (tracing) {
                if (kp.n_light_nodes > 0) {
                    const vec3 inv = v3(safe_rcp(xrd.x), safe_rcp(xrd.y), safe_rcp(xrd.z));
                    auto walk = [&](const BvhNode* __restrict__ lnodes) {
                    int budget = IPT_LWALK_BUDGET;
                    while (xi < kp.n_light_nodes && budget > 0) {
                        int leaf = -1;
                        while (xi < kp.n_light_nodes && budget > 0) {
                            --budget;
                            const BvhNode nd = lnodes[xi];
                            if (COUNT) ++c_lnode;
                            const bool enter = bvh_box_entry(nd, xro, inv) != inf_();
                            if (enter && nd.leaf >= 0) {
                                leaf = nd.leaf;
                                xi = nd.skip;
                                break;
                            }
                            xi = enter ? xi + 1 : nd.skip;
                        }
                        if (leaf >= 0) {
                            const int first = leaf & 0xffffff, cnt = leaf >> 24;
                            for (int l = first; l < first + cnt; ++l) {
                                const LightDev& L = LS.light(l);
                                vec3 hp, hn;
                                const bool h = light_trace<false>(L, xro, xrd, &hp, &hn);
                                if (COUNT) ++c_ltest;
                                if (xis_iter) xlmix += LS.weight(l) * light_pdf(L, xro, h, hp, hn);
                                if (h && (!xhas_li || longer(xli_pos - xro, hp - xro))) {
                                    xhas_li = true;
                                    xli_pos = hp;
                                    xli_pow = L.spow;
                                }
                            }
                        }
                    }
                    };
                    if (kp.lnodes_lds)
                        walk(lnodes_lds);
                    else
                        walk(kp.light_nodes);
                } else {
                    for (int l = 0; l < nl; ++l) {
                        const LightDev& L = LS.light(l);
                        vec3 hp, hn;
                        const bool h = light_trace<false>(L, xro, xrd, &hp, &hn);
                        if (COUNT) ++c_ltest;
                        if (xis_iter) xlmix += LS.weight(l) * light_pdf(L, xro, h, hp, hn);
                        if (h && (!xhas_li || longer(xli_pos - xro, hp - xro))) {
                            xhas_li = true;
                            xli_pos = hp;
                            xli_pow = L.spow;
                        }
                    }
                    xi = kp.n_light_nodes;
                }
                if (xi >= kp.n_light_nodes) {
                    tracing = false;
                    float mult = 0.0f;
                    if (xis_iter) {
                        const float* fc = lfr + (tkind < 5 ? kBlock + tkind : tid);
                        Frame fz;
                        fz.iz = v3(fc[9 * kFrameStride], fc[10 * kFrameStride], fc[11 * kFrameStride]);
                        const float sdf_val = frame_cosine_value(fz, xrd);
                        const float mix = xlmix + w_sdf * sdf_val;
                        mult = div_(sdf_val, mix);
                    }
                    int prim = -1;
                    float t = inf_();
                    if (xrdepth < kp.depth_max) {
                        IPT_PHASE(9);
                        t = trace_geometry<COUNT, GEOM>(kp, xro, xrd, &prim, c_nodes, c_tests);
                    }
                    const vec3 eb = xli_pos - xro;
                    resolve(xrdepth < kp.depth_max, t, prim, xro, xrd, xrdepth, xis_iter, mult, xhas_li, dot(eb, eb),
                            xli_pow);
                }
            }
        } else {
        if (have_ray) {
            IPT_PHASE(8);
            // lights: per-light traces feed both UnionDdf::value (ddf.cpp:157-162)
            // and the child's CollectionLighting::traceRayToLight
            float lmix = 0.0f;
            bool has_li = false;
            vec3 li_pos = v3(0, 0, 0);
            float li_pow = 0.0f;
            // coplanar lattice: the lights' shared n[2]*d[2] and plane quotient,
            // computed once by the lookup below with light_trace_ax's operations
            float lg_ndir = 0.0f, lg_t = 0.0f;
            vec3 lg_q = v3(0, 0, 0);
            auto light_step_with = [&](const LightDev& L, float wl) {
                vec3 hp, hn;
                bool h;
                if constexpr (grid_lights(LMODE) && IPT_LIGHT_INR) {
                    constexpr int XA = lattice_a10(LMODE) ? 1 : 0, YA = 1 - XA;
                    h = light_trace_ax_q<XA, YA>(L, lg_ndir, lg_t, lg_q, &hp, &hn);
                } else {
                    h = ltrace(L, ro, rd, &hp, &hn);
                }
                if (COUNT) ++c_ltest;
                if (is_iter) lmix += wl * lpdf(L, ro, h, hp, hn);
                if (h && (!has_li || longer(li_pos - ro, hp - ro))) {
                    has_li = true;
                    li_pos = hp;
                    li_pow = L.spow;
                }
            };
            auto light_step = [&](int l) {
                if constexpr (grid_lights(LMODE) && IPT_LIGHT_AX_REC) {
                    // the lattice light from its 48-byte record: exactly the
                    // fields light_trace_ax / light_pdf_ax read (ipt_path.h LightAx)
                    constexpr int XA = lattice_a10(LMODE) ? 1 : 0, YA = 1 - XA;
                    float4 a, b, c;
                    if (IPT_LTR_CALC && kp.ltr_calc) {
                        // the record's floats from the lattice's formulas; only
                        // the weight is per light
                        a = make_float4(kp.lc_x0 + (float)(l & ((1 << kp.lc_shift) - 1)) * kp.lc_dx,
                                        kp.lc_y0 + (float)(l >> kp.lc_shift) * kp.lc_dy, kp.lc_ax, kp.lc_ay);
                        b = make_float4(kp.lc_ix, kp.lc_iy, kp.lc_area, kp.lc_spow);
                        c = make_float4(kLaxLds ? lax_lds[3 * l + 2].x : kp.lax[3 * l + 2].x, 0.0f, 0.0f, 0.0f);
                    } else if constexpr (kLaxLds) {
                        a = lax_lds[3 * l]; b = lax_lds[3 * l + 1]; c = lax_lds[3 * l + 2];
                    } else {
                        const float4* r = kp.lax + 3 * l;
                        a = r[0]; b = r[1]; c = r[2];
                    }
                    LightDev L;
                    L.P = v3(a.x, a.y, kp.lg_pn);
                    L.x = XA == 0 ? v3(a.z, 0.0f, 0.0f) : v3(0.0f, a.z, 0.0f);
                    L.y = YA == 0 ? v3(a.w, 0.0f, 0.0f) : v3(0.0f, a.w, 0.0f);
                    L.n = v3(0.0f, 0.0f, kp.lg_nn);
                    L.inv.c[XA] = v3(b.x, 0.0f, 0.0f);
                    L.inv.c[YA] = v3(0.0f, b.y, 0.0f);
                    L.inv.c[2] = v3(0.0f, 0.0f, 0.0f);
                    L.area = b.z;
                    L.spow = b.w;
                    L.type = 0;
                    L.pad = 0;
                    light_step_with(L, c.x);
                } else {
                    light_step_with(LS.light(l), LS.weight(l));
                }
            };
            // the reference's event count: every light traced once for the
            // pdf (iterations) and once for traceRayToLight (depth < max)
            if (COUNT) c_ltr += (uint32_t)nl * ((is_iter ? 1u : 0u) + ((rdepth < kp.depth_max) ? 1u : 0u));
            if constexpr (grid_lights(LMODE)) {
                // the ray's point on the lights' plane and its cell(s): every
                // light whose exact test can pass lies in a cell within
                // kp.lg_e cells of that point (LightGrid::e, derived per
                // lattice by light_grid_build in ipt_path.h from the lattice's
                // tolerance and the rounding of u, v; as small as 2^-14 -- it
                // holds because the light tests below take the same plane
                // point q as this lookup), so the lights of those <= 4 cells,
                // in index order, are the scan's hits (a light that is not hit
                // adds +0 to lmix and is never nearest)
                constexpr int XA = lattice_a10(LMODE) ? 1 : 0, YA = 1 - XA;
                // (the lattice's ranges are proven like the single light's,
                // light_ranges_box: the range-free quotient of light_trace_ax,
                // shared with the light tests below)
                const float n_dir = kp.lg_nn * comp<2>(rd);
                const float num = kp.lg_nn * (kp.lg_pn - comp<2>(ro));
                const float t = IPT_LIGHT_INR ? div_inrange_(num, n_dir) : div_(num, n_dir);
                lg_ndir = n_dir;
                lg_t = t;
                lg_q = ro + rd * t;
                const float u = (comp<XA>(lg_q) - kp.lg_u0) * kp.lg_icw;
                const float v = (comp<YA>(lg_q) - kp.lg_v0) * kp.lg_ich;
                int cand[4] = {-1, -1, -1, -1};
                const float e = kp.lg_e;
                if (u > -1.0f && u < (float)kp.lg_nu + 1.0f && v > -1.0f && v < (float)kp.lg_nv + 1.0f) {
                    const int i0 = (int)floorf(u - e), i1 = (int)floorf(u + e);
                    const int j0 = (int)floorf(v - e), j1 = (int)floorf(v + e);
                    const int* cells = reinterpret_cast<const int*>(lnodes_lds);
                    auto cell = [&](int i, int j) {
                        const bool in = i >= 0 && i < kp.lg_nu && j >= 0 && j < kp.lg_nv;
                        if (IPT_LTR_CALC && kp.lg_ident)
                            return in ? (kp.lg_ident == 1 ? i + kp.lg_nu * j : j + kp.lg_nv * i) : -1;
                        return in ? cells[i + kp.lg_nu * j] : -1;
                    };
                    cand[0] = cell(i0, j0);
                    cand[1] = i1 != i0 ? cell(i1, j0) : -1;
                    cand[2] = j1 != j0 ? cell(i0, j1) : -1;
                    cand[3] = (i1 != i0 && j1 != j0) ? cell(i1, j1) : -1;
                }
                // ascending index order (-1 = none sorts last as 0xffffffff);
                // with the per-lattice margin a second candidate cell is rare
                // (C5: ~1 lookup in 8 000), so the sorting network runs only in
                // waves where some lane has one
                uint32_t c0 = (uint32_t)cand[0], c1 = (uint32_t)cand[1], c2 = (uint32_t)cand[2], c3 = (uint32_t)cand[3];
                auto cs = [](uint32_t& a, uint32_t& b) { const uint32_t lo = a < b ? a : b; b = a < b ? b : a; a = lo; };
                if (__builtin_expect(__any((c1 & c2 & c3) != 0xffffffffu), 0)) {
                    cs(c0, c1); cs(c2, c3); cs(c0, c2); cs(c1, c3); cs(c1, c2);
                }
                if (c0 != 0xffffffffu) light_step((int)c0);
                if (c1 != 0xffffffffu) light_step((int)c1);
                if (c2 != 0xffffffffu) light_step((int)c2);
                if (c3 != 0xffffffffu) light_step((int)c3);
            } else if (LMODE == kLightsGlobal && kp.n_light_nodes > 0) {
                // index-ordered light BVH (ipt_bvh.h): lights met in scan order;
                // a skipped light would add +0 to lmix and never be nearest
                const vec3 inv = v3(safe_rcp(rd.x), safe_rcp(rd.y), safe_rcp(rd.z));
                auto walk = [&](const BvhNode* __restrict__ lnodes) {
                int i = 0;
                // while-while: walk to the next entered leaf, then run the
                // leaf's light steps with every lane that stands on one
                while (i < kp.n_light_nodes) {
                    int leaf = -1;
                    while (i < kp.n_light_nodes) {
                        const BvhNode nd = lnodes[i];
                        if (COUNT) ++c_lnode;
                        const bool enter = bvh_box_entry(nd, ro, inv) != inf_();
                        if (enter && nd.leaf >= 0) {
                            leaf = nd.leaf;
                            i = nd.skip;
                            break;
                        }
                        i = enter ? i + 1 : nd.skip;
                    }
                    if (leaf >= 0) {
                        const int first = leaf & 0xffffff, cnt = leaf >> 24;
                        for (int l = first; l < first + cnt; ++l) light_step(l);
                    }
                }
                };
                if (kp.lnodes_lds)
                    walk(lnodes_lds);
                else
                    walk(kp.light_nodes);
            } else {
                for (int l = 0; l < nl; ++l) light_step(l);
            }
            IPT_STAMP_AT(9);  // light traces + pdf
            float mult = 0.0f;
            if (is_iter) {
                Frame fz;
                fz.iz = v3(frc[9 * kFrameStride], frc[10 * kFrameStride], frc[11 * kFrameStride]);
                const float sdf_val = frame_cosine_value(fz, rd);
                const float mix = lmix + w_sdf * sdf_val;
                mult = div_(sdf_val, mix);
            }
            // child ray_power (main.cpp:100-143): the geometry trace, then resolve
            if (kRes && rdepth < kp.depth_max && (kp.n_nodes > 0 || kp.n_grid > 0)) {
                // resumable walk: keep the ray and the light results, planes now
                xrd = rd;
                xis_iter = is_iter;
                xmult = mult;
                xhas_li = has_li;
                {
                    const vec3 eb = li_pos - ro;
                    xli_y = dot(eb, eb);
                }
                xli_pow = li_pow;
                int xp = -1;
                xi = 0;
                xbest = inf_();
                if (GEOM == IPT_GEOM_SPHERES_IN_BOX)
                    xbest = (IPT_BOXDIV && kp.box_inrange) ? trace_box_planes_only<true>(ro, rd, &xp)
                                                           : trace_box_planes_only<false>(ro, rd, &xp);
                xbidx = -2 - xp;
                if (kp.n_grid > 0) sphere_grid_init(kg, ro, rd, xi, xtm);
                tracing = true;
            } else {
                int prim = -1;
                float t = inf_();
                if (rdepth < kp.depth_max) {
                    IPT_PHASE(9);
                    t = trace_geometry<COUNT, GEOM>(kp, ro, rd, &prim, c_nodes, c_tests);
                    IPT_STAMP_AT(10);  // mixture value + geometry trace
                }
                const vec3 eb = li_pos - ro;
                resolve(rdepth < kp.depth_max, t, prim, ro, rd, rdepth, is_iter, mult, has_li, dot(eb, eb), li_pow);
            }
        }
        IPT_STAMP_AT(11);  // resolve + push
        // (kRes) the walking ray's origin: the lane's node or the camera
        const vec3 xo = xis_iter ? tpos : kp.cam_pos;
        if (kRes && IPT_GRID_WAVE && kp.n_grid > 0) {
            // the whole wave walks (the item tests are spread over its lanes)
            if (__ballot(tracing)) {
                if constexpr (IPT_GRID_WAVE == 2)
                    sphere_grid_walk_wave2<COUNT>(kg, tracing, xo, xrd, xi, xtm, xbest, xbidx, IPT_GRID_BUDGET,
                                                  wslots + (tid & ~63), wown + (tid & ~63), lane, c_nodes, c_tests);
                else
                    sphere_grid_walk_wave<COUNT>(kg, tracing, xo, xrd, xi, xtm, xbest, xbidx, IPT_GRID_BUDGET,
                                                 wslots + (tid & ~63), lane, grid_lds, c_nodes, c_tests IPT_DIAG_ARGS);
            }
            if (tracing && xi < 0) {
                tracing = false;
                if (IPT_GRID_WAVE != 2 && xbidx >= 0) xbidx = grid_item_index(kg, xbidx);  // item position -> original index
#if IPT_RAYLOG
                if (!COUNT && kp.raylog) {
                    const unsigned long long k = atomicAdd(kp.raylog_n, 1ull);
                    if (k % kp.raylog_every == 0 && k / kp.raylog_every < kp.raylog_cap) {
                        RayLogRec r;
                        r.o[0] = xo.x; r.o[1] = xo.y; r.o[2] = xo.z; r.t = xbest;
                        r.d[0] = xrd.x; r.d[1] = xrd.y; r.d[2] = xrd.z; r.hit = xbidx;
                        kp.raylog[k / kp.raylog_every] = r;
                    }
                }
#endif
                resolve(true, xbest, xbidx >= 0 ? 6 + xbidx : -2 - xbidx, xo, xrd, xis_iter ? tdepth + 1 : 0, xis_iter,
                        xmult, xhas_li, xli_y, xli_pow);
            }
        } else if (kRes && tracing) {
            IPT_PHASE(9);
            bool done;
            if (kp.n_grid > 0) {
                sphere_grid_walk<COUNT, IPT_GRID_PIPE != 0>(kg, xo, xrd, xi, xtm, xbest, xbidx, IPT_GRID_BUDGET, c_nodes,
                                                          c_tests IPT_DIAG_ARGS);
                done = xi < 0;
            } else {
                sphere_bvh_walk<COUNT>(kp, xo, xrd, xi, xbest, xbidx, IPT_WALK_BUDGET, c_nodes, c_tests);
                done = xi >= kp.n_nodes;
            }
            if (done) {
                tracing = false;
                if (IPT_GRID_PIPE && kp.n_grid > 0 && xbidx >= 0)
                    xbidx = grid_item_index(kg, xbidx);  // item position -> original index
                resolve(true, xbest, xbidx >= 0 ? 6 + xbidx : -2 - xbidx, xo, xrd, xis_iter ? tdepth + 1 : 0, xis_iter,
                        xmult, xhas_li, xli_y, xli_pow);
            }
        }
        }  // !kResL
        if constexpr (kPreSkip) {
            // The next iteration of the lane's node -- the same node's next one,
            // or the first of the child pushed in this step -- is a certain skip
            // when its pick word (read by the prologue: word jj+3) picks a light
            // and the node lies behind the lights' plane (the prologue's
            // skip-ahead argument). It does nothing but consume its three draws
            // and count (main.cpp:149-163), so it is taken here: a node whose
            // last iteration it was is then done and popped below in this step
            // (instead of a step of its own for the skip). Same draws in the
            // same order, same counts.
            // (as selects: no exec-mask branch)
            const bool back = (tpos.z - kp.sa_pz) * kp.sa_nz < 0.0f;
            const bool lpick = IPT_PICK_INT ? (unsigned long long)pre_w < kp.sa_u : u01(pre_w) < kp.sa_cl;
            const bool take = iter_lane && pre_ok && back && ti < (kp.n_rays >> tdepth) && lpick;
            ti += take ? 1 : 0;
            k += take ? 3u : 0u;
            if (COUNT) {
                c_iter += take ? 1u : 0u;
                c_lsamp += take ? 1u : 0u;
                c_skip += take ? 1u : 0u;
            }
        }
        if constexpr (kFramePf == 3) {
            pop_node();
            IPT_STAMP_AT(6);  // pop (end of step)
            if constexpr (IPT_FRAME_TAB && kFrameInrange) {
                // the frame the lane builds in the next step (a sphere node
                // pushed in this step, or popped back to with its column
                // overwritten): `to` and the table gather now, consumed there
                if (need_frame && active && has_path) {
                    const vec3 to = normalize_inrange_(tpos);
                    const uint32_t u = f2u(to.z), mz = u & 0x7fffffffu;
                    pfok = mz - kFrameTabLo <= kFrameTabSpan;
                    if (pfok) {
                        const float2 e = kp.frame_sc[((mz - kFrameTabLo) << 1) | (u >> 31)];
                        pfs = e.x;
                        pfc = e.y;
                        pto = to;
                    }
                    if constexpr (IPT_FRAME_FB_PF) {
                        // the out-of-table angle computed here as well, so that
                        // the frame phase reads `to`, sin a, cos a unconditionally
                        if (__builtin_expect(__any(!pfok), 0))
                            if (!pfok) {
                                frame_angle_sc(to, &pfs, &pfc);
                                pto = to;
                            }
                    }
                }
            }
            IPT_STAMP_AT(7);  // next frame's `to` + table gather
        }
    }

    IPT_DIAG_FLUSH(kp.counters, kNumCounters)
    if (COUNT) {
        atomicAdd(&kp.counters[0], (unsigned long long)c_paths);
        atomicAdd(&kp.counters[1], (unsigned long long)c_traced);
        atomicAdd(&kp.counters[2], (unsigned long long)c_surf);
        atomicAdd(&kp.counters[3], (unsigned long long)c_light);
        atomicAdd(&kp.counters[4], (unsigned long long)c_exp);
        atomicAdd(&kp.counters[5], (unsigned long long)c_iter);
        atomicAdd(&kp.counters[6], (unsigned long long)c_lsamp);
        atomicAdd(&kp.counters[7], (unsigned long long)c_skip);
        atomicAdd(&kp.counters[8], (unsigned long long)c_sframe);
        atomicAdd(&kp.counters[9], (unsigned long long)c_ltr);
        atomicAdd(&kp.counters[10], (unsigned long long)c_drift);
        atomicAdd(&kp.counters[11], (unsigned long long)c_nodes);
        atomicAdd(&kp.counters[12], (unsigned long long)c_tests);
        atomicAdd(&kp.counters[13], (unsigned long long)c_lnode);
        atomicAdd(&kp.counters[14], (unsigned long long)c_ltest);
    }
}

struct AParams {
    int W, H, spp, n_cand;
    const int* cand_of_row;  // [H] candidate index or -1
    const float* values;
    const uint8_t* codes;
    const uint8_t* flags;
    int tile_rows, n_shards, shard_id;
    float* pixels;
    uint32_t* counters;
    float* sums;
    float* pixel_max;
    // [2]: the launch's first block start and last block end on the 100 MHz
    // wall clock (atomic min / max; the host presets them), for its duration
    unsigned long long* clk;
};

__device__ __forceinline__ void add_ray(float v, float& p, uint32_t& c, float& s, float& m) {
    // GridRenderPlane::addRay (GridRenderPlane.cpp:68-73)
    p = (p * (float)c + v) / (float)(c + 1u);
    ++c;
    s += v;
    if (p > m) m = p;
}

__device__ __forceinline__ void accumulate_pixel(const AParams& ap, int xi, int yi);
__global__ __launch_bounds__(256) void accumulate_kernel(AParams ap) {
    const int xi = blockIdx.x * blockDim.x + threadIdx.x;
    const int yi = blockIdx.y;
    if (threadIdx.x == 0) atomicMin(&ap.clk[0], (unsigned long long)wall_clock64());
    if (xi < ap.W && (ap.n_shards <= 1 || ap.tile_rows <= 0 || ((yi / ap.tile_rows) % ap.n_shards) == ap.shard_id))
        accumulate_pixel(ap, xi, yi);
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&ap.clk[1], (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void accumulate_pixel(const AParams& ap, int xi, int yi) {
    const size_t d = (size_t)yi * ap.W + xi;
    float p = ap.pixels[d];
    uint32_t c = ap.counters[d];
    float s = ap.sums ? ap.sums[d] : 0.0f;
    float m = ap.pixel_max ? ap.pixel_max[d] : 0.0f;
    const size_t pass_stride = (size_t)ap.n_cand * ap.W;
    const int H = ap.H;
    if (ap.flags[d] == 0) {
        // nominal sources only: source row H-2-yi (and H-1 for yi == 0)
        int r0 = H - 2 - yi;
        const int c0 = r0 >= 0 ? ap.cand_of_row[r0] : -1;
        const int c1 = (yi == 0 && H >= 1) ? ap.cand_of_row[H - 1] : -1;
        // the samples' loads issued 8 passes at a time, then the 8 running-mean
        // updates in the same order: one load latency per 8 passes instead of
        // one per pass (the updates are a serial chain per pixel)
        const bool t0 = c0 >= 0, t1 = c1 >= 0 && c1 != c0;
        const float* v0p = ap.values + (size_t)(t0 ? c0 : 0) * ap.W + xi;
        const float* v1p = ap.values + (size_t)(t1 ? c1 : 0) * ap.W + xi;
        int sp = 0;
        for (; sp + 8 <= ap.spp; sp += 8) {
            float a0[8], a1[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const size_t base = (size_t)(sp + q) * pass_stride;
                a0[q] = t0 ? v0p[base] : 0.0f;
                a1[q] = t1 ? v1p[base] : 0.0f;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (t0) add_ray(a0[q], p, c, s, m);
                if (t1) add_ray(a1[q], p, c, s, m);
            }
        }
        for (; sp < ap.spp; ++sp) {
            const size_t base = (size_t)sp * pass_stride;
            if (t0) add_ray(v0p[base], p, c, s, m);
            if (t1) add_ray(v1p[base], p, c, s, m);
        }
    } else {
        int rows[4];
        int nr = 0;
        const int cand_rows[4] = {H - 3 - yi, H - 2 - yi, H - 1 - yi, yi <= 1 ? H - 1 : -1};
        for (int q = 0; q < 4; ++q) {
            const int r = cand_rows[q];
            if (r < 0 || r >= H) continue;
            bool dup = false;
            for (int e = 0; e < nr; ++e) dup |= rows[e] == r;
            if (!dup) rows[nr++] = r;
        }
        // ascending row order (raster order of render_sample)
        for (int a = 0; a < nr; ++a)
            for (int b2 = a + 1; b2 < nr; ++b2)
                if (rows[b2] < rows[a]) { int t = rows[a]; rows[a] = rows[b2]; rows[b2] = t; }
        for (int sp = 0; sp < ap.spp; ++sp) {
            const size_t base = (size_t)sp * pass_stride;
            for (int a = 0; a < nr; ++a) {
                const int iy = rows[a];
                const int ci = ap.cand_of_row[iy];
                if (ci < 0) continue;
                const int yn = H - 2 - iy > 0 ? H - 2 - iy : 0;
                for (int ix = xi - 1; ix <= xi + 1; ++ix) {
                    if (ix < 0 || ix >= ap.W) continue;
                    const size_t idx = base + (size_t)ci * ap.W + ix;
                    const uint8_t code = ap.codes[idx];
                    if (code >= 0x10) continue;
                    const int dx = (code & 3) - 1, dy = ((code >> 2) & 3) - 1;
                    if (ix + dx == xi && yn + dy == yi) add_ray(ap.values[idx], p, c, s, m);
                }
            }
        }
    }
    ap.pixels[d] = p;
    ap.counters[d] = c;
    if (ap.sums) ap.sums[d] = s;
    if (ap.pixel_max) ap.pixel_max[d] = m;
}

// ----------------------------------------------------------- math probes
// Division pairs for the fast-division proof (fn 9): every 32-bit pattern b
// maps to a numerator with b's sign and mantissa and a biased exponent in
// [87, 167] (or +-0 when b's exponent field is 0) and a hashed denominator in
// the same range, so every wave of the self-check takes div_'s fast path.
__device__ __host__ inline float div_pair_a(uint32_t b) {
    const uint32_t e = (b >> 23) & 0xffu;
    if (e == 0u) return u2f(b & 0x80000000u);
    return u2f((b & 0x807fffffu) | ((87u + e % 81u) << 23));
}
__device__ __host__ inline float div_pair_b(uint32_t b) {
    uint32_t h = b * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    return u2f((h & 0x807fffffu) | ((87u + ((h >> 23) & 0xffu) % 81u) << 23));
}

// fn 20: divisors whose significands are all ones or within 2^12 ulps of it
// (the hard case of one-correction division), hashed exponents as above
__device__ __host__ inline float div_pair_b_ones(uint32_t b) {
    uint32_t h = b * 0x85EBCA77u;
    h ^= h >> 13;
    const uint32_t m = 0x007fffffu - (h & 0xfffu);
    return u2f((h & 0x80000000u) | ((87u + ((h >> 12) & 0xffu) % 81u) << 23) | m);
}

// fn 11 / 12 probes: a 32-bit pattern b seeds a pair.
//  11: x = |b| as a float, y = x moved by a hashed -64..63 ulps (every 16th
//      pair: an unrelated hashed float) -> longer_sq(x, y) as 0/1;
//  12: n = b, d = a hashed divisor of hashed magnitude -> udiv_exact(n, d).
__device__ __host__ inline uint32_t probe_hash(uint32_t b) {
    uint32_t h = b * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    return h;
}
__device__ __host__ inline void longer_pair(uint32_t b, float* x, float* y) {
    const uint32_t h = probe_hash(b);
    const uint32_t xb = b & 0x7fffffffu;
    *x = u2f(xb);
    *y = (h & 15u) == 0u ? u2f(probe_hash(h) & 0x7fffffffu) : u2f(xb + ((h >> 4) & 127u) - 64u);
}
__device__ __host__ inline uint32_t udiv_pair_d(uint32_t b) {
    const uint32_t h = probe_hash(b ^ 0x5bd1e995u);
    return (h >> (h & 31u)) | 1u;
}
__device__ __host__ inline float math_fn(int fn, float x) {
    switch (fn) {
        case 10: return div_inrange_(div_pair_a(f2u(x)), div_pair_b(f2u(x)));
        case 11: {
            float a, b;
            longer_pair(f2u(x), &a, &b);
#if defined(__HIP_DEVICE_COMPILE__)
            return longer_sq(a, b) ? 1.0f : 0.0f;
#else
            return sqrt_(a) > sqrt_(b) ? 1.0f : 0.0f;
#endif
        }
        case 12: {
            const uint32_t d = udiv_pair_d(f2u(x));
            return u2f(udiv_exact(f2u(x), d, 1.0 / (double)d));
        }
        case 13:  // the range-free root on its range +0, [2^-96, 2^126); sqrtf elsewhere
            return (f2u(x) == 0u || (x >= 0x1p-96f && x < 0x1p126f)) ? sqrt_inrange_(x) : sqrt_(x);
        case 14:
        case 15: {  // the RotateDdf angle's sin / cos for to.z = x
            float sv, cv;
            frame_angle_sc(v3(0.6f, 0.8f, x), &sv, &cv);
            return fn == 14 ? sv : cv;
        }
        case 17: return rcp_newton_<1>(x);
        case 18: return rcp_newton_<2>(x);
        case 19: return div_inrange_(div_pair_a(f2u(x)), div_pair_b(f2u(x)));
        case 20: return div_inrange_(div_pair_a(f2u(x)), div_pair_b_ones(f2u(x)));
        case 0: return acosf_(x);
        case 1: return sinf_(x);
        case 2: return cosf_(x);
        case 3: return acos_f64_to_f32(x);
        case 4: { float s, c; sincosf_(x, &s, &c); return s; }
        case 5: { float s, c; sincosf_(x, &s, &c); return c; }
        case 6: return sqrt_(x);
        case 7: return div_pi_to_f32(x);
        case 8: return two_pi_times(x);
        case 9: return div_(div_pair_a(f2u(x)), div_pair_b(f2u(x)));
        default: return 0.0f;
    }
}
// Philox blocks for the known-answer tests (ipt_philox): the key arrives as
// kernel arguments, i.e. uniform, as in the path kernel
__global__ void philox_kernel(uint32_t k0, uint32_t k1, const uint4* __restrict__ ctr, uint4* __restrict__ out,
                              long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 c = ctr[i];
    const u32x4 o = philox4x32_10(c.x, c.y, c.z, c.w, k0, k1);
    out[i] = make_uint4(o.v[0], o.v[1], o.v[2], o.v[3]);
}
__global__ void math_kernel(int fn, const float* in, float* out, long long n) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = math_fn(fn, in[i]);
}

// DDF samplers / values exactly as the path kernel evaluates them, for the
// sampler checks (ipt_ddf_sample / ipt_ddf_value; tests/test_ddf_samplers.py).
// kind 0: RotateDdf(CosineDdf, to=params[0..2]); kind 1: DdfFromLight of light
// params[3] at origin params[0..2]; kind 2: the UnionDdf of every light and
// RotateDdf(CosineDdf, normal=params[3..5]) at origin params[0..2].
__global__ void ddf_kernel(int value_mode, int kind, const float* __restrict__ params, const LightDev* __restrict__ lights,
                           const float* __restrict__ weights, const float* __restrict__ cdf, int nl,
                           const float* __restrict__ in, long long n, float* __restrict__ out,
                           const float* __restrict__ cos_a, const float2* __restrict__ cos_b) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const vec3 o = v3(params[0], params[1], params[2]);
    if (kind == 3) kind = value_mode ? 0 : kind;  // table sampler: same DDF value
    if (!value_mode) {
        const float pick = in[3 * i], u1 = in[3 * i + 1], u2 = in[3 * i + 2];
        vec3 v = v3(0.0f, 0.0f, 0.0f);
        if (kind == 0) {
            v = frame_apply(make_frame(o), cosine_sample_local(u1, u2));
        } else if (kind == 3) {
            // the path kernel's table lookup (u on the RNG's 2^-24 grid, checked by the caller)
            const float tr = cos_a[(uint32_t)(u1 * 16777216.0f)];
            const float2 tb = cos_b[(uint32_t)(u2 * 16777216.0f)];
            v = frame_apply(make_frame(o), v3(tr * tb.x, tr * tb.y, sqrt_(u1)));
        } else if (kind == 1) {
            v = light_sample_dir(lights[(int)params[3]], o, u1, u2);
        } else {
            int c = 0;
            while (c <= nl && !(pick < cdf[c])) ++c;
            if (c < nl) v = light_sample_dir(lights[c], o, u1, u2);
            else if (c == nl) v = frame_apply(make_frame(v3(params[3], params[4], params[5])), cosine_sample_local(u1, u2));
        }
        out[3 * i] = v.x;
        out[3 * i + 1] = v.y;
        out[3 * i + 2] = v.z;
    } else {
        const vec3 d = v3(in[3 * i], in[3 * i + 1], in[3 * i + 2]);
        float v;
        if (kind == 0) {
            v = frame_cosine_value(make_frame(o), d);
        } else if (kind == 1) {
            const LightDev& L = lights[(int)params[3]];
            vec3 hp, hn;
            const bool h = light_trace(L, o, d, &hp, &hn);
            v = light_pdf(L, o, h, hp, hn);
        } else {
            float lmix = 0.0f;
            for (int l = 0; l < nl; ++l) {
                vec3 hp, hn;
                const bool h = light_trace(lights[l], o, d, &hp, &hn);
                lmix += weights[l] * light_pdf(lights[l], o, h, hp, hn);
            }
            v = lmix + weights[nl] * frame_cosine_value(make_frame(v3(params[3], params[4], params[5])), d);
        }
        out[i] = v;
    }
}

// Exact CosineDdf tables (ddf.cpp:223-231) over the 2^24 values a draw can
// take (u = i * 2^-24, ipt_math.h u01): a[i] = sinf(acosf(sqrtf(u))) (64 MiB),
// b[i] = sincosf((float)(2*M_PI*u)) as (cos, sin) (128 MiB).
// cosine_sample_local(u1, u2) == (a[i1]*b[i2].x, a[i1]*b[i2].y, sqrtf(u1)) bit
// for bit (same functions, same products).
__global__ void cos_table_kernel(float* __restrict__ a, float2* __restrict__ b) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (1u << 24)) return;
    const float u = u01(i << 8);
    const float cos_alpha = sqrt_(u);
    const float r = sinf_small_(acosf_(cos_alpha));
    float sp, cp;
    sincosf_small_(two_pi_times(u), &sp, &cp);
    a[i] = r;
    b[i] = make_float2(cp, sp);
}

// frame_sc table (frame_sc_lookup): entry i is frame_angle_sc of to.z = the
// float with |bits| = kFrameTabLo + (i >> 1) and sign i & 1 (dot((0,0,1), to)
// is to.z for finite to.x, to.y and to.z != 0).
__global__ void frame_table_kernel(float2* __restrict__ t) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kFrameTabEntries) return;
    const float z = u2f((kFrameTabLo + (uint32_t)(i >> 1)) | ((uint32_t)(i & 1) << 31));
    float sv, cv;
    frame_angle_sc(v3(0.0f, 0.0f, z), &sv, &cv);
    t[i] = make_float2(sv, cv);
}

// Exact restatement of math_fn (differs only where the device uses a fast
// path, i.e. fn 3): the reference for ipt_math_selfcheck.
__device__ float math_fn_exact(int fn, float x) {
    if (fn == 3) return acos_f64_to_f32_exact(x);
    if (fn == 6) return __builtin_sqrtf(x);                                      // IEEE (compiler sequence)
    if (fn == 9 || fn == 10) return div_pair_a(f2u(x)) / div_pair_b(f2u(x));   // IEEE (compiler sequence)
    if (fn == 11) {
        float a, b;
        longer_pair(f2u(x), &a, &b);
        return sqrt_(a) > sqrt_(b) ? 1.0f : 0.0f;  // glm length comparison as written
    }
    if (fn == 12) return u2f(f2u(x) / udiv_pair_d(f2u(x)));
    if (fn == 13) return __builtin_sqrtf(x);  // IEEE (compiler sequence)
    if (fn == 17 || fn == 18) {  // the round-4 reciprocal: one Newton step, two quotient residual steps
        float y = __builtin_amdgcn_rcpf(x);
        y = __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
        const float q1 = __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
        return __builtin_fmaf(__builtin_fmaf(-x, q1, 1.0f), y, q1);
    }
    if (fn == 19) return div_pair_a(f2u(x)) / div_pair_b(f2u(x));       // IEEE (compiler sequence)
    if (fn == 20) return div_pair_a(f2u(x)) / div_pair_b_ones(f2u(x));  // IEEE (compiler sequence)
    return math_fn(fn, x);
}

// Self-check 16: a sphere-in-box-like normal from the bit pattern b (hashed
// coordinates with |nrm| around 0.5, plus the edge cases the fast frame must
// hand to the exact build: zero or tiny x / y, both tiny, z = +-1 directions,
// x = +-y) -> to = normalize(nrm); true when the fast frame says ok and any of
// its 12 floats differs from make_frame_sc<true>'s bits.
__device__ bool frame_fast_mismatch(uint32_t b) {
    const uint32_t h1 = probe_hash(b), h2 = probe_hash(h1 ^ 0x9e3779b9u), h3 = probe_hash(h2 + 0x7f4a7c15u);
    float x = (float)(int)(h1 >> 8) * 0x1p-24f - 0.5f;  // [-0.5, 0.5)
    float y = (float)(int)(h2 >> 8) * 0x1p-24f - 0.5f;
    float z = (float)(int)(h3 >> 8) * 0x1p-24f - 0.5f;
    switch (b & 15u) {
        case 0: x = 0.0f; break;
        case 1: y = 0.0f; break;
        case 2: x = u2f(h1 & 0x0fffffffu) * (h2 & 1 ? 1.0f : -1.0f); break;           // tiny x
        case 3: x = u2f(h1 & 0x0fffffffu); y = -u2f(h2 & 0x0fffffffu); break;        // tiny x and y
        case 4: x = -0.0f; y = u2f(h3 & 0x1fffffffu); break;
        case 5: y = x; break;
        case 6: y = -x; break;
        case 7: x = u2f(h1 & 0x33ffffffu); y = u2f(h2 & 0x33ffffffu); break;         // |x|, |y| ~ 1e-7
        default: break;
    }
    if (!(z != 0.0f)) z = 0.25f;
    const vec3 to = normalize_inrange_(v3(x, y, z));
    float s, c;
    frame_angle_sc(to, &s, &c);
    bool ok;
    const Frame f = make_frame_sc_fast(to, s, c, ok);
    if (!ok) return false;
    const Frame e = make_frame_sc<true>(to, s, c);
    const float* pf = &f.m0.x;
    const float* pe = &e.m0.x;
    bool diff = false;
    for (int k = 0; k < 12; ++k) diff |= f2u(pf[k]) != f2u(pe[k]);
    return diff;
}

// fn 21: the range-free division over EVERY pair of significands, a and b in
// [1, 2) (index i: a = 1 + (i >> 23) 2^-23, b = 1 + (i & (2^23 - 1)) 2^-23,
// 2^46 pairs), against IEEE a/b. With fn 22 (the reciprocal scales exactly)
// this extends to every in-range operand: the remaining operations (the
// Newton fma, a*y, the residual fma, the correction fma) are IEEE operations
// and commute with scaling by powers of two while nothing over- or
// underflows, which the callers' range [2^-40, 2^41) guarantees; RN is
// symmetric, so signs follow too. Mismatches counted; `first` = the lowest a
// significand index (i >> 23) with one.
__global__ void divcheck_kernel(unsigned long long lo, unsigned long long n, unsigned long long* bad,
                                unsigned int* first) {
    unsigned long long local = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned long long k = lo + i;
        const float a = u2f(0x3f800000u | (uint32_t)(k >> 23));
        const float b = u2f(0x3f800000u | (uint32_t)(k & 0x7fffffu));
        float bv = b;
        asm volatile("" : "+v"(bv));  // no constant folding of the IEEE sequence
        if (f2u(div_inrange_(a, bv)) != f2u(a / bv)) {
            ++local;
            atomicMin(first, (unsigned int)(k >> 23));
        }
    }
    if (local) atomicAdd(bad, local);
}
// fn 22: the reciprocal scales exactly: for every float b with |b| in
// [2^-40, 2^41), rcp_newton_<1>(b) == sign(b) 2^-e rcp_newton_<1>(m) for b =
// sign(b) m 2^e, m in [1, 2) (other patterns: not counted)
__device__ bool rcp_scale_mismatch(uint32_t bb) {
    const uint32_t e = (bb >> 23) & 0xffu;
    if (e < 127u - 40u || e >= 127u + 41u) return false;
    const float b = u2f(bb);
    const float m = u2f(0x3f800000u | (bb & 0x7fffffu));
    const float ym = rcp_newton_<1>(m);
    const float want = __builtin_amdgcn_ldexpf(ym, 127 - (int)e);
    const float y = rcp_newton_<1>(b);
    return f2u(y) != (f2u(want) ^ (bb & 0x80000000u));
}

__global__ void selfcheck_kernel(int fn, unsigned long long lo, unsigned long long n,
                                 unsigned long long* bad, unsigned int* first, const float2* __restrict__ ftab) {
    unsigned long long local = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t b = (uint32_t)(lo + i);
        const float x = u2f(b);
        if (fn == 16 || fn == 22) {  // 16: make_frame_sc_fast == make_frame_sc<true> wherever it reports ok
            if (fn == 16 ? frame_fast_mismatch(b) : rcp_scale_mismatch(b)) {
                ++local;
                atomicMin(first, b);
            }
            continue;
        }
        float a = math_fn(fn, x);
        const float e = math_fn_exact(fn, x);
        if (fn == 14 || fn == 15) {  // the path kernel's table lookup (frame_sc_lookup)
            float sv = 0.0f, cv = 0.0f;
            frame_sc_lookup(ftab, v3(0.6f, 0.8f, x), sv, cv);
            a = fn == 14 ? sv : cv;
        }
        // fn 10 / 19 / 20: a zero quotient's sign is not observed by the callers
        if (!(f2u(a) == f2u(e) || (a != a && e != e) || ((fn == 10 || fn >= 19) && a == 0.0f && e == 0.0f))) {
            ++local;
            atomicMin(first, b);
        }
    }
    if (local) atomicAdd(bad, local);
}

// ---------------------------------------------------------------- context
std::mutex g_err_mu;
std::string g_err_global;

}  // namespace

// One set of per-launch work buffers (radiance, drift codes, raygen records,
// drifted-pixel flags, the shard's candidate rows, the work-unit counter) with
// its own stream for raygen + path kernel. Consecutive launches -- chunks of
// one call and consecutive calls alike -- alternate between two slots, so a
// launch's workgroups take the CUs its predecessor's tail leaves idle (lanes
// out of paths while the longest trees finish); the
// GridRenderPlane replays run on the caller's stream in call order, each after
// its own path kernel (an event), so the image is accumulated exactly as by
// sequential calls.
struct WorkSlot {
    float* d_values = nullptr;
    uint8_t* d_codes = nullptr;
    uint4* d_rg = nullptr;  // raygen_kernel records, 2 x 16 B per element
    size_t work_cap = 0;    // elements
    uint8_t* d_flags = nullptr;
    size_t flags_cap = 0;
    int* d_cand_rows = nullptr;
    int* d_cand_of_row = nullptr;
    int cand_cap_rows = 0, cand_cap_h = 0;
    int plan[4] = {-1, -1, -1, -1};  // (H, tile_rows, n_shards, shard_id) whose rows are on the device
    unsigned long long* d_unit = nullptr;
    // pool-drained flag in signal memory (hipExtMallocWithFlags(hipMallocSignalMemory),
    // the memory hipStreamWaitValue64 is specified for) and the sequence
    // number of the slot's last queued launch (the value it stores there)
    unsigned long long* d_drained = nullptr;
    unsigned long long seq = 0;
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;  // after the last reader of the slot's buffers (accumulate or host copies)
    hipEvent_t path_end = nullptr;  // after its last path kernel
    unsigned long long total = 0;   // work units of its last launch
    bool used = false;
    bool idle = true;  // its last launch is known complete (a drain since): nothing to wait for
};
#if IPT_RAYLOG
// IPT_RAYLOG's buffer (scripts/probes/walk_split.hip arms it)
static RayLogRec* g_raylog = nullptr;
static unsigned long long* g_raylog_n = nullptr;
static unsigned long long g_raylog_cap = 0;
static unsigned g_raylog_every = 1;
#endif

struct ChunkTiming {
    hipEvent_t t0 = nullptr, t1 = nullptr;  // raygen start, path-kernel end (slot stream)
    hipEvent_t a0 = nullptr, a1 = nullptr;  // accumulate (caller stream; null without an image)
    int clk = -1;           // the accumulate's wall-clock pair in ctx->d_clk (ring entry)
    bool recorded = false;  // every event of the launch was recorded (its queueing succeeded)
};
constexpr int kClkRing = 32;  // > the launches settle_oldest lets queue up (8) plus the last settled one

// ipt_render's device-resident GridRenderPlane: the caller's host image is
// the truth, the device keeps a copy of its OWNED rows (all rows unsharded,
// the shard's tiles otherwise) across calls, and a host shadow holds those
// rows as the previous call returned them. A call uploads only the owned row
// runs whose host bytes differ from the shadow (none when the caller left the
// plane alone between calls, e.g. progressive rendering), renders, and
// downloads only the owned rows: 16 B per owned pixel per call (pixels,
// counters, and sums / per-pixel max when the image has them) instead of the
// whole plane both ways.
struct ResidentPlane {
    int W = 0, H = 0;
    bool has_sums = false, has_pmax = false;
    int plan[3] = {-1, -1, -1};  // (tile_rows, n_shards, shard_id) of `runs`
    float* d_pixels = nullptr;
    uint32_t* d_counters = nullptr;
    float* d_sums = nullptr;
    float* d_pmax = nullptr;
    std::vector<std::pair<int, int>> runs;  // owned rows [y0, y1)
    size_t owned_px = 0;
    std::vector<uint8_t> shadow;  // per field, the owned runs' bytes as last returned
    bool shadow_ok = false;
    unsigned long long h2d = 0, d2h = 0;  // bytes moved by the last ipt_render
};

struct ipt_ctx {
    int device = 0;
    ResidentPlane rp;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    std::string err;
    bool has_scene = false;
    int geometry_kind = 0;
    int n_lights = 0;
    LightDev* d_lights = nullptr;
    float* d_weights = nullptr;
    float* d_cdf = nullptr;
    Frame* d_wall = nullptr;
    float4* d_spheres = nullptr;
    int n_spheres = 0;
    BvhNode* d_bvh_nodes = nullptr;
    BvhSphere* d_bvh_prims = nullptr;
    int n_nodes = 0;
    float bvh_tmargin = 0.0f;  // sphere BVH pruning margin (ipt_bvh.h)
    SphereGrid grid;           // geometry of the uniform sphere grid (host copy)
    int n_grid = 0;
    size_t grid_n_items = 0;
    int* d_grid_start = nullptr;
    int* d_grid_packed = nullptr;  // IPT_GRID_LDS (KParams::grid_packed)
    int grid_packed_words = 0, grid_packed_nb = 0;
    BvhSphere* d_grid_items = nullptr;
    float4* d_grid_c4 = nullptr;  // [items] centre/radius, then [items] original indices
    GridCell* d_grid_cells = nullptr;  // 64-byte cell records (IPT_GRID_INLINE)
    BvhNode* d_light_nodes = nullptr;
    int n_light_nodes = 0;
    int cdf_bsearch = 0;
    int cdf_p2 = 0, cdf_p2e = 0;
    int lpf_calc = 0, lc_shift = 0;  // KParams::lpf_calc
    int ltr_calc = 0, lg_ident = 0;  // KParams::ltr_calc, lg_ident
    float lc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float cdf_p2s = 0.0f, cdf_end = 0.0f;
    int* d_cdf_lo = nullptr;  // cdf bucket starts (global light modes), null when a bucket is crowded
    bool any_round_light = false;
    int light_axis = 0;  // axis_aligned_light() of a single AreaLight (kLightsOneA10/A01)
    LightGrid lgrid;     // lgrid.pattern != 0: coplanar light lattice (kLightsGridA10/A01)
    unsigned long long pk_u0 = 0, pk_u1 = 0, sa_u = 0;  // word thresholds (KParams)
    int sa_on = 0;       // the lights' sample points share the plane z = sa_pz, normal (0, 0, sa_nz) (skip-ahead)
    float sa_pz = 0.0f, sa_nz = 0.0f, sa_cl = 0.0f;
    int* d_lgrid = nullptr;
    LightAx* d_lax = nullptr;  // lattice lights' compact records (IPT_LIGHT_AX_REC)
    int bpc_override = 0;
    int lnodes_lds = 1;  // stage the light BVH in LDS (IPT_LNODES_LDS=0: global memory)
    int light_grid_on = 1;  // coplanar light lattices by cell lookup (IPT_LIGHT_GRID=0: the light BVH)
    vec3 cam_pos, cam_dir, cam_right, cam_up;
    int box_inrange = 0;
    // work buffers: two slots, used by consecutive launches in turn (WorkSlot)
    WorkSlot slot[2];
    unsigned next_slot = 0;
    // a launch starts once its predecessor's work pool is drained (its unit
    // counter reached its total: hipStreamWaitValue64 on that counter, in
    // device memory); without stream value waits (or IPT_NO_TAIL_OVERLAP=1)
    // once the predecessor has finished (an event)
    bool gate_on_pool = false;
    size_t chunk_cap_test = 0;  // IPT_TEST_CHUNK_UNITS: at most this many units per launch (tests)
    // timing of the launches queued since the last drain (event sets from ev_pool)
    std::vector<ChunkTiming> pending;
    ChunkTiming prev{};  // the last processed launch (its path-end event bounds the next one's start)
    std::vector<hipEvent_t> ev_pool;
    float run_path_ms = 0.0f, run_acc_ms = 0.0f;
    // accumulate_kernel's start / end wall-clock stamps, a ring of kClkRing
    // pairs (HIP events on the caller's stream are stamped when its wait for
    // the path kernel is queued, not when it is released)
    unsigned long long* d_clk = nullptr;
    unsigned long long* d_clk_dummy = nullptr;  // (2 words: stamps of an untimed launch)
    unsigned next_clk = 0;
    double clk_khz = 100000.0;
    unsigned long long* d_counters = nullptr;
    float* d_cos_a = nullptr;   // CosineDdf tables (cos_table_kernel): r 64 MiB,
                                // (cos phi, sin phi) 128 MiB
    float2* d_cos_b = nullptr;
    float2* d_frame_sc = nullptr;  // frame_table_kernel (IPT_FRAME_TAB), 1 GiB
    float last_path_ms = 0.0f, last_acc_ms = 0.0f;
    int blocks_per_cu = 0;      // of the last path-kernel launch
    bool lattice_lds = true;    // IPT_LATTICE_LDS=0: the lattice instances with global records (tests)
    size_t max_lds = 160 * 1024;  // the device's LDS per workgroup (hipDeviceAttributeMaxSharedMemoryPerBlock)
};

namespace {

int fail(ipt_ctx* ctx, int code, const std::string& msg) {
    if (ctx) {
        ctx->err = msg;
    } else {
        std::lock_guard<std::mutex> g(g_err_mu);
        g_err_global = msg;
    }
    return code;
}
#define HIPCHECK(ctx, expr)                                                             \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(ctx, e_ == hipErrorOutOfMemory ? IPT_E_OOM : IPT_E_DEVICE,      \
                        std::string(#expr) + ": " + hipGetErrorString(e_));             \
    } while (0)

using ipt_internal::DevBuf;

// The exact sampling tables are built once per context. Each is published in
// the context only after its allocation, its build kernel and that kernel's
// completion all succeeded, so a failure leaves no half-built table behind.
int ensure_cos_tables(ipt_ctx* ctx, hipStream_t st) {
    if (ctx->d_cos_a && ctx->d_cos_b) return IPT_OK;
    const size_t n = (size_t)1 << 24;
    DevBuf<float> a;
    DevBuf<float2> b;
    HIPCHECK(ctx, hipMalloc(&a.p, n * sizeof(float)));
    HIPCHECK(ctx, hipMalloc(&b.p, n * sizeof(float2)));
    hipLaunchKernelGGL(cos_table_kernel, dim3((unsigned)(n / 256)), dim3(256), 0, st, a.p, b.p);
    HIPCHECK(ctx, hipGetLastError());
    HIPCHECK(ctx, hipStreamSynchronize(st));
    ctx->d_cos_a = a.release();
    ctx->d_cos_b = b.release();
    return IPT_OK;
}

// the geometries whose sphere-node frames read the frame-angle table
constexpr bool frame_table_user(int geom) {
    return geom == IPT_GEOM_SPHERE_IN_BOX || (IPT_FRAME_TAB_LISTS && geom == IPT_GEOM_SPHERES_IN_BOX);
}
int ensure_frame_table(ipt_ctx* ctx, hipStream_t st) {
    if (!IPT_FRAME_TAB || ctx->d_frame_sc) return IPT_OK;
    DevBuf<float2> t;
    HIPCHECK(ctx, hipMalloc(&t.p, kFrameTabEntries * sizeof(float2)));
    hipLaunchKernelGGL(frame_table_kernel, dim3((unsigned)((kFrameTabEntries + 255) / 256)), dim3(256), 0, st, t.p);
    HIPCHECK(ctx, hipGetLastError());
    HIPCHECK(ctx, hipStreamSynchronize(st));
    ctx->d_frame_sc = t.release();
    return IPT_OK;
}

// Work buffers grow on demand. A buffer's capacity is dropped to 0 together
// with the buffer, so a failed regrowth never leaves a stale capacity over a
// null pointer.
int ensure_work(ipt_ctx* ctx, WorkSlot& S, size_t elems, size_t npix, int H, int n_cand) {
    // (the caller has waited for the slot's previous launch and its readers)
    if (elems > S.work_cap) {
        if (S.d_values) hipFree(S.d_values);
        if (S.d_codes) hipFree(S.d_codes);
        if (S.d_rg) hipFree(S.d_rg);
        S.d_values = nullptr;
        S.d_codes = nullptr;
        S.d_rg = nullptr;
        S.work_cap = 0;
        DevBuf<float> v;
        DevBuf<uint8_t> c;
        DevBuf<uint4> g;
        HIPCHECK(ctx, hipMalloc(&v.p, elems * sizeof(float)));
        HIPCHECK(ctx, hipMalloc(&c.p, elems));
        if (IPT_RAYGEN) HIPCHECK(ctx, hipMalloc(&g.p, elems * 2 * sizeof(uint4)));
        S.d_values = v.release();
        S.d_codes = c.release();
        S.d_rg = g.release();
        S.work_cap = elems;
    }
    if (npix > S.flags_cap) {
        if (S.d_flags) hipFree(S.d_flags);
        S.d_flags = nullptr;
        S.flags_cap = 0;
        HIPCHECK(ctx, hipMalloc(&S.d_flags, npix));
        S.flags_cap = npix;
    }
    if (n_cand > S.cand_cap_rows || H > S.cand_cap_h) {
        if (S.d_cand_rows) hipFree(S.d_cand_rows);
        if (S.d_cand_of_row) hipFree(S.d_cand_of_row);
        S.d_cand_rows = nullptr;
        S.d_cand_of_row = nullptr;
        S.cand_cap_rows = S.cand_cap_h = 0;
        S.plan[0] = -1;
        DevBuf<int> r, o;
        HIPCHECK(ctx, hipMalloc(&r.p, sizeof(int) * std::max(n_cand, 1)));
        HIPCHECK(ctx, hipMalloc(&o.p, sizeof(int) * std::max(H, 1)));
        S.d_cand_rows = r.release();
        S.d_cand_of_row = o.release();
        S.cand_cap_rows = n_cand;
        S.cand_cap_h = H;
    }
    return IPT_OK;
}

hipEvent_t pool_event(ipt_ctx* ctx) {
    if (!ctx->ev_pool.empty()) {
        hipEvent_t e = ctx->ev_pool.back();
        ctx->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
void pool_return(ipt_ctx* ctx, ChunkTiming& c) {
    for (hipEvent_t e : {c.t0, c.t1, c.a0, c.a1})
        if (e) ctx->ev_pool.push_back(e);
    c = ChunkTiming{};
}

// Adds the oldest pending launch's times to the running sums (waiting for
// it): its path time counts from its own start or from its predecessor's end,
// whichever is later, so overlapped launches sum to their span; then the
// accumulate kernel's time.
// A launch whose queueing failed part-way (`recorded` false: its end events
// were never recorded) is dropped without timing: its events go back to the
// pool and the caller keeps the error message of the failure itself.
int settle_oldest(ipt_ctx* ctx) {
    ChunkTiming c = ctx->pending.front();
    ctx->pending.erase(ctx->pending.begin());
    if (!c.recorded) {
        pool_return(ctx, c);
        return IPT_OK;
    }
    const hipError_t e = hipEventSynchronize(c.a1 ? c.a1 : c.t1);
    float path = 0.0f, d = 0.0f, acc = 0.0f;
    if (e != hipSuccess || hipEventElapsedTime(&path, c.t0, c.t1) != hipSuccess ||
        (c.a1 && hipEventElapsedTime(&acc, c.a0, c.a1) != hipSuccess)) {
        pool_return(ctx, c);
        return fail(ctx, IPT_E_DEVICE, std::string("render launch failed: ") + hipGetErrorString(e != hipSuccess ? e : hipGetLastError()));
    }
    // the accumulate kernel's own duration from its wall-clock stamps (the
    // events bracket the caller stream's wait for the path kernel as well)
    if (c.a1 && c.clk >= 0 && ctx->d_clk) {
        unsigned long long h[2] = {~0ull, 0ull};
        if (hipMemcpy(h, ctx->d_clk + 2 * c.clk, sizeof h, hipMemcpyDeviceToHost) == hipSuccess && h[0] != ~0ull &&
            h[1] >= h[0])
            acc = (float)((double)(h[1] - h[0]) / ctx->clk_khz);
    }
    if (ctx->prev.t1 && hipEventElapsedTime(&d, c.t0, ctx->prev.t1) == hipSuccess && d > 0.0f)
        path = std::max(0.0f, path - d);
    ctx->run_path_ms += path;
    ctx->run_acc_ms += acc;
    pool_return(ctx, ctx->prev);
    ctx->prev = c;
    return IPT_OK;
}

// Waits for every queued launch and its readers; the launches' times since
// the previous drain become ipt_last_kernel_ms's.
int drain(ipt_ctx* ctx) {
    int rc = IPT_OK;
    for (WorkSlot& S : ctx->slot) {
        if (S.st && hipStreamSynchronize(S.st) != hipSuccess) rc = fail(ctx, IPT_E_DEVICE, "slot stream failed");
        if (S.used && S.done && hipEventSynchronize(S.done) != hipSuccess) rc = fail(ctx, IPT_E_DEVICE, "slot readers failed");
        S.idle = true;  // (synchronous calls therefore queue no stream value waits)
    }
    while (!ctx->pending.empty()) {
        const int r = settle_oldest(ctx);
        if (r && !rc) rc = r;
    }
    pool_return(ctx, ctx->prev);
    if (ctx->run_path_ms > 0.0f || ctx->run_acc_ms > 0.0f) {
        ctx->last_path_ms = ctx->run_path_ms;
        ctx->last_acc_ms = ctx->run_acc_ms;
    }
    ctx->run_path_ms = ctx->run_acc_ms = 0.0f;
    return rc;
}

bool owned_host(const ipt_params* p, int yi) {
    if (p->n_shards <= 1 || p->tile_rows <= 0) return true;
    return ((yi / p->tile_rows) % p->n_shards) == p->shard_id;
}

// Source rows whose samples can land in an owned destination row:
// nominal row H-2-iy (0 for iy=H-1) within +-1 of an owned row.
void candidate_rows(const ipt_params* p, std::vector<int>& rows, std::vector<int>& of_row) {
    const int H = p->height;
    rows.clear();
    of_row.assign(H, -1);
    for (int iy = 0; iy < H; ++iy) {
        const int yn = H - 2 - iy > 0 ? H - 2 - iy : 0;
        bool c = false;
        for (int dy = -1; dy <= 1; ++dy) {
            const int y = yn + dy;
            if (y >= 0 && y < H && owned_host(p, y)) c = true;
        }
        if (c) {
            of_row[iy] = (int)rows.size();
            rows.push_back(iy);
        }
    }
}

// The draw word w's u01(w) = (w >> 8) 2^-24 is below c exactly when w >> 8 <
// T = ceil(c 2^24) (both sides exact: an integer against c scaled by a power
// of two), i.e. when w < T << 8: T = 0 for c <= 0 or NaN (never), 2^24 for
// c >= 1 (always, as a 64-bit bound).
unsigned long long word_threshold(float c) {
    const double x = (double)c * 16777216.0;
    if (!(x > 0.0)) return 0ull;
    if (x >= 16777216.0) return 1ull << 32;
    return (unsigned long long)std::ceil(x) << 8;
}

int needed_susp(const ipt_params* p);
int validate(ipt_ctx* ctx, const ipt_params* p) {
    if (!ctx) return IPT_E_INVALID;
    if (!p) return fail(ctx, IPT_E_INVALID, "params is NULL");
    if (!ctx->has_scene) return fail(ctx, IPT_E_NOSCENE, "no scene uploaded");
    if (p->width <= 0 || p->height <= 0 || p->width > 65536 || p->height > 65536)
        return fail(ctx, IPT_E_INVALID, "width/height out of range");
    if ((int64_t)p->width * p->height > (int64_t)1 << 31)
        return fail(ctx, IPT_E_INVALID, "frame larger than 2^31 pixels");
    if (p->spp < 0 || p->spp_offset < 0) return fail(ctx, IPT_E_INVALID, "negative spp");
    // a suspended level stores its iteration count in the low bits of its meta
    // word (ti | kind << s, ti <= n_rays): s = 8 for n_rays < 256, else 16,
    // which leaves 16 bits for the node kind (6 + sphere index)
    if (p->n_rays < 0 || p->n_rays > 65535) return fail(ctx, IPT_E_UNSUPPORTED, "n_rays must be in [0,65535]");
    if (p->n_rays > 255 && ctx->n_spheres > 65535 - 6)
        return fail(ctx, IPT_E_UNSUPPORTED, "n_rays > 255 with more than 65529 spheres");
    if (p->depth_max < 0 || p->depth_max > 64) return fail(ctx, IPT_E_INVALID, "depth_max out of range");
    // the deepest pushed node: n_rays < 256 bounds it by 7 (a node at depth d
    // has n_rays >> d children) whatever depth_max; larger n_rays need
    // depth_max <= 9 (the MAXSUSP = 8 instances)
    if (needed_susp(p) > 8)
        return fail(ctx, IPT_E_UNSUPPORTED, "n_rays > 255 with depth_max > 9: more than 8 suspended levels");
    if (p->n_shards > 1 && (p->shard_id < 0 || p->shard_id >= p->n_shards))
        return fail(ctx, IPT_E_INVALID, "shard_id out of range");
    return IPT_OK;
}

// Number of suspended stack levels the DFS can need.
int needed_susp(const ipt_params* p) {
    // a node at depth d is pushed iff d < depth_max and (n_rays >> d) > 0
    int maxpush = -1;
    for (int d = 0; d < p->depth_max; ++d)
        if ((p->n_rays >> d) > 0) maxpush = d;
    return maxpush < 0 ? 0 : maxpush;  // suspended levels = depth of deepest pushed node
}

// dynamic LDS bytes of a path-kernel instance (the layout at the top of path_kernel)
template <int MAXSUSP, int LMODE, int GEOM>
size_t path_lds_bytes(const KParams& kp) {
    constexpr int kBlock = block_of(LMODE, GEOM);
    const size_t cells = (size_t)kp.lg_nu * kp.lg_nv;
    return ((size_t)MAXSUSP * kStackFields * kBlock + scene_lds_words(LMODE, GEOM) +
            ((IPT_GRID_LDS && resumable_geom(GEOM)) ? (size_t)kp.grid_packed_words : 0) +
            (LMODE == kLightsGlobal ? global_light_lds_words(kp.n_lights, kp.lnodes_lds ? kp.n_light_nodes : 0) : 0) +
            (grid_lights(LMODE) ? global_light_lds_words(kp.n_lights, 0, true) +
                                      (lax_in_lds(LMODE) ? ((cells + 3) & ~(size_t)3) + 12 * (size_t)kp.n_lights : cells)
                                : 0)) *
           sizeof(float);
}

template <int MAXSUSP, bool COUNT, int LMODE, int GEOM>
int launch_path4(ipt_ctx* ctx, const KParams& kp, hipStream_t st) {
    constexpr int kBlock = block_of(LMODE, GEOM);
    if (IPT_GRID_LDS && resumable_geom(GEOM) && kp.n_grid > 0 && !kp.grid_packed)
        return fail(ctx, IPT_E_UNSUPPORTED, "IPT_GRID_LDS build: the grid's ranges do not pack into bytes");
    const size_t lds = path_lds_bytes<MAXSUSP, LMODE, GEOM>(kp);
    const void* fn = (const void*)path_kernel<MAXSUSP, COUNT, LMODE, GEOM>;
    HIPCHECK(ctx, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    // persistent grid: every block the CUs can hold at once (a work queue, no
    // inter-block waits, so an over-reported residency only queues blocks)
    int bpc = 0;
    HIPCHECK(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, fn, kBlock, lds));
    bpc = std::max(1, std::min(bpc, 2048 / kBlock));  // (at most 32 waves per CU)
    if (ctx->bpc_override > 0) bpc = std::min(bpc, ctx->bpc_override);  // IPT_BLOCKS_PER_CU (profiling)
    ctx->blocks_per_cu = bpc;
    dim3 grid(ctx->n_cu * bpc), block(kBlock);
    hipLaunchKernelGGL((path_kernel<MAXSUSP, COUNT, LMODE, GEOM>), grid, block, lds, st, kp);
    HIPCHECK(ctx, hipGetLastError());
    return IPT_OK;
}
// -DIPT_AB_BUILD -DIPT_C2_ONLY=1: experiment builds (scripts/variants.sh)
// instantiate the sample_scenes[0] kernel alone (ipt_knobs.h).
template <int MAXSUSP, bool COUNT, int LMODE>
int launch_path3(ipt_ctx* ctx, const KParams& kp, hipStream_t st) {
    if constexpr (IPT_C2_ONLY != 0) {
        if (MAXSUSP != 4 || LMODE != IPT_C2_LMODE || kp.geometry_kind != IPT_GEOM_SPHERE_IN_BOX)
            return fail(ctx, IPT_E_UNSUPPORTED, "IPT_C2_ONLY experiment build");
        return launch_path4<4, COUNT, IPT_C2_LMODE, IPT_GEOM_SPHERE_IN_BOX>(ctx, kp, st);
    } else {
    switch (kp.geometry_kind) {
        case IPT_GEOM_SPHERES_IN_BOX: return launch_path4<MAXSUSP, COUNT, LMODE, IPT_GEOM_SPHERES_IN_BOX>(ctx, kp, st);
        case IPT_GEOM_FLOOR: return launch_path4<MAXSUSP, COUNT, LMODE, IPT_GEOM_FLOOR>(ctx, kp, st);
        case IPT_GEOM_CORNER: return launch_path4<MAXSUSP, COUNT, LMODE, IPT_GEOM_CORNER>(ctx, kp, st);
        case IPT_GEOM_SPHERES: return launch_path4<MAXSUSP, COUNT, LMODE, IPT_GEOM_SPHERES>(ctx, kp, st);
        case IPT_GEOM_SMALLPT: return launch_path4<MAXSUSP, COUNT, LMODE, IPT_GEOM_SMALLPT>(ctx, kp, st);
        default: return launch_path4<MAXSUSP, COUNT, LMODE, IPT_GEOM_SPHERE_IN_BOX>(ctx, kp, st);
    }
    }
}
template <int MAXSUSP, bool COUNT>
int launch_path2(ipt_ctx* ctx, const KParams& kp, hipStream_t st) {
    if (ctx->any_round_light) return launch_path3<MAXSUSP, COUNT, kLightsAny>(ctx, kp, st);
    if (kp.n_lights == 1) {
        if (ctx->light_axis == 1) return launch_path3<MAXSUSP, COUNT, kLightsOneA10>(ctx, kp, st);
        if (ctx->light_axis == 2) return launch_path3<MAXSUSP, COUNT, kLightsOneA01>(ctx, kp, st);
        return launch_path3<MAXSUSP, COUNT, kLightsOne>(ctx, kp, st);
    }
    if (kp.n_lights <= kLdsLights) return launch_path3<MAXSUSP, COUNT, kLightsLds>(ctx, kp, st);
    if constexpr (IPT_C2_ONLY == 0) {
        // (the lattice is only built for sphere-in-box scenes)
        // the records-in-LDS instance wherever its LDS fits one workgroup per CU
        constexpr int G = IPT_GEOM_SPHERE_IN_BOX;
        if (ctx->lgrid.pattern == 1 && kp.geometry_kind == G) {
            if (IPT_LAX_LDS && ctx->lattice_lds && path_lds_bytes<MAXSUSP, kLightsGridA10L, G>(kp) <= ctx->max_lds)
                return launch_path4<MAXSUSP, COUNT, kLightsGridA10L, G>(ctx, kp, st);
            return launch_path4<MAXSUSP, COUNT, kLightsGridA10, G>(ctx, kp, st);
        }
        if (ctx->lgrid.pattern == 2 && kp.geometry_kind == G) {
            if (IPT_LAX_LDS && ctx->lattice_lds && path_lds_bytes<MAXSUSP, kLightsGridA01L, G>(kp) <= ctx->max_lds)
                return launch_path4<MAXSUSP, COUNT, kLightsGridA01L, G>(ctx, kp, st);
            return launch_path4<MAXSUSP, COUNT, kLightsGridA01, G>(ctx, kp, st);
        }
    }
    return launch_path3<MAXSUSP, COUNT, kLightsGlobal>(ctx, kp, st);
}
template <int MAXSUSP>
int launch_path(ipt_ctx* ctx, const KParams& kp, hipStream_t st, bool count) {
    return count ? launch_path2<MAXSUSP, true>(ctx, kp, st) : launch_path2<MAXSUSP, false>(ctx, kp, st);
}

int render_chunks(ipt_ctx* ctx, const ipt_params* p, ipt_image* img, hipStream_t st,
                  float* host_values, uint8_t* host_codes) {
    std::vector<int> rows, of_row;
    candidate_rows(p, rows, of_row);
    const int n_cand = (int)rows.size();
    const int W = p->width, H = p->height;
    const size_t per_pass = (size_t)n_cand * W;
    if (per_pass == 0 || p->spp == 0) return IPT_OK;
    // chunk passes so that the work buffers stay bounded: at most 2^29 units
    // (37 B each: 2 GiB of radiance + 512 MiB of codes + 16 GiB of raygen
    // records, of 288 GB), and at most 3/4 of the device memory this context
    // can still obtain (hipMemGetInfo's free memory plus its own work buffers,
    // less the sampling tables not yet built), so that contexts sharing a
    // device split their passes into more launches instead of failing with
    // IPT_E_OOM. Equal chunks: each launch ends with a tail in which lanes run
    // out of work (the longest paths finish alone; 7 % of a 32-spp C2 launch),
    // so few large launches beat many small ones (C2 1024^2 x 256 spp is a
    // single launch).
    constexpr size_t kUnitBytes = sizeof(float) + 1 + (IPT_RAYGEN ? 2 * sizeof(uint4) : 0);
    size_t budget = (size_t)1 << 29;
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            size_t avail = free_b + (ctx->slot[0].work_cap + ctx->slot[1].work_cap) * kUnitBytes;
            const size_t tables = (ctx->d_cos_a ? 0 : ((size_t)3 << 26)) +
                                  (ctx->d_frame_sc || !frame_table_user(ctx->geometry_kind)
                                       ? 0 : kFrameTabEntries * sizeof(float2));
            avail = avail > tables ? avail - tables : 0;
            // (two slots: consecutive launches hold a chunk each)
            budget = std::min(budget, std::max<size_t>(per_pass, avail / 8 * 3 / kUnitBytes));
        }
    }
    if (ctx->chunk_cap_test) budget = std::min(budget, std::max<size_t>(per_pass, ctx->chunk_cap_test));
    const size_t n_chunks = std::max<size_t>(1, ((size_t)p->spp * per_pass + budget - 1) / budget);
    int chunk = (int)std::max<size_t>(1, ((size_t)p->spp + n_chunks - 1) / n_chunks);
    while (chunk > 1 && (size_t)chunk * per_pass > budget) --chunk;
    int rc = ensure_cos_tables(ctx, st);
    if (rc) return rc;
    if (frame_table_user(ctx->geometry_kind)) {  // path_kernel's frame builds
        rc = ensure_frame_table(ctx, st);
        if (rc) return rc;
    }
    const int susp = needed_susp(p);  // <= 8 (validate)
    const bool count = (p->flags & IPT_FLAG_COUNTERS) != 0;
    for (int s0 = 0; s0 < p->spp; s0 += chunk) {
        const int ns = std::min(chunk, p->spp - s0);
        // this launch's slot; its previous launch and that launch's readers
        // (accumulate, host copies) must be done before its buffers are
        // regrown or rewritten: the slot stream waits for them on the device,
        // the host only where it rewrites device memory itself
        WorkSlot& S = ctx->slot[ctx->next_slot];
        ctx->next_slot ^= 1u;
        const bool grow = (size_t)chunk * per_pass > S.work_cap || (size_t)W * H > S.flags_cap ||
                          n_cand > S.cand_cap_rows || H > S.cand_cap_h;
        const int plan[4] = {H, p->tile_rows, p->n_shards, p->shard_id};
        const bool replan = !std::equal(plan, plan + 4, S.plan);
        if (S.used && (grow || replan)) HIPCHECK(ctx, hipEventSynchronize(S.done));
        rc = ensure_work(ctx, S, (size_t)chunk * per_pass, (size_t)W * H, H, n_cand);
        if (rc) return rc;
        if (replan) {
            // (synchronous copies: the host vectors do not outlive the call)
            HIPCHECK(ctx, hipMemcpy(S.d_cand_rows, rows.data(), sizeof(int) * n_cand, hipMemcpyHostToDevice));
            HIPCHECK(ctx, hipMemcpy(S.d_cand_of_row, of_row.data(), sizeof(int) * H, hipMemcpyHostToDevice));
            std::copy(plan, plan + 4, S.plan);
        }
        if (S.used) HIPCHECK(ctx, hipStreamWaitEvent(S.st, S.done, 0));
        // start in the predecessor's tail: once its pool is drained (or, without
        // stream value waits, once it has finished)
        const unsigned sidx = (unsigned)(&S - ctx->slot);
        WorkSlot& P = ctx->slot[sidx ^ 1u];
        // (P's counter is reset only by P's next launch, which waits for this
        // launch's pool in turn, so this wait cannot miss its value)
        if (P.used && !P.idle) {
            if (ctx->gate_on_pool)
                HIPCHECK(ctx, hipStreamWaitValue64(S.st, P.d_drained, P.seq, hipStreamWaitValueGte, ~0ull));
            else
                HIPCHECK(ctx, hipStreamWaitEvent(S.st, P.path_end, 0));
        }
        // bounded timing backlog: settle launches far behind (they are done or
        // nearly so; the queue of launches ahead is untouched)
        while (ctx->pending.size() >= 8) {
            rc = settle_oldest(ctx);
            if (rc) return rc;
        }
        ChunkTiming tm;
        tm.t0 = pool_event(ctx);
        tm.t1 = pool_event(ctx);
        if (img) {
            tm.a0 = pool_event(ctx);
            tm.a1 = pool_event(ctx);
        }
        if (!tm.t0 || !tm.t1 || (img && (!tm.a0 || !tm.a1))) {
            pool_return(ctx, tm);
            return fail(ctx, IPT_E_DEVICE, "hipEventCreate failed");
        }
        KParams kp{};
        kp.W = W;
        kp.H = H;
        kp.spp = ns;
        kp.spp_offset = p->spp_offset + s0;
        kp.n_rays = p->n_rays;
        kp.meta_shift = p->n_rays > 255 ? 16 : 8;
        kp.depth_max = p->depth_max;
        kp.key0 = (uint32_t)p->seed;
        kp.key1 = (uint32_t)(p->seed >> 32);
        kp.n_cand = n_cand;
        kp.cand_rows = S.d_cand_rows;
        kp.tile_rows = p->tile_rows;
        kp.n_shards = p->n_shards;
        kp.shard_id = p->shard_id;
        kp.total_units = (unsigned long long)ns * per_pass;
        if (kp.total_units >= (1ull << 32)) return fail(ctx, IPT_E_INVALID, "more than 2^32 work units in one launch");
        kp.per_pass32 = (uint32_t)per_pass;
        kp.box_inrange = ctx->box_inrange;
        kp.inv_per_pass = 1.0 / (double)per_pass;
        kp.inv_w = 1.0 / (double)W;
        kp.unit_counter = S.d_unit;
        kp.drained = ctx->gate_on_pool ? S.d_drained : nullptr;
#if IPT_RAYLOG
        kp.raylog = g_raylog;
        kp.raylog_n = g_raylog_n;
        kp.raylog_cap = g_raylog_cap;
        kp.raylog_every = g_raylog_every;
#endif
        kp.drain_seq = S.seq + 1;
        kp.values = S.d_values;
        kp.codes = S.d_codes;
        kp.flags = S.d_flags;
        kp.counters = ctx->d_counters;
        kp.geometry_kind = ctx->geometry_kind;
        kp.n_lights = ctx->n_lights;
        kp.lights = ctx->d_lights;
        kp.weights = ctx->d_weights;
        kp.cdf = ctx->d_cdf;
        kp.wall_frames = ctx->d_wall;
        kp.cam_pos = ctx->cam_pos;
        kp.cam_dir = ctx->cam_dir;
        kp.cam_right = ctx->cam_right;
        kp.cam_up = ctx->cam_up;
        kp.n_spheres = ctx->n_spheres;
        kp.spheres = ctx->d_spheres;
        kp.bvh_nodes = ctx->d_bvh_nodes;
        kp.bvh_tmargin = ctx->bvh_tmargin;
        kp.n_grid = ctx->n_grid;
        for (int a = 0; a < 3; ++a) {
            kp.grid_g0[a] = ctx->grid.g0[a];
            kp.grid_h[a] = ctx->grid.h[a];
            kp.grid_inv_h[a] = ctx->grid.inv_h[a];
            kp.grid_n[a] = ctx->grid.n[a];
            kp.grid_g1[a] = ctx->grid.g0[a] + (float)ctx->grid.n[a] * ctx->grid.h[a];
        }
        kp.grid_m = ctx->grid.m;
        kp.grid_start = ctx->d_grid_start;
        kp.grid_packed = ctx->d_grid_packed;
        kp.grid_packed_words = ctx->grid_packed_words;
        kp.grid_packed_nb = ctx->grid_packed_nb;
        kp.grid_items = ctx->d_grid_items;
        kp.grid_c4 = ctx->d_grid_c4;
        kp.grid_idx = ctx->d_grid_c4 ? reinterpret_cast<const int*>(ctx->d_grid_c4 + ctx->grid_n_items) : nullptr;
        kp.grid_cells = ctx->d_grid_cells;
        kp.bvh_prims = ctx->d_bvh_prims;
        kp.n_nodes = ctx->n_nodes;
        kp.light_nodes = ctx->d_light_nodes;
        kp.n_light_nodes = ctx->n_light_nodes;
        // light BVH staged in LDS (IPT_LNODES_LDS=0 at ipt_create keeps it in
        // global memory): the resumable light walk runs at 3 workgroups/CU, which
        // the extra LDS keeps, and gains 10 % on C5 (43.8 vs 40.2 Mpaths/s)
        kp.lnodes_lds = (ctx->lnodes_lds && ctx->n_light_nodes > 0 && ctx->n_light_nodes <= kLdsLightNodesMax) ? 1 : 0;
        kp.cdf_bsearch = ctx->cdf_bsearch;
        kp.cdf_p2 = ctx->cdf_p2;
        kp.cdf_p2s = ctx->cdf_p2s;
        kp.cdf_end = ctx->cdf_end;
        kp.cdf_p2e = ctx->cdf_p2e;
        kp.lpf_calc = ctx->lpf_calc;
        kp.lc_shift = ctx->lc_shift;
        kp.lc_x0 = ctx->lc[0];
        kp.lc_y0 = ctx->lc[1];
        kp.lc_dx = ctx->lc[2];
        kp.lc_dy = ctx->lc[3];
        kp.lc_ax = ctx->lc[4];
        kp.lc_ay = ctx->lc[5];
        kp.ltr_calc = ctx->ltr_calc;
        kp.lg_ident = ctx->lg_ident;
        kp.lc_ix = ctx->lc[6];
        kp.lc_iy = ctx->lc[7];
        kp.lc_area = ctx->lc[8];
        kp.lc_spow = ctx->lc[9];
        kp.cdf_end_t = (uint32_t)(word_threshold(ctx->cdf_end) >> 8);
        kp.cdf_lo = ctx->d_cdf_lo;
        kp.lgrid = ctx->d_lgrid;
        kp.lax = reinterpret_cast<const float4*>(ctx->d_lax);
        kp.lg_nu = ctx->lgrid.nu;
        kp.lg_nv = ctx->lgrid.nv;
        kp.lg_u0 = ctx->lgrid.u0;
        kp.lg_v0 = ctx->lgrid.v0;
        kp.lg_icw = ctx->lgrid.icw;
        kp.lg_ich = ctx->lgrid.ich;
        kp.lg_e = ctx->lgrid.e;
        kp.pk_u0 = ctx->pk_u0;
        kp.pk_u1 = ctx->pk_u1;
        kp.sa_u = ctx->sa_u;
        kp.sa_on = ctx->sa_on;
        kp.sa_pz = ctx->sa_pz;
        kp.sa_nz = ctx->sa_nz;
        kp.sa_cl = ctx->sa_cl;
        kp.lg_pn = ctx->lgrid.pn;
        kp.lg_nn = ctx->lgrid.nn;
        kp.cos_a = ctx->d_cos_a;
        kp.cos_b = ctx->d_cos_b;
        kp.frame_sc = ctx->d_frame_sc;
        kp.rg = S.d_rg;
        kp.count = count ? 1 : 0;
        // the slot stream: t0..t1 is the path's per-sample work, raygen_kernel
        // (render_sample's jitter, camera ray, Philox block 0; ~0.2 % of a C2
        // launch) and path_kernel
        const hipStream_t ss = S.st;
        ctx->pending.push_back(tm);  // (settled by drain, also on an error below: unrecorded, untimed)
        ChunkTiming& tmq = ctx->pending.back();
        S.used = true;
        S.idle = false;
        S.total = 0;  // (until its kernel is queued: a successor must not wait on a launch that failed)
        HIPCHECK(ctx, hipMemsetAsync(S.d_unit, 0, sizeof(unsigned long long), ss));
        HIPCHECK(ctx, hipMemsetAsync(S.d_flags, 0, (size_t)W * H, ss));
        HIPCHECK(ctx, hipEventRecord(tm.t0, ss));
        if (IPT_RAYGEN) {
            hipLaunchKernelGGL(raygen_kernel, dim3((unsigned)((kp.total_units + 255) / 256)), dim3(256), 0, ss, kp);
            HIPCHECK(ctx, hipGetLastError());
        }
        rc = susp <= 4 ? launch_path<4>(ctx, kp, ss, count) : launch_path<8>(ctx, kp, ss, count);
        if (rc) return rc;
        S.total = kp.total_units;
        S.seq = kp.drain_seq;
        HIPCHECK(ctx, hipEventRecord(tm.t1, ss));
        HIPCHECK(ctx, hipEventRecord(S.path_end, ss));
        if (host_values) {  // [spp][H][W] (whole frames: per_pass == W * H)
            HIPCHECK(ctx, hipMemcpyAsync(host_values + (size_t)s0 * per_pass, S.d_values, sizeof(float) * ns * per_pass,
                                         hipMemcpyDeviceToHost, ss));
            HIPCHECK(ctx, hipMemcpyAsync(host_codes + (size_t)s0 * per_pass, S.d_codes, ns * per_pass,
                                         hipMemcpyDeviceToHost, ss));
        }
        if (!img) HIPCHECK(ctx, hipEventRecord(S.done, ss));
        if (img) {
            // the GridRenderPlane replay: on the caller's stream, in call order,
            // after this launch's path kernel
            HIPCHECK(ctx, hipStreamWaitEvent(st, tm.t1, 0));
            HIPCHECK(ctx, hipEventRecord(tm.a0, st));
            unsigned long long* clk = nullptr;
            if (ctx->d_clk) {
                tmq.clk = (int)(ctx->next_clk++ % kClkRing);
                clk = ctx->d_clk + 2 * tmq.clk;
                HIPCHECK(ctx, hipMemsetAsync(clk, 0xff, sizeof(unsigned long long), st));
                HIPCHECK(ctx, hipMemsetAsync(clk + 1, 0, sizeof(unsigned long long), st));
            }
            AParams ap{};
            ap.W = W;
            ap.H = H;
            ap.spp = ns;
            ap.n_cand = n_cand;
            ap.cand_of_row = S.d_cand_of_row;
            ap.values = S.d_values;
            ap.codes = S.d_codes;
            ap.flags = S.d_flags;
            ap.tile_rows = p->tile_rows;
            ap.n_shards = p->n_shards;
            ap.shard_id = p->shard_id;
            ap.pixels = img->pixels;
            ap.counters = img->counters;
            ap.sums = img->sums;
            ap.pixel_max = img->pixel_max;
            ap.clk = clk ? clk : ctx->d_clk_dummy;
            dim3 grid((W + 255) / 256, H), block(256);
            hipLaunchKernelGGL(accumulate_kernel, grid, block, 0, st, ap);
            HIPCHECK(ctx, hipGetLastError());
            HIPCHECK(ctx, hipEventRecord(tm.a1, st));
            HIPCHECK(ctx, hipEventRecord(S.done, st));
        }
        tmq.recorded = true;
    }
    return IPT_OK;
}

}  // namespace

// Hooks for the library's other translation units (ipt_internal.h).
namespace ipt_internal {
int ctx_fail(ipt_ctx* ctx, int code, const std::string& msg) { return fail(ctx, code, msg); }
hipStream_t ctx_stream(ipt_ctx* ctx) { return ctx->stream; }
int ctx_device(ipt_ctx* ctx) { return ctx->device; }
int ctx_cus(ipt_ctx* ctx) { return ctx->n_cu; }
}  // namespace ipt_internal

extern "C" {

int ipt_abi_version(void) { return IPT_ABI_VERSION; }

const char* ipt_last_error(ipt_ctx* ctx) {
    if (ctx) return ctx->err.c_str();
    std::lock_guard<std::mutex> g(g_err_mu);
    return g_err_global.c_str();
}

int ipt_create(int hip_device, ipt_ctx** out) {
    if (!out) return fail(nullptr, IPT_E_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(nullptr, IPT_E_DEVICE, "no HIP device available (the path tracer has no CPU fallback)");
    if (hip_device < 0 || hip_device >= n) return fail(nullptr, IPT_E_INVALID, "bad device index");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, hip_device) != hipSuccess)
        return fail(nullptr, IPT_E_DEVICE, "hipGetDeviceProperties failed");
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
        return fail(nullptr, IPT_E_DEVICE, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950 only");
    ipt_ctx* ctx = new ipt_ctx();
    ctx->device = hip_device;
    ctx->n_cu = prop.multiProcessorCount;
    {
        // the records-in-LDS lattice instances are chosen against the device's
        // own limit (160 KiB on gfx950), so a smaller one falls back to the
        // global-record instances instead of failing the launch
        // (the larger of the per-block limit and its opt-in value)
        int lds = 0, optin = 0;
        if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, hip_device) != hipSuccess) lds = 0;
        if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, hip_device) != hipSuccess) optin = 0;
        if (std::max(lds, optin) > 0) ctx->max_lds = (size_t)std::max(lds, optin);
        (void)hipGetLastError();  // an unsupported attribute must not leave a sticky error behind
    }
    if (const char* e = std::getenv("IPT_BLOCKS_PER_CU")) ctx->bpc_override = std::atoi(e);  // profiling only
    if (const char* e = std::getenv("IPT_LNODES_LDS")) ctx->lnodes_lds = std::atoi(e) != 0;
    if (const char* e = std::getenv("IPT_LIGHT_GRID")) ctx->light_grid_on = std::atoi(e) != 0;
    if (const char* e = std::getenv("IPT_LATTICE_LDS")) ctx->lattice_lds = std::atoi(e) != 0;
    if (hipSetDevice(hip_device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return fail(nullptr, IPT_E_DEVICE, "stream creation failed");
    }
    if (const char* e = std::getenv("IPT_TEST_CHUNK_UNITS")) ctx->chunk_cap_test = (size_t)std::atoll(e);  // tests
    {
        // (round 4 measured hipStreamWaitValue64 on hipMalloc memory releasing
        // the waiting stream ~0.6 us after a kernel's atomicAdd reached the
        // value, scripts/probes/waitvalue_probe.hip; since round 6 the wait is
        // on a signal-memory flag, the memory the API specifies). A tool that serialises the
        // dispatches to collect counters or traces (rocprofv3 --pmc / --att,
        // which export ROCPROF_COUNTER_COLLECTION / ROCPROF_ADVANCED_THREAD_TRACE
        // to the profiled process) never released such a wait queued behind a
        // serialised dispatch, and the wait has no timeout: then
        // every launch is gated on its predecessor's path-end event instead
        // (the same images; consecutive launches lose their tail overlap).
        auto env_on = [](const char* n) {
            const char* v = std::getenv(n);
            return v && *v && std::strcmp(v, "0") != 0 && strcasecmp(v, "false") != 0 && strcasecmp(v, "off") != 0;
        };
        // (IPT_FORCE_POOL_GATE=1: keep the pool gate under such a tool --
        // diagnostics of that hang only)
        const bool serialising_tool = (env_on("ROCPROF_COUNTER_COLLECTION") || env_on("ROCPROF_ADVANCED_THREAD_TRACE")) &&
                                      !env_on("IPT_FORCE_POOL_GATE");
        int wv = 0;
        ctx->gate_on_pool = !env_on("IPT_NO_TAIL_OVERLAP") && !serialising_tool &&
                            hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, hip_device) ==
                                hipSuccess &&
                            wv;
        (void)hipGetLastError();  // (an unsupported query leaves no sticky error for the caller's runtime)
    }
    for (WorkSlot& S : ctx->slot) {
        if (hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&S.done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.path_end, hipEventDisableTiming) != hipSuccess ||
            hipMalloc(&S.d_unit, sizeof(unsigned long long)) != hipSuccess) {
            ipt_destroy(ctx);
            return fail(nullptr, IPT_E_DEVICE, "work-slot stream / event / counter creation failed");
        }
        // the pool-drained flag: signal memory, set to 0 by a stream write
        // (without it -- allocation refused -- launches gate on events)
        if (ctx->gate_on_pool) {
            void* sig = nullptr;
            if (hipExtMallocWithFlags(&sig, sizeof(unsigned long long), hipMallocSignalMemory) != hipSuccess ||
                hipStreamWriteValue64(S.st, sig, 0ull, 0) != hipSuccess || hipStreamSynchronize(S.st) != hipSuccess) {
                if (sig) hipFree(sig);
                sig = nullptr;
                ctx->gate_on_pool = false;
                (void)hipGetLastError();
            }
            S.d_drained = reinterpret_cast<unsigned long long*>(sig);
        }
    }
    if (!ctx->gate_on_pool)
        for (WorkSlot& S : ctx->slot) {
            if (S.d_drained) hipFree(S.d_drained);
            S.d_drained = nullptr;
        }
    if (hipMalloc(&ctx->d_counters, sizeof(unsigned long long) * (kNumCounters + 2 * kProfPhases + kStamps)) != hipSuccess ||
        hipMalloc(&ctx->d_wall, sizeof(Frame) * 5) != hipSuccess) {
        ipt_destroy(ctx);
        return fail(nullptr, IPT_E_OOM, "hipMalloc failed");
    }
    hipMemset(ctx->d_counters, 0, sizeof(unsigned long long) * (kNumCounters + 2 * kProfPhases + kStamps));
    if (hipMalloc(&ctx->d_clk, sizeof(unsigned long long) * 2 * (kClkRing + 1)) != hipSuccess) {
        ipt_destroy(ctx);
        return fail(nullptr, IPT_E_OOM, "hipMalloc failed");
    }
    ctx->d_clk_dummy = ctx->d_clk + 2 * kClkRing;
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, hip_device) == hipSuccess && khz > 0)
            ctx->clk_khz = (double)khz;
        (void)hipGetLastError();
    }
    *out = ctx;
    return IPT_OK;
}

void ipt_destroy(ipt_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    (void)drain(ctx);  // nothing queued may still use the buffers
    void* bufs[] = {ctx->d_cdf_lo, ctx->d_lgrid, ctx->d_lax, ctx->d_bvh_nodes, ctx->d_bvh_prims, ctx->d_light_nodes, ctx->d_lights, ctx->d_weights, ctx->d_cdf, ctx->d_wall, ctx->d_spheres,
                    ctx->d_counters, ctx->d_cos_a, ctx->d_cos_b, ctx->d_clk,
                    ctx->d_grid_start, ctx->d_grid_items, ctx->d_grid_c4, ctx->d_grid_cells, ctx->d_frame_sc,
                    ctx->d_grid_packed};
    for (void* b : bufs)
        if (b) hipFree(b);
    for (WorkSlot& S : ctx->slot) {
        void* sb[] = {S.d_values, S.d_codes, S.d_rg, S.d_flags, S.d_cand_rows, S.d_cand_of_row, S.d_unit, S.d_drained};
        for (void* b : sb)
            if (b) hipFree(b);
        if (S.done) hipEventDestroy(S.done);
        if (S.path_end) hipEventDestroy(S.path_end);
        if (S.st) hipStreamDestroy(S.st);
    }
    for (hipEvent_t e : ctx->ev_pool) hipEventDestroy(e);
    for (void* b : {(void*)ctx->rp.d_pixels, (void*)ctx->rp.d_counters, (void*)ctx->rp.d_sums, (void*)ctx->rp.d_pmax})
        if (b) hipFree(b);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
}

int ipt_upload_scene(ipt_ctx* ctx, const ipt_scene* s) {
    if (!ctx) return IPT_E_INVALID;
    hipSetDevice(ctx->device);
    {
        const int rc = drain(ctx);  // queued launches read the scene being replaced
        if (rc) return rc;
    }
    ctx->has_scene = false;  // any failure below leaves no scene (ipt_capi.h)
    if (!s) return fail(ctx, IPT_E_INVALID, "scene is NULL");
    if (s->geometry_kind < IPT_GEOM_SPHERE_IN_BOX || s->geometry_kind > IPT_GEOM_SMALLPT)
        return fail(ctx, IPT_E_UNSUPPORTED, "unknown geometry_kind");
    if (s->n_lights < 0 || s->n_lights > kMaxLights || (s->n_lights > 0 && !s->lights))
        return fail(ctx, IPT_E_UNSUPPORTED, "n_lights out of range");
    if (s->n_spheres < 0 || (s->n_spheres > 0 && !s->spheres))
        return fail(ctx, IPT_E_INVALID, "bad sphere array");
    hipSetDevice(ctx->device);
    const int nl = s->n_lights;
    std::vector<LightDev> L(std::max(nl, 1));
    std::vector<float> powers(std::max(nl, 1));
    bool any_round = false;
    for (int i = 0; i < nl; ++i) {
        const ipt_area_light& a = s->lights[i];
        if (a.type < IPT_LIGHT_AREA_DIAMOND || a.type > IPT_LIGHT_OUTER_SPHERE)
            return fail(ctx, IPT_E_UNSUPPORTED, "unknown light type");
        if (a.type >= IPT_LIGHT_SPHERE) any_round = true;
        L[i] = make_light(v3(a.position[0], a.position[1], a.position[2]),
                          v3(a.x_axis[0], a.x_axis[1], a.x_axis[2]),
                          v3(a.y_axis[0], a.y_axis[1], a.y_axis[2]), a.power, a.type);
        powers[i] = a.power;
    }
    std::vector<float> wts(nl + 1), cdf(nl + 1);
    mixture_weights(powers.data(), nl, wts.data());
    float acc = 0.0f;
    for (int i = 0; i <= nl; ++i) {
        acc += wts[i];  // UnionDdf::sample's running sum (ddf.cpp:145-146)
        cdf[i] = acc;
    }
    // plane frames, indexed by the plane primitive the geometry trace returns:
    // box: RotateDdf(CosineDdf, -plane) for planes {+x,+y,+z,-x,-z};
    // corner: RotateDdf(CosineDdf, n) for n = +x, +y, +z (GeometryCorner.cpp:16-28);
    // floor: its unrotated CosineDdf == make_frame((0,0,1)), which is exactly
    // the identity (axis falls back to +x, angle acos(1) = 0, sin 0 = 0, cos 0 = 1)
    const vec3 planes[5] = {v3(1, 0, 0), v3(0, 1, 0), v3(0, 0, 1), v3(-1, 0, 0), v3(0, 0, -1)};
    Frame wall[5];
    for (int i = 0; i < 5; ++i) wall[i] = make_frame(-planes[i]);
    if (s->geometry_kind == IPT_GEOM_CORNER)
        for (int i = 0; i < 3; ++i) wall[i] = make_frame(planes[i]);
    if (s->geometry_kind == IPT_GEOM_FLOOR) wall[0] = make_frame(v3(0, 0, 1));
    std::vector<float4> sph(std::max(s->n_spheres, 1));
    for (int i = 0; i < s->n_spheres; ++i)
        sph[i] = make_float4(s->spheres[i].center[0], s->spheres[i].center[1], s->spheres[i].center[2], s->spheres[i].radius);
    // Bound of every surface point a ray can start from: the box [-1,1]^3 and
    // the spheres (ipt_bvh.h pads item boxes from it and the camera).
    float B = 1.0f;
    for (int i = 0; i < s->n_spheres; ++i)
        B = std::max(B, std::max(std::fabs(sph[i].x), std::max(std::fabs(sph[i].y), std::fabs(sph[i].z))) +
                            std::fabs(sph[i].w));
    const float cam[3] = {s->camera.position[0], s->camera.position[1], s->camera.position[2]};
    std::vector<BvhNode> bnodes;
    std::vector<BvhSphere> bprims;
    int per_order = 0;
    float tmargin = 0.0f;
    // many spheres inside the box: a uniform grid; otherwise (and if the grid
    // cannot be built) the BVH
    SphereGrid grid;
    bool use_grid = IPT_SPHERE_GRID && s->geometry_kind == IPT_GEOM_SPHERES_IN_BOX && s->n_spheres > 256 &&
                    grid_build_spheres(reinterpret_cast<const float*>(sph.data()), s->n_spheres, cam, B, grid);
    if (!use_grid && (s->geometry_kind == IPT_GEOM_SPHERES_IN_BOX || s->geometry_kind == IPT_GEOM_SPHERES) &&
        s->n_spheres > 16)
        bvh_build_spheres(reinterpret_cast<const float*>(sph.data()), s->n_spheres, cam, B, bnodes, bprims,
                          &per_order, &tmargin);
    // light BVH: only for the global-memory light mode (n_lights > kLdsLights)
    std::vector<BvhNode> lnodes;
    int n_lnodes = 0;
    if (nl > kLdsLights && !any_round) {  // the light BVH indexes AreaLights only
        std::vector<std::array<float, 3>> lp(nl), lx(nl), ly(nl);
        std::vector<std::array<float, 9>> li(nl);
        for (int i = 0; i < nl; ++i) {
            lp[i] = {L[i].P.x, L[i].P.y, L[i].P.z};
            lx[i] = {L[i].x.x, L[i].x.y, L[i].x.z};
            ly[i] = {L[i].y.x, L[i].y.y, L[i].y.z};
            for (int c = 0; c < 3; ++c) {
                li[i][3 * c + 0] = L[i].inv.c[c].x;
                li[i][3 * c + 1] = L[i].inv.c[c].y;
                li[i][3 * c + 2] = L[i].inv.c[c].z;
            }
        }
        if (!bvh_build_lights(nl, reinterpret_cast<const float(*)[3]>(lp.data()),
                              reinterpret_cast<const float(*)[3]>(lx.data()),
                              reinterpret_cast<const float(*)[3]>(ly.data()),
                              reinterpret_cast<const float(*)[9]>(li.data()), cam, B, lnodes, &n_lnodes)) {
            lnodes.clear();
            n_lnodes = 0;
        }
    }
    LightGrid lg;
    const bool use_lgrid = IPT_LIGHT_GRID && ctx->light_grid_on && nl > kLdsLights && !any_round &&
                           s->geometry_kind == IPT_GEOM_SPHERE_IN_BOX && light_grid_build(L.data(), nl, lg);
    // (the lattice instances take the range-free light arithmetic: every
    // light's ranges proven as for the single light)
    bool lg_inr = use_lgrid;
    for (int i = 0; lg_inr && i < nl; ++i) lg_inr = light_ranges_box(L[i], 2, cam);
    if (!use_lgrid || !lg_inr) lg = LightGrid{};
    // bucket starts of the pick's scan: lo[b] = first c with cdf[c] > b/256
    // (the float compare the scan makes; nl+1 if none); kept when no bucket
    // spans more than 8 entries
    std::vector<int> cdf_lo(kCdfBuckets);
    bool use_cdf_lo = IPT_CDF_LO && nl > kLdsLights && !any_round;
    for (int b = 0; use_cdf_lo && b < kCdfBuckets; ++b) {
        const float start = (float)b / (float)kCdfBuckets;
        int c = 0;
        while (c <= nl && !(start < cdf[c])) ++c;
        cdf_lo[b] = c;
        const float end = (float)(b + 1) / (float)kCdfBuckets;
        int e = c;
        while (e <= nl && !(end < cdf[e])) ++e;
        if (e - c > 8) use_cdf_lo = false;
    }
    bool cdf_mono = true;
    for (int i = 0; i <= nl; ++i)
        if (!(cdf[i] == cdf[i]) || (i > 0 && !(cdf[i - 1] <= cdf[i]))) cdf_mono = false;
    // Device phase, transactional: every buffer of the new scene is allocated
    // and filled in a temporary first. Until all of them succeeded the context
    // has no scene (renders fail with IPT_E_NOSCENE, never launch on a
    // half-built one); on success the old buffers are freed and the new ones
    // swapped in. IPT_TEST_FAIL_UPLOAD_ALLOC=k makes the k-th allocation of an
    // upload fail (tests/test_gpu_parity.py exercises the failure path).
    ctx->has_scene = false;
    int n_alloc = 0;
    int fail_at = 0;
    if (const char* e = std::getenv("IPT_TEST_FAIL_UPLOAD_ALLOC")) fail_at = std::atoi(e);
    auto upload = [&](auto& buf, const auto* src, size_t count) -> int {
        using T = std::remove_pointer_t<decltype(buf.p)>;
        if (++n_alloc == fail_at) return fail(ctx, IPT_E_OOM, "injected allocation failure (IPT_TEST_FAIL_UPLOAD_ALLOC)");
        HIPCHECK(ctx, hipMalloc(&buf.p, sizeof(T) * std::max<size_t>(count, 1)));
        if (count) HIPCHECK(ctx, hipMemcpy(buf.p, src, sizeof(T) * count, hipMemcpyHostToDevice));
        return IPT_OK;
    };
    DevBuf<int> n_grid_start, n_lgrid, n_cdf_lo, n_grid_packed;
    DevBuf<LightAx> n_lax;
    DevBuf<BvhSphere> n_grid_items, n_bvh_prims;
    DevBuf<float4> n_grid_c4;
    DevBuf<GridCell> n_grid_cells;
    DevBuf<BvhNode> n_light_nodes, n_bvh_nodes;
    DevBuf<LightDev> n_lights;
    DevBuf<float> n_weights, n_cdf;
    DevBuf<float4> n_spheres;
    DevBuf<Frame> n_wall;
    int rc = IPT_OK;
    if (use_grid && !rc) rc = upload(n_grid_start, grid.start.data(), grid.start.size());
    if (use_grid && !rc) rc = upload(n_grid_items, grid.items.data(), grid.items.size());
    // IPT_GRID_LDS: grid.start as 8-entry block bases + byte offsets (every
    // offset must fit a byte, else the instance is refused at render time)
    std::vector<int> packed;
    int packed_nb = 0;
    if (IPT_GRID_LDS && use_grid) {
        const size_t ne = grid.start.size();
        packed_nb = (int)((ne + 7) / 8);
        packed.assign((size_t)packed_nb + (ne + 3) / 4, 0);
        uint8_t* off = reinterpret_cast<uint8_t*>(packed.data() + packed_nb);
        bool fits = true;
        for (size_t e = 0; e < ne; ++e) {
            if (e % 8 == 0) packed[e / 8] = grid.start[e];
            const int d = grid.start[e] - packed[e / 8];
            fits &= d >= 0 && d <= 255;
            off[e] = (uint8_t)d;
        }
        if (!fits) packed.clear();
        if (!packed.empty() && !rc) rc = upload(n_grid_packed, packed.data(), packed.size());
    }
    if (IPT_GRID_C4 && use_grid && !rc) {
        const size_t ni = grid.items.size();
        std::vector<float4> c4(ni + (ni + 3) / 4);
        int* idx = reinterpret_cast<int*>(c4.data() + ni);
        for (size_t k = 0; k < ni; ++k) {
            const BvhSphere& b = grid.items[k];
            c4[k] = make_float4(b.c[0], b.c[1], b.c[2], b.r);
            idx[k] = b.index;
        }
        rc = upload(n_grid_c4, c4.data(), c4.size());
    }
    std::vector<GridCell> gcells;
    if (IPT_GRID_INLINE && use_grid) grid_cells_build(grid, gcells);
    if (IPT_GRID_INLINE && use_grid && !rc) rc = upload(n_grid_cells, gcells.data(), gcells.size());
    if (!lnodes.empty() && !rc) rc = upload(n_light_nodes, lnodes.data(), lnodes.size());
    if (lg.pattern && !rc) rc = upload(n_lgrid, lg.cells.data(), lg.cells.size());
    std::vector<LightAx> laxr;
    if (lg.pattern)
        for (int i = 0; i < nl; ++i) laxr.push_back(light_ax_record(L[i], lg.pattern, wts[i]));
    if (lg.pattern && !rc) rc = upload(n_lax, laxr.data(), laxr.size());
    // IPT_LPF_CALC: is every lattice light's sample record the formula of its
    // index (a power-of-two row length, one origin, one pitch per axis)? The
    // exact float operations of the kernel are replayed here for every light.
    int lpf_calc = 0, lc_shift = 0, ltr_calc = 0, lg_ident = 0;
    float lcv[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (IPT_LPF_CALC && lg.pattern && nl >= 2) {
        int row = 1;
        while (row < nl && laxr[row].py == laxr[0].py) ++row;
        const bool p2 = row >= 2 && (row & (row - 1)) == 0 && nl % row == 0;
        if (p2) {
            lc_shift = 0;
            while ((1 << lc_shift) < row) ++lc_shift;
            const float cand[2] = {laxr[0].xa, laxr[0].ya};
            for (int cx = 0; cx < 2 && !lpf_calc; ++cx)
                for (int cy = 0; cy < 2 && !lpf_calc; ++cy) {
                    const float x0 = laxr[0].px, y0 = laxr[0].py, dx = cand[cx], dy = cand[cy];
                    bool ok = true;
                    for (int i = 0; ok && i < nl; ++i) {
                        volatile float fx = (float)(i & (row - 1)) * dx;  // (no contraction, as the kernel)
                        volatile float fy = (float)(i >> lc_shift) * dy;
                        const float px = x0 + fx, py = y0 + fy;
                        ok = f2u(px) == f2u(laxr[i].px) && f2u(py) == f2u(laxr[i].py) &&
                             f2u(laxr[i].xa) == f2u(laxr[0].xa) && f2u(laxr[i].ya) == f2u(laxr[0].ya);
                    }
                    if (ok) {
                        lpf_calc = 1;
                        lcv[0] = x0; lcv[1] = y0; lcv[2] = dx; lcv[3] = dy;
                        lcv[4] = laxr[0].xa; lcv[5] = laxr[0].ya;
                    }
                }
        }
        // the light tests' records: the rest uniform, the cells an index formula
        if (IPT_LTR_CALC && lpf_calc) {
            bool same = true;
            for (int i = 1; same && i < nl; ++i)
                same = f2u(laxr[i].ix) == f2u(laxr[0].ix) && f2u(laxr[i].iy) == f2u(laxr[0].iy) &&
                       f2u(laxr[i].area) == f2u(laxr[0].area) && f2u(laxr[i].spow) == f2u(laxr[0].spow);
            if (same) {
                ltr_calc = 1;
                lcv[6] = laxr[0].ix; lcv[7] = laxr[0].iy; lcv[8] = laxr[0].area; lcv[9] = laxr[0].spow;
            }
            bool id1 = (int)lg.cells.size() == lg.nu * lg.nv, id2 = id1;
            for (int j = 0; (id1 || id2) && j < lg.nv; ++j)
                for (int i = 0; i < lg.nu; ++i) {
                    const int c = lg.cells[i + lg.nu * j];
                    id1 = id1 && c == i + lg.nu * j;
                    id2 = id2 && c == j + lg.nv * i;
                }
            lg_ident = id1 ? 1 : (id2 ? 2 : 0);
        }
    }
    if (use_cdf_lo && !rc) rc = upload(n_cdf_lo, cdf_lo.data(), cdf_lo.size());
    if (!bnodes.empty() && !rc) rc = upload(n_bvh_nodes, bnodes.data(), bnodes.size());
    if (!bnodes.empty() && !rc) rc = upload(n_bvh_prims, bprims.data(), bprims.size());
    if (!rc) rc = upload(n_lights, L.data(), L.size());
    if (!rc) rc = upload(n_weights, wts.data(), (size_t)nl + 1);
    if (!rc) rc = upload(n_cdf, cdf.data(), (size_t)nl + 1);
    if (!rc) rc = upload(n_wall, wall, 5);
    if (!rc) rc = upload(n_spheres, sph.data(), sph.size());
    if (rc) return rc;  // the temporaries free themselves; the context keeps no scene
    void* old[] = {ctx->d_lights, ctx->d_weights, ctx->d_cdf, ctx->d_spheres, ctx->d_bvh_nodes, ctx->d_bvh_prims,
                   ctx->d_light_nodes, ctx->d_grid_start, ctx->d_grid_items, ctx->d_grid_c4, ctx->d_grid_cells, ctx->d_wall, ctx->d_lgrid, ctx->d_lax,
                   ctx->d_cdf_lo, ctx->d_grid_packed};
    for (void* b : old)
        if (b) hipFree(b);
    ctx->d_grid_start = n_grid_start.release();
    ctx->d_grid_packed = n_grid_packed.release();
    ctx->grid_packed_words = (int)packed.size();
    ctx->grid_packed_nb = packed_nb;
    ctx->d_grid_items = n_grid_items.release();
    ctx->d_grid_c4 = n_grid_c4.release();
    ctx->d_grid_cells = n_grid_cells.release();
    ctx->n_grid = 0;
    if (use_grid) {
        ctx->n_grid = (int)(grid.start.size() - 1);
        ctx->grid_n_items = grid.items.size();
        ctx->bvh_tmargin = grid.tmargin;
        grid.start.clear();
        grid.items.clear();
        ctx->grid = grid;
    }
    ctx->d_light_nodes = n_light_nodes.release();
    ctx->n_light_nodes = lnodes.empty() ? 0 : n_lnodes;
    ctx->d_lgrid = n_lgrid.release();
    ctx->d_lax = n_lax.release();
    ctx->d_cdf_lo = n_cdf_lo.release();
    ctx->lpf_calc = lpf_calc;
    ctx->lc_shift = lc_shift;
    ctx->ltr_calc = ltr_calc;
    ctx->lg_ident = lg_ident;
    std::copy(lcv, lcv + 10, ctx->lc);
    lg.cells.clear();
    ctx->lgrid = lg;
    ctx->cdf_bsearch = cdf_mono ? 1 : 0;
    ctx->pk_u0 = word_threshold(cdf[0]);
    ctx->pk_u1 = word_threshold(nl >= 1 ? cdf[1] : 0.0f);
    // nearly equal lights (e.g. 256 of one power: weights within rounding of
    // 0.5/256 = 2^-9): with w = 2^-e and every light's |cdf[i] - (i+1) w| <= d
    // < w/2 on a non-decreasing cdf, the first c with r < cdf[c] is ce - 1, ce
    // or ce + 1 for ce = floor(r/w) = floor(r 2^e) (exact: r = m 2^-24): cdf[ce-2]
    // <= (ce-1) w + d < ce w <= r and cdf[ce+1] >= (ce+2) w - d > r + w - d > r.
    // Past the lights (ce >= nl) the scan's answer is ce's clamp to nl - 1, then
    // cdf[nl]. The kernel reads cdf[ce-1] and cdf[ce] only.
    ctx->cdf_p2 = 0;
    for (int e = 1; IPT_CDF_POW2 && cdf_mono && nl > kLdsLights && !any_round && e <= 20 && !ctx->cdf_p2; ++e) {
        const double w = std::ldexp(1.0, -e);
        bool ok = (double)nl * w <= 1.0;
        for (int i = 0; ok && i < nl; ++i) ok = std::fabs((double)cdf[i] - (double)(i + 1) * w) < 0.25 * w;
        if (ok) {
            ctx->cdf_p2 = 1;
            // exactly uniform on the draw's 24-bit integer: every light's
            // ceil(cdf[i] 2^24) is (i+1) 2^(24-e) (C5's 256 equal emitters),
            // so the integer pick reads no cdf entry at all (KParams::cdf_p2 2)
            if (IPT_PICK_INT_CDF && IPT_CDF_EXACT && e <= 24) {
                bool exact = true;
                for (int i = 0; exact && i < nl; ++i)
                    exact = (word_threshold(cdf[i]) >> 8) == ((unsigned long long)(i + 1) << (24 - e));
                if (exact) ctx->cdf_p2 = 2;
            }
            ctx->cdf_p2s = std::ldexp(1.0f, e);
            ctx->cdf_p2e = e;
            ctx->cdf_end = cdf[nl];
        }
    }
    ctx->any_round_light = any_round;
    // the axis-aligned single-light instances also take the range-free roots
    // and quotients: only where their ranges are proven (sphere-in-box scenes)
    ctx->light_axis = (nl == 1 && !any_round && IPT_LIGHT_AXIS) ? axis_aligned_light(L[0]) : 0;
    if (ctx->light_axis && !(s->geometry_kind == IPT_GEOM_SPHERE_IN_BOX && light_ranges_box(L[0], 2, cam)))
        ctx->light_axis = 0;
    // skip-ahead plane: one area light (or a lattice, whose lights share P.z
    // and n.z bit for bit) whose axes have zero z components, so that every
    // sampled point (x*u1 + y*u2) + P has z = P.z exactly, and whose normal is
    // (+-0, +-0, n.z): a light sample's cosinus then has the sign of
    // n.z * (o.z - P.z) whatever the draws (lighting.cpp:93-104, 125-134)
    ctx->sa_on = 0;
    {
        auto zero = [](float f) { return (f2u(f) & 0x7fffffffu) == 0u; };
        bool ok = nl >= 1 && !any_round && (nl == 1 || lg.pattern != 0);
        for (int i = 0; ok && i < nl; ++i)
            ok = (L[i].type == 0 || L[i].type == 1) && zero(L[i].x.z) && zero(L[i].y.z) && zero(L[i].n.x) &&
                 zero(L[i].n.y) && !zero(L[i].n.z) && std::isfinite(L[i].n.z) && std::fabs(L[i].P.z) >= 0x1p-32f &&
                 std::fabs(L[i].P.z) <= 0x1p32f &&
                 f2u(L[i].P.z) == f2u(L[0].P.z) && f2u(L[i].n.z) == f2u(L[0].n.z);
        if (ok) {
            ctx->sa_on = 1;
            ctx->sa_pz = L[0].P.z;
            ctx->sa_nz = L[0].n.z;
            // UnionDdf::sample picks a light (c < nl) iff r < cdf[c] for some
            // c < nl, i.e. iff r < cdf[nl - 1] on a non-decreasing cdf
            ctx->sa_cl = (nl == 1 || cdf_mono) ? cdf[nl - 1] : 0.0f;
        }
        ctx->sa_u = word_threshold(ctx->sa_on ? ctx->sa_cl : 0.0f);
    }
    ctx->d_bvh_nodes = n_bvh_nodes.release();
    ctx->d_bvh_prims = n_bvh_prims.release();
    ctx->n_nodes = 0;
    if (!bnodes.empty()) {
        ctx->n_nodes = per_order;  // nodes per octant order; buffer holds kBvhOrders of them
        ctx->bvh_tmargin = tmargin;
    }
    ctx->d_lights = n_lights.release();
    ctx->d_weights = n_weights.release();
    ctx->d_cdf = n_cdf.release();
    ctx->d_wall = n_wall.release();
    ctx->d_spheres = n_spheres.release();
    ctx->geometry_kind = s->geometry_kind;
    ctx->n_lights = nl;
    ctx->n_spheres = s->n_spheres;
    const ipt_camera& c = s->camera;
    ctx->cam_pos = v3(c.position[0], c.position[1], c.position[2]);
    ctx->cam_dir = v3(c.direction[0], c.direction[1], c.direction[2]);
    ctx->cam_right = v3(c.right[0], c.right[1], c.right[2]);
    ctx->cam_up = v3(c.up[0], c.up[1], c.up[2]);
    // every ray origin (camera, surface points within B) inside 2^39: the box
    // planes may use the range-free division (box_plane_t<true>)
    const float lim = 549755813888.0f;  // 2^39
    ctx->box_inrange = B < lim && std::fabs(cam[0]) < lim && std::fabs(cam[1]) < lim && std::fabs(cam[2]) < lim;
    ctx->has_scene = true;
    return IPT_OK;
}

int ipt_render_device_async(ipt_ctx* ctx, const ipt_params* p, ipt_image* img, void* hip_stream) {
    int rc = validate(ctx, p);
    if (rc) return rc;
    if (!img || !img->pixels || !img->counters) return fail(ctx, IPT_E_INVALID, "image pixels/counters are NULL");
    hipSetDevice(ctx->device);
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    return render_chunks(ctx, p, img, st, nullptr, nullptr);
}

int ipt_render_wait(ipt_ctx* ctx) {
    if (!ctx) return IPT_E_INVALID;
    hipSetDevice(ctx->device);
    return drain(ctx);
}

int ipt_render_device(ipt_ctx* ctx, const ipt_params* p, ipt_image* img, void* hip_stream) {
    const int rc = ipt_render_device_async(ctx, p, img, hip_stream);
    const int rw = ctx ? drain(ctx) : IPT_OK;
    return rc ? rc : rw;
}

int ipt_render(ipt_ctx* ctx, const ipt_params* p, ipt_image* himg) {
    int rc = validate(ctx, p);
    if (rc) return rc;
    if (!himg || !himg->pixels || !himg->counters) return fail(ctx, IPT_E_INVALID, "image pixels/counters are NULL");
    hipSetDevice(ctx->device);
    ResidentPlane& R = ctx->rp;
    R.h2d = R.d2h = 0;
    const int W = p->width, H = p->height;
    const bool has_sums = himg->sums != nullptr, has_pmax = himg->pixel_max != nullptr;
    if (R.W != W || R.H != H || R.has_sums != has_sums || R.has_pmax != has_pmax || !R.d_pixels) {
        for (void* b : {(void*)R.d_pixels, (void*)R.d_counters, (void*)R.d_sums, (void*)R.d_pmax})
            if (b) hipFree(b);
        R = ResidentPlane{};
        const size_t npix = (size_t)W * H;
        HIPCHECK(ctx, hipMalloc(&R.d_pixels, npix * 4));
        HIPCHECK(ctx, hipMalloc(&R.d_counters, npix * 4));
        if (has_sums) HIPCHECK(ctx, hipMalloc(&R.d_sums, npix * 4));
        if (has_pmax) HIPCHECK(ctx, hipMalloc(&R.d_pmax, npix * 4));
        R.W = W;
        R.H = H;
        R.has_sums = has_sums;
        R.has_pmax = has_pmax;
    }
    const bool sharded = p->n_shards > 1 && p->tile_rows > 0;
    const int plan[3] = {sharded ? p->tile_rows : 0, sharded ? p->n_shards : 1, sharded ? p->shard_id : 0};
    if (!std::equal(plan, plan + 3, R.plan)) {
        R.runs.clear();
        R.owned_px = 0;
        for (int y = 0; y < H;) {
            if (!owned_host(p, y)) { ++y; continue; }
            int y1 = y + 1;
            while (y1 < H && owned_host(p, y1)) ++y1;
            R.runs.emplace_back(y, y1);
            R.owned_px += (size_t)(y1 - y) * W;
            y = y1;
        }
        std::copy(plan, plan + 3, R.plan);
        R.shadow_ok = false;
    }
    // (host field, device field) in shadow order
    struct Field { uint8_t* h; uint8_t* d; };
    std::vector<Field> fields = {{reinterpret_cast<uint8_t*>(himg->pixels), reinterpret_cast<uint8_t*>(R.d_pixels)},
                                 {reinterpret_cast<uint8_t*>(himg->counters), reinterpret_cast<uint8_t*>(R.d_counters)}};
    if (has_sums) fields.push_back({reinterpret_cast<uint8_t*>(himg->sums), reinterpret_cast<uint8_t*>(R.d_sums)});
    if (has_pmax) fields.push_back({reinterpret_cast<uint8_t*>(himg->pixel_max), reinterpret_cast<uint8_t*>(R.d_pmax)});
    const size_t field_bytes = R.owned_px * 4;
    if (R.shadow.size() != fields.size() * field_bytes) {
        R.shadow.assign(fields.size() * field_bytes, 0);
        R.shadow_ok = false;
    }
    hipStream_t st = ctx->stream;
    // upload the owned runs the caller changed since the last call (all of
    // them when the shadow is not valid)
    for (size_t f = 0; f < fields.size(); ++f) {
        size_t off = f * field_bytes;
        for (const auto& r : R.runs) {
            const size_t b0 = (size_t)r.first * W * 4, len = (size_t)(r.second - r.first) * W * 4;
            if (!R.shadow_ok || std::memcmp(fields[f].h + b0, R.shadow.data() + off, len) != 0) {
                HIPCHECK(ctx, hipMemcpyAsync(fields[f].d + b0, fields[f].h + b0, len, hipMemcpyHostToDevice, st));
                R.h2d += len;
            }
            off += len;
        }
    }
    R.shadow_ok = false;  // (valid again only once this call's rows are back)
    ipt_image d{R.d_pixels, R.d_counters, R.d_sums, R.d_pmax};
    rc = render_chunks(ctx, p, &d, st, nullptr, nullptr);
    if (rc) {
        (void)drain(ctx);  // nothing queued may still use the buffers
        (void)hipStreamSynchronize(st);
        return rc;
    }
    for (size_t f = 0; f < fields.size(); ++f)
        for (const auto& r : R.runs) {
            const size_t b0 = (size_t)r.first * W * 4, len = (size_t)(r.second - r.first) * W * 4;
            HIPCHECK(ctx, hipMemcpyAsync(fields[f].h + b0, fields[f].d + b0, len, hipMemcpyDeviceToHost, st));
            R.d2h += len;
        }
    HIPCHECK(ctx, hipStreamSynchronize(st));
    rc = drain(ctx);
    if (rc) return rc;
    for (size_t f = 0; f < fields.size(); ++f) {
        size_t off = f * field_bytes;
        for (const auto& r : R.runs) {
            const size_t b0 = (size_t)r.first * W * 4, len = (size_t)(r.second - r.first) * W * 4;
            std::memcpy(R.shadow.data() + off, fields[f].h + b0, len);
            off += len;
        }
    }
    R.shadow_ok = true;
    return IPT_OK;
}

int ipt_transfer_bytes(ipt_ctx* ctx, uint64_t* host_to_device, uint64_t* device_to_host) {
    if (!ctx || !host_to_device || !device_to_host) return IPT_E_INVALID;
    *host_to_device = ctx->rp.h2d;
    *device_to_host = ctx->rp.d2h;
    return IPT_OK;
}

int ipt_render_values(ipt_ctx* ctx, const ipt_params* p, float* values, uint8_t* codes) {
    int rc = validate(ctx, p);
    if (rc) return rc;
    if (!values || !codes) return fail(ctx, IPT_E_INVALID, "values/codes are NULL");
    if (p->n_shards > 1) return fail(ctx, IPT_E_UNSUPPORTED, "ipt_render_values renders whole frames");
    hipSetDevice(ctx->device);
    rc = render_chunks(ctx, p, nullptr, ctx->stream, values, codes);
    const int rw = drain(ctx);  // the host copies run on the slot streams
    if (rc) return rc;
    if (rw) return rw;
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    return IPT_OK;
}

int ipt_shard_plan(const ipt_params* p, uint8_t* owned_rows, int32_t* cand_rows, int32_t* n_cand) {
    if (!p || !owned_rows || !cand_rows || !n_cand || p->height <= 0) return IPT_E_INVALID;
    std::vector<int> rows, of_row;
    candidate_rows(p, rows, of_row);
    for (int y = 0; y < p->height; ++y) owned_rows[y] = owned_host(p, y) ? 1 : 0;
    for (size_t i = 0; i < rows.size(); ++i) cand_rows[i] = rows[i];
    *n_cand = (int32_t)rows.size();
    return IPT_OK;
}

int ipt_get_counters(ipt_ctx* ctx, ipt_counters* out) {
    if (!ctx || !out) return IPT_E_INVALID;
    hipSetDevice(ctx->device);
    if (const int rc = drain(ctx)) return rc;
    unsigned long long h[kNumCounters];
    HIPCHECK(ctx, hipMemcpy(h, ctx->d_counters, sizeof h, hipMemcpyDeviceToHost));
    out->paths = h[0];
    out->traced_rays = h[1];
    out->surface_hits = h[2];
    out->light_hits = h[3];
    out->expanded_nodes = h[4];
    out->iterations = h[5];
    out->light_samples = h[6];
    out->skipped = h[7];
    out->sphere_frames = h[8];
    out->light_traces = h[9];
    out->drifted = h[10];
    out->bvh_nodes = h[11];
    out->sphere_tests = h[12];
    out->light_nodes = h[13];
    out->light_tests = h[14];
    return IPT_OK;
}

int ipt_get_profile(ipt_ctx* ctx, uint64_t* out, int n) {
    if (!ctx || !out || n < 0) return IPT_E_INVALID;
    hipSetDevice(ctx->device);
    if (const int rc = drain(ctx)) return rc;
    unsigned long long h[2 * kProfPhases + kStamps];
    HIPCHECK(ctx, hipMemcpy(h, ctx->d_counters + kNumCounters, sizeof h, hipMemcpyDeviceToHost));
    for (int i = 0; i < n && i < 2 * kProfPhases + kStamps; ++i) out[i] = h[i];
    return IPT_OK;
}

int ipt_reset_counters(ipt_ctx* ctx) {
    if (!ctx) return IPT_E_INVALID;
    hipSetDevice(ctx->device);
    if (const int rc = drain(ctx)) return rc;
    HIPCHECK(ctx, hipMemset(ctx->d_counters, 0, sizeof(unsigned long long) * (kNumCounters + 2 * kProfPhases + kStamps)));
    return IPT_OK;
}

int ipt_last_kernel_ms(ipt_ctx* ctx, float* path_ms, float* accumulate_ms) {
    if (!ctx) return IPT_E_INVALID;
    if (path_ms) *path_ms = ctx->last_path_ms;
    if (accumulate_ms) *accumulate_ms = ctx->last_acc_ms;
    return IPT_OK;
}

int ipt_math_host(int fn, const float* in, float* out, int64_t n) {
    if (!in || !out || n < 0 || fn < 0 || fn > 15) return IPT_E_INVALID;
    const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([=]() {
            for (int64_t i = t; i < n; i += nt) out[i] = math_fn(fn, in[i]);
        });
    for (auto& x : th) x.join();
    return IPT_OK;
}

int ipt_math_device(ipt_ctx* ctx, int fn, const float* in, float* out, int64_t n) {
    if (!ctx || !in || !out || n < 0 || fn < 0 || fn > 15) return IPT_E_INVALID;
    hipSetDevice(ctx->device);
    DevBuf<float> din, dout;
    HIPCHECK(ctx, hipMalloc(&din.p, std::max<int64_t>(n, 1) * 4));
    HIPCHECK(ctx, hipMalloc(&dout.p, std::max<int64_t>(n, 1) * 4));
    HIPCHECK(ctx, hipMemcpy(din.p, in, n * 4, hipMemcpyHostToDevice));
    const long long blocks = (n + 255) / 256;
    if (blocks > 0)
        hipLaunchKernelGGL(math_kernel, dim3((unsigned)blocks), dim3(256), 0, ctx->stream, fn, din.p, dout.p, (long long)n);
    HIPCHECK(ctx, hipGetLastError());
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHECK(ctx, hipMemcpy(out, dout.p, n * 4, hipMemcpyDeviceToHost));
    return IPT_OK;
}

int ipt_philox(ipt_ctx* ctx, uint32_t key0, uint32_t key1, const uint32_t* ctr, uint32_t* out, int64_t n) {
    if (!ctr || !out || n < 0) return ctx ? fail(ctx, IPT_E_INVALID, "ipt_philox: bad arguments") : IPT_E_INVALID;
    if (!ctx) {
        for (int64_t i = 0; i < n; ++i) {
            const u32x4 o = philox4x32_10(ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3], key0, key1);
            for (int q = 0; q < 4; ++q) out[4 * i + q] = o.v[q];
        }
        return IPT_OK;
    }
    hipSetDevice(ctx->device);
    DevBuf<uint4> din, dout;
    HIPCHECK(ctx, hipMalloc(&din.p, std::max<int64_t>(n, 1) * sizeof(uint4)));
    HIPCHECK(ctx, hipMalloc(&dout.p, std::max<int64_t>(n, 1) * sizeof(uint4)));
    HIPCHECK(ctx, hipMemcpy(din.p, ctr, n * sizeof(uint4), hipMemcpyHostToDevice));
    if (n > 0)
        hipLaunchKernelGGL(philox_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, key0, key1,
                           din.p, dout.p, (long long)n);
    HIPCHECK(ctx, hipGetLastError());
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHECK(ctx, hipMemcpy(out, dout.p, n * sizeof(uint4), hipMemcpyDeviceToHost));
    return IPT_OK;
}

static int ddf_call(ipt_ctx* ctx, int value_mode, int kind, const float* params, const float* in, int64_t n,
                    float* out) {
    if (!ctx) return IPT_E_INVALID;
    if (!params || !in || !out || n < 0 || kind < 0 || kind > 3) return fail(ctx, IPT_E_INVALID, "ipt_ddf: bad arguments");
    if (kind == 3 && !value_mode)
        for (int64_t i = 0; i < n; ++i)
            for (int c = 1; c < 3; ++c) {
                const float u = in[3 * i + c];
                if (!(u >= 0.0f && u < 1.0f) || u * 16777216.0f != (float)(uint32_t)(u * 16777216.0f))
                    return fail(ctx, IPT_E_INVALID, "ipt_ddf: table sampler needs u on the 2^-24 grid");
            }
    if (kind == 3) {
        const int rc = ensure_cos_tables(ctx, ctx->stream);
        if (rc) return rc;
    }
    if (!ctx->has_scene) return fail(ctx, IPT_E_INVALID, "ipt_ddf: no scene uploaded");
    if (kind == 1 && (params[3] < 0.0f || params[3] >= (float)ctx->n_lights || params[3] != (float)(int)params[3]))
        return fail(ctx, IPT_E_INVALID, "ipt_ddf: light index out of range");
    hipSetDevice(ctx->device);
    const size_t in_w = 3, out_w = value_mode ? 1 : 3;
    DevBuf<float> dp, din, dout;
    HIPCHECK(ctx, hipMalloc(&dp.p, 8 * sizeof(float)));
    HIPCHECK(ctx, hipMalloc(&din.p, std::max<int64_t>(n, 1) * in_w * sizeof(float)));
    HIPCHECK(ctx, hipMalloc(&dout.p, std::max<int64_t>(n, 1) * out_w * sizeof(float)));
    float hp[8] = {0};
    for (int k = 0; k < (kind == 0 || kind == 3 ? 3 : (kind == 1 ? 4 : 6)); ++k) hp[k] = params[k];
    HIPCHECK(ctx, hipMemcpy(dp.p, hp, sizeof hp, hipMemcpyHostToDevice));
    HIPCHECK(ctx, hipMemcpy(din.p, in, n * in_w * sizeof(float), hipMemcpyHostToDevice));
    if (n > 0)
        hipLaunchKernelGGL(ddf_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, value_mode, kind,
                           dp.p, ctx->d_lights, ctx->d_weights, ctx->d_cdf, ctx->n_lights, din.p, (long long)n, dout.p,
                           ctx->d_cos_a, ctx->d_cos_b);
    HIPCHECK(ctx, hipGetLastError());
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHECK(ctx, hipMemcpy(out, dout.p, n * out_w * sizeof(float), hipMemcpyDeviceToHost));
    return IPT_OK;
}

int ipt_ddf_sample(ipt_ctx* ctx, int kind, const float* params, const float* u, int64_t n, float* dirs) {
    return ddf_call(ctx, 0, kind, params, u, n, dirs);
}

int ipt_ddf_value(ipt_ctx* ctx, int kind, const float* params, const float* dirs, int64_t n, float* values) {
    return ddf_call(ctx, 1, kind, params, dirs, n, values);
}

int ipt_math_selfcheck(ipt_ctx* ctx, int fn, uint64_t lo_bits, uint64_t hi_bits, uint64_t* mismatches,
                       uint32_t* first_bad) {
    if (!ctx || !mismatches || !first_bad || fn < 0 || fn > 22 || hi_bits > (1ull << (fn == 21 ? 46 : 32)) ||
        lo_bits > hi_bits)
        return IPT_E_INVALID;
    hipSetDevice(ctx->device);
    if (fn == 14 || fn == 15) {
        if (!IPT_FRAME_TAB) return fail(ctx, IPT_E_INVALID, "ipt_math_selfcheck: built without the frame table");
        const int rc = ensure_frame_table(ctx, ctx->stream);
        if (rc) return rc;
    }
    DevBuf<unsigned long long> d_bad;
    DevBuf<unsigned int> d_first;
    HIPCHECK(ctx, hipMalloc(&d_bad.p, sizeof(unsigned long long)));
    HIPCHECK(ctx, hipMalloc(&d_first.p, sizeof(unsigned int)));
    HIPCHECK(ctx, hipMemsetAsync(d_bad.p, 0, sizeof(unsigned long long), ctx->stream));
    HIPCHECK(ctx, hipMemsetAsync(d_first.p, 0xff, sizeof(unsigned int), ctx->stream));
    const unsigned long long n = hi_bits - lo_bits;
    if (n > 0 && fn == 21)
        hipLaunchKernelGGL(divcheck_kernel, dim3(ctx->n_cu * 64), dim3(256), 0, ctx->stream,
                           (unsigned long long)lo_bits, n, d_bad.p, d_first.p);
    else if (n > 0)
        hipLaunchKernelGGL(selfcheck_kernel, dim3(ctx->n_cu * 8), dim3(256), 0, ctx->stream, fn,
                           (unsigned long long)lo_bits, n, d_bad.p, d_first.p, ctx->d_frame_sc);
    HIPCHECK(ctx, hipGetLastError());
    unsigned long long hb = 0;
    unsigned int hf = 0;
    HIPCHECK(ctx, hipMemcpyAsync(&hb, d_bad.p, sizeof hb, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipMemcpyAsync(&hf, d_first.p, sizeof hf, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    *mismatches = hb;
    *first_bad = hf;
    return IPT_OK;
}

}  // extern "C"
