/* ipt_capi.h — C-ABI of the MI355X path-tracing inner loop (libipt_hip.so).
 *
 * This is the drop-in boundary for dimalit/ipt's hot path. The reference has
 * no FFI; its boundary is a set of C++ virtual interfaces called per ray
 * (reference src/tracer_interfaces.h:26-54) driven by
 *   render_sample(const Scene&, RenderPlane&, StatsNode*)   src/main.cpp:186-223
 *   ray_power_recursive(...)                                 src/main.cpp:98-184
 * Per-ray virtual calls cannot cross to a GPU, so this ABI works at frame
 * granularity: the caller flattens a Scene (camera + geometry + lights) into
 * the POD structs below once, then asks for whole sample passes.
 *
 * Conventions: plain pointers and sizes, no exceptions, every call returns
 * IPT_OK (0) or a negative IPT_E_* code, the message of the last failure is
 * available from ipt_last_error(). Calls are synchronous unless they take a
 * stream argument. One context per HIP device; contexts are independent, a
 * single context is not reentrant. There is NO CPU fallback: without a usable
 * gfx950 device every rendering call fails with IPT_E_DEVICE.
 */
#ifndef IPT_CAPI_H
#define IPT_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IPT_ABI_VERSION 5

enum {
    IPT_OK = 0,
    IPT_E_INVALID = -1,     /* bad argument / size / pointer */
    IPT_E_DEVICE = -2,      /* HIP runtime or device failure, no gfx950 device */
    IPT_E_UNSUPPORTED = -3, /* scene or parameter outside what the kernels implement */
    IPT_E_NOSCENE = -4,     /* ipt_render before ipt_upload_scene */
    IPT_E_OOM = -5
};

/* Geometry kinds (reference src/geometry/). */
enum {
    /* GeometrySphereInBox (GeometrySphereInBox.cpp:10-81): planes
       {+x,+y,+z,-x,-z} of the cube [-1,1]^3 (no -y wall) then a sphere of
       radius 0.5 at the origin. The sample_scenes[0] geometry. */
    IPT_GEOM_SPHERE_IN_BOX = 0,
    /* The same five box planes followed by N extra spheres scanned in order
       with FractalSpheres' acceptance rule (FractalSpheres.cpp:75-84); the
       10k-primitive stress configuration of BASELINE.json configs[2]. */
    IPT_GEOM_SPHERES_IN_BOX = 1,
    /* GeometryFloor (GeometryFloor.cpp:10-23): the z = -1 face of the cube
       ([-1,1]^2 through intersection_with_box_plane), unrotated CosineDdf.
       sample_scenes' make_scene_square_lit_by_square. */
    IPT_GEOM_FLOOR = 2,
    /* GeometryCorner (GeometryCorner.cpp:10-42): the x = -1, y = -1, z = -1
       faces, strict-< nearest in that order, RotateDdf(CosineDdf, normal).
       sample_scenes' make_scene_lit_corner. */
    IPT_GEOM_CORNER = 3,
    /* FractalSpheres (FractalSpheres.cpp:69-97): the sphere list alone, no
       walls, with the same acceptance rule as IPT_GEOM_SPHERES_IN_BOX.
       sample_scenes' make_scene_fractal. */
    IPT_GEOM_SPHERES = 4,
    /* GeometrySmallPt (GeometrySmallPt.cpp:11-58): the sphere list (smallpt's
       room: pass its 7 spheres) intersected in double precision
       (Sphere::intersect, eps 1e-4), strict-< nearest, normal flipped for
       radius >= 100. sample_scenes' make_scene_smallpt. */
    IPT_GEOM_SMALLPT = 5
};

/* Light kinds (reference src/lighting/lighting.h). Round lights use the
   ipt_area_light record with position = centre and x_axis[0] = radius
   (y_axis unused): SphereLight(centre, radius, power) (lighting.h:44-54),
   PointLight(position, virtual_radius, power) (radius unused, lighting.h:
   31-42), InvertedSphereLight(centre, radius, power) (addOuterLight,
   lighting.h:57-72). */
enum {
    IPT_LIGHT_AREA_DIAMOND = 0,
    IPT_LIGHT_AREA_TRIANGLE = 1,
    IPT_LIGHT_SPHERE = 2,
    IPT_LIGHT_POINT = 3,
    IPT_LIGHT_OUTER_SPHERE = 4
};

/* AreaLight constructor arguments (lighting.cpp:79-90); derived fields
   (area, normal, inverse_matrix, surface power) are computed by
   ipt_upload_scene with the constructor's own float operation order. */
typedef struct ipt_area_light {
    float position[3]; /* Light::position, the corner */
    float x_axis[3];
    float y_axis[3];
    float power;
    int32_t type; /* IPT_LIGHT_AREA_* */
} ipt_area_light;

/* SimpleCamera public fields after construction (SimpleCamera.h:11-13). */
typedef struct ipt_camera {
    float position[3];
    float direction[3];
    float right[3];
    float up[3];
} ipt_camera;

typedef struct ipt_sphere {
    float center[3];
    float radius;
} ipt_sphere;

typedef struct ipt_scene {
    int32_t geometry_kind;     /* IPT_GEOM_* */
    int32_t n_lights;          /* CollectionLighting::lights, insertion order */
    const ipt_area_light* lights;
    int32_t n_spheres;         /* extra spheres for IPT_GEOM_SPHERES_IN_BOX */
    const ipt_sphere* spheres;
    ipt_camera camera;
} ipt_scene;

typedef struct ipt_params {
    int32_t width, height;  /* GridRenderPlane size; render_sample hardcodes 640x640 */
    int32_t spp;            /* number of render_sample passes in this call */
    int32_t spp_offset;     /* absolute index of the first pass (RNG counter) */
    int32_t n_rays;         /* branching factor of the root node (main.cpp:94), 0..65535
                               (above 255: at most 8 suspended levels, i.e. depth_max <= 9
                               once n_rays >= 512, and at most 65529 spheres) */
    int32_t depth_max;      /* main.cpp:95 */
    uint64_t seed;          /* Philox key */
    /* Destination-row sharding across devices: rows are cut into tiles of
       tile_rows rows, tile t belongs to shard t % n_shards. n_shards <= 1 or
       tile_rows <= 0 means this call owns the whole frame. */
    int32_t tile_rows;
    int32_t n_shards;
    int32_t shard_id;
    uint32_t flags;         /* IPT_FLAG_* */
} ipt_params;

enum {
    IPT_FLAG_COUNTERS = 1u /* accumulate ipt_counters during the call */
};

/* Caller-owned GridRenderPlane state (GridRenderPlane.h:9-12), width*height
   row-major each. ipt_render ACCUMULATES into it with GridRenderPlane::addRay's
   running-mean update (GridRenderPlane.cpp:61-75), sample passes in order and
   each pass in render_sample's raster order, so repeated calls with increasing
   spp_offset continue the same image bit-for-bit. Zero-initialise before the
   first call. `sums` (sequential per-pixel sum in the same order) and
   `pixel_max` (per-pixel running maximum; GridRenderPlane::max_value is its
   maximum over the frame) may be NULL. */
typedef struct ipt_image {
    float* pixels;
    uint32_t* counters;
    float* sums;
    float* pixel_max;
} ipt_image;

/* Event counters (SURVEY.md Appendix C vocabulary), summed over the call. */
typedef struct ipt_counters {
    uint64_t paths;           /* root ray_power calls */
    uint64_t traced_rays;     /* Geometry::traceRay calls */
    uint64_t surface_hits;    /* Geometry::traceRay calls that hit */
    uint64_t light_hits;      /* Lighting::traceRayToLight calls that hit */
    uint64_t expanded_nodes;  /* distributionInPoint calls (surface nodes) */
    uint64_t iterations;      /* UnionDdf::sample calls */
    uint64_t light_samples;   /* iterations that sampled a light component */
    uint64_t skipped;         /* iterations that returned vec3() */
    uint64_t sphere_frames;   /* RotateDdf builds at non-wall normals */
    uint64_t light_traces;    /* AreaLight::traceRay calls */
    uint64_t drifted;         /* samples GridRenderPlane maps off their nominal pixel */
    uint64_t bvh_nodes;       /* sphere-BVH nodes visited (IPT_GEOM_SPHERES_IN_BOX) */
    uint64_t sphere_tests;    /* intersection_with_sphere evaluations on the sphere list */
    uint64_t light_nodes;     /* light-BVH nodes visited (many-light scenes) */
    uint64_t light_tests;     /* AreaLight::traceRay evaluations actually run */
} ipt_counters;

typedef struct ipt_ctx ipt_ctx;

int ipt_abi_version(void);
const char* ipt_last_error(ipt_ctx* ctx); /* ctx may be NULL (creation errors) */

/* A context owns its stream and device buffers. The first render allocates its
 * exact sampling tables once: CosineDdf 192 MiB and, for sphere-in-box scenes,
 * the RotateDdf frame-angle table 1 GiB (freed by ipt_destroy). Work buffers
 * grow to the largest render: 37 B per sample (radiance, drift code, raygen
 * record) in equal chunks of at most 2^29 samples (18.5 GiB) and at most 3/4
 * of the device memory free at the call (plus the context's own work
 * buffers), so a context's footprint is <= ~20 GiB and contexts sharing a
 * device get smaller chunks rather than IPT_E_OOM; a call renders all its
 * passes in as few path-kernel launches as that allows (each launch ends in
 * a tail where lanes have run out of paths, so batch passes per call).
 * Environment read here (diagnostics): IPT_LNODES_LDS=0 keeps the light BVH in
 * global memory, IPT_LIGHT_GRID=0 disables the light-lattice lookup (the light
 * BVH is used instead), IPT_LATTICE_LDS=0 keeps the lattice lights' records
 * in global memory (256-thread workgroups instead of one 1024-thread
 * workgroup per CU), IPT_BLOCKS_PER_CU caps the path kernel's residency. */
int ipt_create(int hip_device, ipt_ctx** out);
void ipt_destroy(ipt_ctx* ctx);

/* Copies the scene (caller keeps ownership of its arrays). Transactional: on
   any failure (IPT_E_OOM, IPT_E_DEVICE, ...) the context is left with NO
   scene, so a later render returns IPT_E_NOSCENE instead of rendering a
   half-uploaded one; upload again to recover. */
int ipt_upload_scene(ipt_ctx* ctx, const ipt_scene* scene);

/* Host buffers (the caller's GridRenderPlane state): renders p->spp passes
   into them. Device-resident: the context keeps the rows this call
   accumulates -- every row, or with p->n_shards > 1 the shard's owned tiles
   (ipt_shard_plan) -- on its device across calls, uploads only the owned rows
   whose host bytes changed since it last returned them (none in a
   progressive loop that leaves the plane alone between calls) and downloads
   only the owned rows: 16 B per owned pixel per call with sums and per-pixel
   max, 8 B without. Rows it does not own are neither read nor written, so the
   contexts of a multi-device render can share one host plane (one thread per
   context). Results are identical to copying the whole image each way. */
int ipt_render(ipt_ctx* ctx, const ipt_params* p, ipt_image* host_img);
/* Bytes the last ipt_render moved host -> device and device -> host. */
int ipt_transfer_bytes(ipt_ctx* ctx, uint64_t* host_to_device, uint64_t* device_to_host);

/* Device buffers (hipMalloc'd or torch CUDA tensors). The GridRenderPlane
   replays run on `hip_stream` (NULL = the context's own stream) after the work
   already queued there, in call order; the per-sample work (raygen + path
   kernel) runs on the context's two work-slot streams, consecutive launches
   alternating, so a launch fills the CUs its predecessor's tail leaves idle.
   Synchronous: the call returns when the image is complete (it waits for the
   path and accumulate kernels of every chunk and of every call queued before
   it; ipt_last_kernel_ms then holds their times). */
int ipt_render_device(ipt_ctx* ctx, const ipt_params* p, ipt_image* dev_img, void* hip_stream);

/* The same, returning once the launches are queued (the progressive loop of
   main.cpp:256-285 without a host wait per pass): the image is complete when
   `hip_stream` reaches the point after the call, or after ipt_render_wait.
   NULL is NOT the HIP null stream here but the context's own non-blocking
   stream, which the caller's kernels are not ordered with: a caller that
   passes NULL (torch's default-stream handle is 0) must call ipt_render_wait
   before reading the image. The image buffers must stay valid until then.
   Calls into the same image on the same stream accumulate exactly as
   sequential synchronous calls (bit-identical). ipt_upload_scene, the counter
   calls and ipt_destroy wait for queued work first.
   Consecutive launches (the chunks of one call, or queued calls) start in
   their predecessor's tail: a launch's stream waits (hipStreamWaitValue64) for
   the predecessor's work pool to drain. Under a tool that serialises
   dispatches for counter collection or thread trace (rocprofv3 --pmc / --att,
   detected at ipt_create from ROCPROF_COUNTER_COLLECTION /
   ROCPROF_ADVANCED_THREAD_TRACE), or with IPT_NO_TAIL_OVERLAP=1, a launch
   waits for its predecessor's end instead (same images). */
int ipt_render_device_async(ipt_ctx* ctx, const ipt_params* p, ipt_image* dev_img, void* hip_stream);
/* Waits for every queued render; ipt_last_kernel_ms then holds the times of
   the launches since the previous wait (a synchronous render call waits). */
int ipt_render_wait(ipt_ctx* ctx);

/* Per-sample radiance, for bit-exact verification: values[s][iy][ix] is the
   clamped root ray_power of pass p->spp_offset+s at source pixel (ix,iy)
   (main.cpp:211-214) and codes[s][iy][ix] the GridRenderPlane drift code
   (bits 0-1: dx+1, bits 2-3: dy+1 relative to the nominal destination
   (ix, max(H-2-iy,0)); 0x05 = nominal). Host buffers of spp*width*height. */
int ipt_render_values(ipt_ctx* ctx, const ipt_params* p, float* values, uint8_t* codes);

/* Host-only (no device needed): the tile plan of a sharded render.
   owned_rows[H] = 1 for destination rows this shard accumulates;
   cand_rows[*n_cand] = source rows whose samples it traces (the nominal
   sources of its rows +-1 for GridRenderPlane drift). Arrays sized H. */
int ipt_shard_plan(const ipt_params* p, uint8_t* owned_rows, int32_t* cand_rows, int32_t* n_cand);

int ipt_get_counters(ipt_ctx* ctx, ipt_counters* out);
int ipt_reset_counters(ipt_ctx* ctx);
/* Phase profile of the path kernel: out[2q] = wave executions of phase q,
 * out[2q+1] = active lanes summed over them (words 0..23, -DIPT_PROF=1
 * builds); out[24+s] = wave-cycles in step segment s (words 24..35,
 * -DIPT_STAMP=1 builds; scripts/prof_phases.sh). Zeros in product builds.
 * Cleared by ipt_reset_counters. */
int ipt_get_profile(ipt_ctx* ctx, uint64_t* out, int n);

/* Timing of the kernels of the render calls completed by the most recent wait
   (a synchronous render, or ipt_render_wait after asynchronous ones): ms from
   HIP events, summed over their launches: [0] = the path's per-sample work,
   raygen_kernel + path_kernel (raygen ~0.2 % of it), each launch counted from
   its start or from its predecessor's end, whichever is later (overlapped
   launches sum to their span); [1] = accumulate kernels. */
int ipt_last_kernel_ms(ipt_ctx* ctx, float* path_ms, float* accumulate_ms);

/* ---- image post-process on the GPU, bit-exact --------
   ipt_smooth: GridRenderPlane::smooth(side) (in_place = 1: pixels are
   replaced, as the reference's in-place filter leaves them) or
   computeSmoothedMax(side) (in_place = 0: pixels untouched); *max_value gets
   the reference's max_value (GridRenderPlane.cpp:10-59). Host buffers
   (width*height floats, row-major). side 1 is undefined behaviour in the
   reference (its size_t loop runs past row 0): IPT_E_UNSUPPORTED.
   ipt_glare: Gui's glare bloom (gui.cpp:28-52), out = glare(in, cutoff);
   images up to 4096 x 4096. */
int ipt_smooth(ipt_ctx* ctx, float* pixels, int width, int height, int side, int in_place, float* max_value);
int ipt_glare(ipt_ctx* ctx, const float* in, float* out, int width, int height, float cutoff);

/* ---- the path's DDF samplers, exactly as the kernels evaluate them -----------
   For sampler validation (the reference's chi^2 harness, check_ddf.cpp:114-203)
   and bit-exact checks. Uses the uploaded scene. kind:
     IPT_DDF_COSINE  RotateDdf(CosineDdf, to): params = to[3]
     IPT_DDF_LIGHT   DdfFromLight (lighting.cpp:38-73) of scene light params[3]
                     at origin params[0..2]
     IPT_DDF_MIXTURE UnionDdf(lights..., RotateDdf(CosineDdf, normal)) with
                     the scene's unite() weights: origin params[0..2], normal
                     params[3..5]
     IPT_DDF_COSINE_TABLE  IPT_DDF_COSINE as the path kernel samples it, from
                     the exact CosineDdf tables indexed by the draws' 24 bits
                     (u1, u2 must lie on the RNG's 2^-24 grid)
   ipt_ddf_sample: u = n x {pick, u1, u2} uniforms in [0,1) -> n directions
   (vec3() where the reference's sampler returns it); ipt_ddf_value: n
   directions -> n DDF values. Host buffers. */
#define IPT_DDF_COSINE 0
#define IPT_DDF_LIGHT 1
#define IPT_DDF_MIXTURE 2
#define IPT_DDF_COSINE_TABLE 3
int ipt_ddf_sample(ipt_ctx* ctx, int kind, const float* params, const float* u, int64_t n, float* dirs);
int ipt_ddf_value(ipt_ctx* ctx, int kind, const float* params, const float* dirs, int64_t n, float* values);

/* ---- portable-math probes (same code as the kernels), for tests ---------
   fn: 0 acosf, 1 sinf, 2 cosf, 3 (float)acos((double)x), 4 sincosf->sin,
       5 sincosf->cos, 6 sqrtf, 7 CosineDdf z/M_PI, 8 (float)(2*M_PI*u),
       9 a/b over the division pairs of the fast-division proof (x's bit
         pattern -> an in-range numerator and hashed denominator),
      10 the range-free division (box planes) over the same pairs,
      11 the squares-first length comparison over near-tie pairs (0/1),
      12 the 32-bit work-unit division over hashed (n, d) pairs (bit pattern),
      13 the range-free sqrtf on [2^-96, 2^126) (sqrtf elsewhere),
      14 / 15 sin / cos of the RotateDdf angle (float)acos((double)z) for
         z = x; the self-check compares the path kernel's frame table
      16 (ipt_math_selfcheck only) the sphere-in-box frame without glm's
         zero terms against the exact build, over directions hashed from
         the bit pattern (incl. zero / tiny x and y)
      17 / 18 (ipt_math_selfcheck only) the reciprocal by the hardware rcp
         and one / two Newton corrections against the round-4 range-free
         1.0f / x sequence (three corrections)
      19 / 20 (ipt_math_selfcheck only) the range-free division against
         IEEE a/b over the division pairs of 10 / pairs whose divisors have
         all-ones-like significands
      21 (ipt_math_selfcheck only) the range-free division against IEEE a/b
         over every pair of significands (a, b in [1, 2)): pattern indices
         up to 2^46, i = (a's significand << 23) | b's; first_bad reports
         the a significand (i >> 23)
      22 (ipt_math_selfcheck only) the range-free reciprocal's exact scaling:
         rcp(b) == sign(b) 2^-e rcp(m) for |b| = m 2^e in [2^-40, 2^41) */
int ipt_math_host(int fn, const float* in, float* out, int64_t n);
/* Philox4x32-10 blocks exactly as the kernels generate the per-path stream
   that replaces randf() (include/randf.h:6-11; draw k of path (pass s, pixel
   p) is word k%4 of philox({k/4, s, p, 0}, {seed lo, seed hi})), for
   known-answer tests: out[4i..4i+3] = philox(ctr[4i..4i+3], {key0, key1}).
   ctx NULL: the host build of the same code; otherwise on ctx's device. */
int ipt_philox(ipt_ctx* ctx, uint32_t key0, uint32_t key1, const uint32_t* ctr, uint32_t* out, int64_t n);
int ipt_math_device(ipt_ctx* ctx, int fn, const float* in, float* out, int64_t n);
/* Device self-check of the fast math paths: for every float bit pattern b in
 * [lo_bits, hi_bits) (hi_bits <= 2^32; 2^46 for fn 21) compares function fn as the kernels
 * compute it with its exact restatement, on the device. Returns the number of
 * differing results (NaN == NaN) and the lowest differing pattern (0xffffffff
 * if none). Used to prove a fast path exhaustively (all 2^32 inputs). */
int ipt_math_selfcheck(ipt_ctx* ctx, int fn, uint64_t lo_bits, uint64_t hi_bits, uint64_t* mismatches,
                       uint32_t* first_bad);

#ifdef __cplusplus
}
#endif
#endif /* IPT_CAPI_H */
