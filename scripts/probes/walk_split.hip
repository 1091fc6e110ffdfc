// C3's geometry query as a traversal stage of its own:
// what would splitting the sphere-grid walk out of the path megakernel buy?
//
// The megakernel walks C3's 25^3 grid inside the persistent DFS loop, at the
// occupancy its per-lane DFS stack and frame column allow (4 waves per SIMD,
// 156 B of LDS per lane). A split design would have the path stage emit ray
// records and a traversal kernel -- no DFS stack, only the walk's 8-byte slot
// per lane in LDS -- return the nearest hit. This probe measures that
// traversal kernel alone on the megakernel's own ray stream:
//
//  1. the product source built with -DIPT_RAYLOG=1 renders part of the C3
//     frame and logs every k-th finished sphere-list trace (origin, direction,
//     the walk's t and hit) -- the rays and results the real kernel produced;
//  2. walk_split_kernel re-traces the logged rays with the same functions
//     (trace_box_planes_only, sphere_grid_init, sphere_grid_walk_wave), one
//     ray per lane, lanes refilled from a queue, at a chosen occupancy, and
//     counts the rays whose (t bits, hit) differ from the log (must be 0).
//
// Build (CPU container): bash scripts/probes/build_walk_split.sh
// Run: python scripts/probes/walk_split.py (GPU box)
#include "../../ipt_amd/csrc/ipt_kernels.hip"

extern "C" int probe_raylog_arm(unsigned long long cap, unsigned every) {
    if (g_raylog) return 0;
    if (hipMalloc(&g_raylog, cap * sizeof(RayLogRec)) != hipSuccess) return -1;
    if (hipMalloc(&g_raylog_n, sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMemset(g_raylog_n, 0, sizeof(unsigned long long)) != hipSuccess) return -1;
    g_raylog_cap = cap;
    g_raylog_every = every ? every : 1;
    return 0;
}

// traces seen by the logging launches, and records held
extern "C" int probe_raylog_count(unsigned long long* seen, unsigned long long* held) {
    unsigned long long n = 0;
    if (!g_raylog_n || hipMemcpy(&n, g_raylog_n, sizeof n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    *seen = n;
    const unsigned long long h = (n + g_raylog_every - 1) / g_raylog_every;
    *held = h < g_raylog_cap ? h : g_raylog_cap;
    return 0;
}

// out: [0] rays whose result differs from the log, [1] cells walked, [2] item
// tests (COUNT), [3] rays traced
template <int WPS, bool COUNT>
__global__ __launch_bounds__(256, WPS) void walk_split_kernel(KParams kp, const RayLogRec* __restrict__ rays,
                                                              unsigned long long n, unsigned long long* next,
                                                              unsigned long long* out, int budget) {
    extern __shared__ unsigned long long wslots[];  // 8 B per lane (+ occupancy padding)
    const int tid = threadIdx.x, lane = tid & 63;
    unsigned long long* slots = wslots + (tid & ~63);
    bool tracing = false, pool = true;
    vec3 o = v3(0, 0, 0), d = v3(0, 0, 1), tmx = v3(0, 0, 0);
    int cell = -1, bidx = -1;
    float best = 0.0f;
    unsigned long long my = 0, bad = 0, done = 0;
    unsigned long long pnext = 0, pend = 0;  // the wave's claimed chunk [pnext, pend)
    constexpr unsigned long long kChunk = 256;
    uint32_t c_nodes = 0, c_tests = 0;
    for (;;) {
        // idle lanes take the next rays from the wave's chunk of the queue (one
        // atomic per kChunk rays, like the megakernel's work pool)
        const uint64_t idle = __ballot(!tracing);
        if (pool && idle) {
            const unsigned long long cnt = (unsigned long long)__popcll(idle), avail = pend - pnext;
            unsigned long long nb = 0;
            if (cnt > avail) {
                const int leader = __ffsll((long long)idle) - 1;
                if (lane == leader) nb = atomicAdd(next, (unsigned long long)kChunk);
                nb = __shfl(nb, leader);
            }
            if (!tracing) {
                const unsigned long long r = (unsigned long long)__popcll(idle & ((1ull << lane) - 1));
                my = r < avail ? pnext + r : nb + (r - avail);
                if (my < n) {
                    const RayLogRec rr = rays[my];
                    o = v3(rr.o[0], rr.o[1], rr.o[2]);
                    d = v3(rr.d[0], rr.d[1], rr.d[2]);
                    int xp = -1;
                    best = (IPT_BOXDIV && kp.box_inrange) ? trace_box_planes_only<true>(o, d, &xp)
                                                          : trace_box_planes_only<false>(o, d, &xp);
                    bidx = -2 - xp;
                    sphere_grid_init(kp, o, d, cell, tmx);
                    tracing = true;
                }
            }
            if (cnt > avail) {
                pnext = nb + (cnt - avail);
                pend = nb + kChunk;
            } else {
                pnext += cnt;
            }
            pool = pnext < n;  // (chunks are claimed in increasing order)
        }
        if (!__ballot(tracing)) break;
        sphere_grid_walk_wave<COUNT>(kp, tracing, o, d, cell, tmx, best, bidx, budget, slots, lane, nullptr,
                                     c_nodes, c_tests IPT_DIAG_NULL_ARGS);
        if (tracing && cell < 0) {
            tracing = false;
            const int hit = bidx >= 0 ? grid_item_index(kp, bidx) : bidx;
            const RayLogRec& r = rays[my];
            bad += (__float_as_uint(best) != __float_as_uint(r.t) || hit != r.hit) ? 1u : 0u;
            ++done;
        }
    }
    if (bad) atomicAdd(&out[0], bad);
    if (COUNT) {
        atomicAdd(&out[1], (unsigned long long)c_nodes);
        atomicAdd(&out[2], (unsigned long long)c_tests);
    }
    atomicAdd(&out[3], done);
}

template <int WPS, bool COUNT>
static int run_walk(ipt_ctx* ctx, unsigned long long n, int wgs_per_cu, int budget, float* ms,
                    unsigned long long* out_h) {
    KParams kp{};
    kp.box_inrange = ctx->box_inrange;
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
    kp.grid_items = ctx->d_grid_items;
    kp.grid_c4 = ctx->d_grid_c4;
    kp.grid_idx = ctx->d_grid_c4 ? reinterpret_cast<const int*>(ctx->d_grid_c4 + ctx->grid_n_items) : nullptr;
    kp.grid_cells = ctx->d_grid_cells;
    if (kp.n_grid <= 0) return -3;
    unsigned long long *next = nullptr, *out = nullptr;
    if (hipMalloc(&next, 8) != hipSuccess || hipMalloc(&out, 32) != hipSuccess) return -1;
    hipMemset(next, 0, 8);
    hipMemset(out, 0, 32);
    // the CU's LDS split over wgs_per_cu workgroups caps the occupancy at
    // wgs_per_cu x 4 waves (the VGPR cap WPS permitting)
    const size_t lds = std::max<size_t>(256 * 8, (size_t)(160 * 1024) / (size_t)wgs_per_cu - 256);
    auto fn = walk_split_kernel<WPS, COUNT>;
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return -4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(fn, dim3((unsigned)(ctx->n_cu * wgs_per_cu)), dim3(256), lds, 0, kp, g_raylog, n, next, out,
                       budget);
    hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return -2;
    hipEventElapsedTime(ms, e0, e1);
    hipMemcpy(out_h, out, 32, hipMemcpyDeviceToHost);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipFree(next);
    hipFree(out);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// wps: the kernel's __launch_bounds__ waves per SIMD (4: <= 128 VGPRs, 8: <= 64)
extern "C" int probe_walk(ipt_ctx* ctx, int wps, int count, int wgs_per_cu, int budget, unsigned long long n,
                          float* ms, unsigned long long* out4) {
    if (!g_raylog) return -5;
    if (wps == 4) return count ? run_walk<4, true>(ctx, n, wgs_per_cu, budget, ms, out4)
                               : run_walk<4, false>(ctx, n, wgs_per_cu, budget, ms, out4);
    if (wps == 6) return count ? run_walk<6, true>(ctx, n, wgs_per_cu, budget, ms, out4)
                               : run_walk<6, false>(ctx, n, wgs_per_cu, budget, ms, out4);
    if (wps == 8) return count ? run_walk<8, true>(ctx, n, wgs_per_cu, budget, ms, out4)
                               : run_walk<8, false>(ctx, n, wgs_per_cu, budget, ms, out4);
    return -6;
}
