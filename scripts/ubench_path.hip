// Profiling-only microbenchmark: cost of each path primitive (ipt_path.h /
// ipt_math.h) in SIMD-cycles per wave64 call at full occupancy, on inputs of
// the kind the path kernel feeds it. Guides where the kernel's VALU time goes.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
//          -I ipt_amd/csrc -o scripts/ubench_path scripts/ubench_path.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "ipt_path.h"

using namespace ipt;

constexpr int kIters = 256;

__device__ __forceinline__ float sink(float a, float b) { return a + b * 1e-30f; }

template <int OP>
__global__ __launch_bounds__(256) void bench(float* out, float seed) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    // per-lane inputs: a unit normal, a ray inside the box, two uniforms
    float u1 = (float)((t * 2654435761u) >> 8) * 0x1p-24f, u2 = (float)((t * 40503u + 7u) & 0xffffff) * 0x1p-24f;
    float acc = 0.0f;
    LightDev L = make_light(v3(0.1f, -0.9f, -0.15f), v3(0.0f, 0.2f, 0.0f), v3(0.2f, 0.0f, 0.0f), 1.0f, 0);
    for (int i = 0; i < kIters; ++i) {
        const float a = u1 * 2.0f - 1.0f, b = u2 * 2.0f - 1.0f;
        const vec3 o = v3(a * 0.9f, b * 0.9f, 0.3f * a + seed);
        const vec3 d = normalize(v3(b + 0.01f, 0.7f, -a - 0.2f));
        if (OP == 0) {  // baseline: the input generation alone
            acc = sink(acc, o.x + d.y);
        } else if (OP == 1) {
            const Frame f = make_frame(d);
            acc = sink(acc, f.m0.x + f.m1.y + f.m2.z + f.iz.x);
        } else if (OP == 2) {
            acc = sink(acc, acos_f64_to_f32_exact(a));
        } else if (OP == 3) {
            acc = sink(acc, acos_f64_to_f32(a));
        } else if (OP == 4) {
            acc = sink(acc, acosf_(u1));
        } else if (OP == 5) {
            float s, c;
            sincosf_small_(u1 * 3.0f, &s, &c);
            acc = sink(acc, s + c);
        } else if (OP == 6) {
            const vec3 v = cosine_sample_local(u1, u2);
            acc = sink(acc, v.x + v.y + v.z);
        } else if (OP == 7) {
            int p;
            acc = sink(acc, trace_box(o, d, &p) + (float)p);
        } else if (OP == 8) {
            vec3 h;
            const bool hit = light_trace(L, o, d, &h);
            acc = sink(acc, h.x + (hit ? 1.0f : 0.0f));
        } else if (OP == 9) {
            vec3 h = o + d;
            acc = sink(acc, light_pdf(L, o, true, h));
        } else if (OP == 10) {
            const vec3 n = normalize(o + d);
            acc = sink(acc, n.x + n.y + n.z);
        } else if (OP == 11) {
            const u32x4 r = philox4x32_10(t, (uint32_t)i, 3u, 0u, 0x1234u, 0x5678u);
            acc = sink(acc, (float)(r.v[0] ^ r.v[1] ^ r.v[2] ^ r.v[3]));
        } else if (OP == 12) {
            acc = sink(acc, o.x / d.y);
        } else if (OP == 13) {
            acc = sink(acc, sqrt_(u1 + 0.5f));
        } else if (OP == 14) {
            acc = sink(acc, length(o - d));
        } else if (OP == 15) {
            const vec3 v = light_sample_dir(L, o, u1, u2);
            acc = sink(acc, v.x + v.y + v.z);
        }
        u1 = u1 * 0.5f + 0.25f + acc * 1e-30f;
        u2 = u2 * 0.75f + 0.1f;
    }
    out[t] = acc;
}

template <int OP>
double run(const char* name, float* out, int grid, double base) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(bench<OP>, dim3(grid), dim3(256), 0, 0, out, 0.0f);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(bench<OP>, dim3(grid), dim3(256), 0, 0, out, 0.0f);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double wave_calls = (double)grid * 4 * kIters;  // 4 waves per block
    const double cyc = ms * 1e-3 * 2.4e9 * 1024 / wave_calls;
    printf("{\"op\": \"%s\", \"ms\": %.3f, \"simd_cycles_per_wave_call\": %.1f, \"minus_baseline\": %.1f}\n", name,
           ms, cyc, cyc - base);
    return cyc;
}

int main() {
    float* out;
    (void)hipMalloc(&out, sizeof(float) * 256 * 256 * 16);
    const int grid = 256 * 16;  // 16 blocks of 4 waves per CU: 4 waves/SIMD, as the path kernel
    const double base = run<0>("baseline (input generation)", out, grid, 0.0);
    run<1>("make_frame (fast acos)", out, grid, base);
    run<2>("acos f64->f32 exact (fdlibm)", out, grid, base);
    run<3>("acos f64->f32 fast (Ziv)", out, grid, base);
    run<4>("acosf (glibc float)", out, grid, base);
    run<5>("sincosf small", out, grid, base);
    run<6>("cosine_sample_local", out, grid, base);
    run<7>("trace_box", out, grid, base);
    run<8>("light_trace", out, grid, base);
    run<9>("light_pdf (hit)", out, grid, base);
    run<10>("normalize", out, grid, base);
    run<11>("philox4x32_10", out, grid, base);
    run<12>("f32 divide", out, grid, base);
    run<13>("sqrtf", out, grid, base);
    run<14>("length", out, grid, base);
    run<15>("light_sample_dir", out, grid, base);
    (void)hipFree(out);
    return 0;
}
