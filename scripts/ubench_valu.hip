// Profiling-only microbenchmark: chip-wide throughput of the instruction
// classes the path kernel is made of (IEEE f32 divide/sqrt, 32x32->64 integer
// multiply used by Philox, f64 ops, selects). Full occupancy, 8 independent
// chains per lane, results consumed so nothing is dead.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o ubench scripts/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int kIters = 4096;

#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(256) void bench(float* out, uint32_t seed) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    float f[CHAINS];
    uint32_t u[CHAINS];
    double d[CHAINS];
    typedef float f2_t __attribute__((ext_vector_type(2)));
    f2_t v[CHAINS];
    for (int c = 0; c < CHAINS; ++c) {
        f[c] = 1.0f + (float)((t * 7 + c) & 255) * 1e-3f;
        u[c] = t * 2654435761u + c + seed;
        d[c] = 1.0 + (double)c * 1e-3;
        v[c] = f2_t{f[c], f[c] * 0.5f};
    }
    const float g = 1.0000001f + (float)(seed & 1);
    const f2_t g2 = f2_t{g, g * 0.999f};
    const uint32_t m = 0xD2511F53u + seed;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (OP == 0) f[c] = f[c] + g;                                  // v_add_f32
            if (OP == 1) f[c] = __builtin_fmaf(f[c], g, 0.5f);             // v_fma_f32
            if (OP == 2) f[c] = g / f[c];                                  // IEEE f32 divide
            if (OP == 3) f[c] = __builtin_sqrtf(f[c]) + g;                 // IEEE sqrtf (+add)
            if (OP == 4) {                                                 // 32x32->64 (Philox)
                const uint64_t p = (uint64_t)u[c] * m;
                u[c] = (uint32_t)(p >> 32) ^ (uint32_t)p;
            }
            if (OP == 5) u[c] = __umulhi(u[c], m) + c;                     // v_mul_hi_u32 (+add)
            if (OP == 6) u[c] = u[c] * m + c;                              // v_mul_lo_u32 (+add)
            if (OP == 7) d[c] = d[c] * 1.0000001;                          // v_mul_f64
            if (OP == 8) d[c] = __builtin_fma(d[c], 1.0000001, 1e-9);      // v_fma_f64
            if (OP == 9) f[c] = __builtin_amdgcn_rcpf(f[c]);               // v_rcp_f32
            if (OP == 10) u[c] = u[c] ^ (u[c] >> 3);                       // 2 int ops
            if (OP == 11) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v[c]) : "v"(g2));   // packed: 2 lanes-ops each
            if (OP == 12) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(v[c]) : "v"(g2));
            if (OP == 13) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(v[c]) : "v"(g2));
            if (OP == 14) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "v"(g));        // asm baseline
        }
    }
    float acc = 0.0f;
    for (int c = 0; c < CHAINS; ++c) acc += f[c] + (float)u[c] + (float)d[c] + v[c].x + v[c].y;
    out[t] = acc;
}

template <int OP>
void run(const char* name, int ops_per_iter, float* out, int grid, int waves_per_simd = 8) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(bench<OP>, dim3(grid), dim3(256), 0, 0, out, 0u);
    hipEventRecord(a);
    hipLaunchKernelGGL(bench<OP>, dim3(grid), dim3(256), 0, 0, out, 0u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double lane_ops = (double)grid * 256 * kIters * CHAINS * ops_per_iter;
    // wave64 instructions per SIMD-cycle at 2.4 GHz, 1024 SIMDs
    const double per_simd_cycle = lane_ops / 64.0 / (ms * 1e-3 * 2.4e9 * 1024);
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"T_lane_ops\": %.2f, \"cycles_per_wave_op\": %.2f}\n", name,
           waves_per_simd, ms, lane_ops / (ms * 1e-3) / 1e12, 1.0 / per_simd_cycle);
}

int main() {
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * 256 * 32);
    const int grid = 256 * 32;  // 32 blocks of 4 waves per CU: 8 waves/SIMD
    run<0>("v_add_f32", 1, out, grid);
    run<1>("v_fma_f32", 1, out, grid);
    run<2>("f32 divide (IEEE)", 1, out, grid);
    run<3>("sqrtf (IEEE) + add", 1, out, grid);
    run<4>("u32*u32->u64 + xor", 1, out, grid);
    run<5>("mul_hi_u32 + add", 1, out, grid);
    run<6>("mul_lo_u32 + add", 1, out, grid);
    run<7>("v_mul_f64", 1, out, grid);
    run<8>("v_fma_f64", 1, out, grid);
    run<9>("v_rcp_f32", 1, out, grid);
    run<10>("xor+shift", 1, out, grid);
    // packed f32 (2 lane-ops per lane per instruction), 8 and 4 waves per SIMD
    for (int w : {8, 4}) {
        const int gr = 256 * 4 * w;
        run<14>("v_add_f32 (asm)", 1, out, gr, w);
        run<11>("v_pk_add_f32", 2, out, gr, w);
        run<12>("v_pk_mul_f32", 2, out, gr, w);
        run<13>("v_pk_fma_f32", 2, out, gr, w);
    }
    hipFree(out);
    return 0;
}
