// Where random gathers into a table of a given size are served (DESIGN.md §6,
// the path kernel's ~120 memory-side reads per path go to
// the 64 MiB CosineDdf r table and the 1 GiB frame-angle table). Each lane
// runs a dependent chain of 4-byte gathers at hashed indices into a table of
// S MiB (the next index depends on the loaded word, so every gather waits for
// the previous one) and the kernel reports the mean time per gather, for
// S = 1 MiB .. 4 GiB, at 1 wave per CU (unloaded latency) and 16 waves per CU
// (loaded, like the path kernel's 4 waves per SIMD). Latency plateaus show the
// level that serves each size: L2 (4 MiB per XCD), the Infinity Cache (256 MiB
// memory-side), HBM. Build: hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_gather scripts/ubench_gather.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ void fill(uint32_t* t, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        t[i] = mix((uint32_t)i * 2654435761u);
}

__global__ void chase(const uint32_t* __restrict__ t, uint32_t mask, int steps, unsigned long long* ticks,
                      uint32_t* sink) {
    uint32_t idx = mix(blockIdx.x * blockDim.x + threadIdx.x) & mask;
    uint32_t acc = 0;
    const unsigned long long t0 = wall_clock64();
    for (int s = 0; s < steps; ++s) {
        const uint32_t v = t[idx];
        acc += v;
        idx = mix(idx ^ v) & mask;
    }
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) atomicAdd(ticks, t1 - t0);
    if (acc == 0x12345678u) sink[0] = idx;  // keeps the chain alive
}

int main() {
    int khz = 0, ncu = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t max_bytes = (size_t)4 << 30;
    uint32_t* t = nullptr;
    if (hipMalloc(&t, max_bytes) != hipSuccess) return 1;
    hipLaunchKernelGGL(fill, dim3(ncu * 8), dim3(256), 0, 0, t, max_bytes / 4);
    unsigned long long* ticks;
    uint32_t* sink;
    hipMalloc(&ticks, 8);
    hipMalloc(&sink, 4);
    hipDeviceSynchronize();
    const int steps = 2000;
    for (int waves_per_cu : {1, 16}) {
        for (size_t mib : {1, 2, 4, 16, 64, 128, 256, 512, 1024, 4096}) {
            const uint32_t mask = (uint32_t)((mib << 20) / 4 - 1);
            const int blocks = ncu * waves_per_cu;
            hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, t, mask, 200, ticks, sink);  // warm
            hipMemset(ticks, 0, 8);
            hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, t, mask, steps, ticks, sink);
            unsigned long long h = 0;
            hipMemcpy(&h, ticks, 8, hipMemcpyDeviceToHost);
            const double ns = (double)h / blocks / steps / khz * 1e6;
            std::printf("{\"waves_per_cu\": %d, \"table_MiB\": %zu, \"ns_per_dependent_gather\": %.1f}\n", waves_per_cu,
                        mib, ns);
        }
    }
    hipFree(t);
    return 0;
}
