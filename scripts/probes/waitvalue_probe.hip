// Probe: hipStreamWaitValue64 on plain device memory and on signal memory,
// and device atomics on signal memory (for the tail-overlap gating).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void spin_then_add(unsigned long long* ctr, long long ticks) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        long long t0 = wall_clock64();
        while (wall_clock64() - t0 < ticks) {}
        atomicAdd(ctr, 100ull);
    }
}
__global__ void stamp(unsigned long long* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = (unsigned long long)wall_clock64();
}
__global__ void many_atomics(unsigned long long* ctr, int n) {
    for (int i = 0; i < n; ++i) atomicAdd(ctr, 1ull);
}

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int test(const char* name, unsigned long long* ctr) {
    hipStream_t a, b;
    hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    unsigned long long* out;
    hipMalloc(&out, 16);
    hipMemset(out, 0, 16);
    hipMemcpy(ctr, &(const unsigned long long&)0ull, 8, hipMemcpyDefault);
    hipPointerAttribute_t at{};
    hipPointerGetAttributes(&at, ctr);
    std::printf("%s: memoryType %d\n", name, (int)at.type);
    hipError_t e = hipStreamWaitValue64(b, ctr, 100, hipStreamWaitValueGte, ~0ull);
    std::printf("%s: hipStreamWaitValue64 -> %s\n", name, hipGetErrorString(e));
    if (e != hipSuccess) return 1;
    hipLaunchKernelGGL(stamp, 1, 64, 0, b, out + 1);
    auto t = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(spin_then_add, 1, 64, 0, a, ctr, 50000000LL);  // 0.5 s of the 100 MHz wall clock
    hipLaunchKernelGGL(stamp, 1, 64, 0, a, out);
    hipStreamSynchronize(a);
    double ta = ms_since(t);
    hipError_t eb = hipStreamSynchronize(b);
    double tb = ms_since(t);
    unsigned long long h[2];
    hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
    std::printf("%s: stream a done %.1f ms, b done %.1f ms (%s); b stamp - a stamp = %lld ticks\n", name, ta, tb,
                hipGetErrorString(eb), (long long)(h[1] - h[0]));
    // atomics rate on this memory
    hipMemcpy(ctr, &(const unsigned long long&)0ull, 8, hipMemcpyDefault);
    t = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(many_atomics, 256, 64, 0, a, ctr, 16);
    hipStreamSynchronize(a);
    unsigned long long v = 0;
    hipMemcpy(&v, ctr, 8, hipMemcpyDefault);
    std::printf("%s: 262144 atomics in %.2f ms, value %llu\n", name, ms_since(t), v);
    return 0;
}

int main() {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    int wv = 0, rate = 0;
    hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    std::printf("wall clock %d kHz\n", rate);
    hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, 0);
    std::printf("CanUseStreamWaitValue %d\n", wv);
    unsigned long long* dev = nullptr;
    hipMalloc(&dev, 8);
    test("hipMalloc", dev);
    // (hipMallocSignalMemory is host memory here (memoryType 1): a kernel's
    // atomicAdd on it never released the waiting stream within 30 s on the
    // MI355X box, so the library gates on device memory only)
    return 0;
}
