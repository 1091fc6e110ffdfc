// ipt_post.hip — the reference's image post-process on the GPU (SURVEY.md
// §8(f) row 2), bit-exact:
//   GridRenderPlane::smooth(side) / computeSmoothedMax(side)
//                                  (src/GridRenderPlane.cpp:10-59)
//   Gui's glare bloom               (src/gui.cpp:28-52: draw_halo + glare)
//
// smooth: the reference filters in place, walking y and x downwards from the
// bottom-right corner and reading pixels (y-yy, x-xx), yy, xx < side. Every
// pixel it reads is at or above-left of the one it writes and is written later
// (or is the same pixel, read before the write), so the in-place filter equals
// an out-of-place one: one thread per pixel, the side*side sum in the
// reference's order (yy outer, xx inner, float adds), accum /= side*side.
// The running max starts at 0 and takes `accum > max` (NaN never wins).
//
// glare: out = img; for every pixel with !(val <= cutoff), in raster order,
// coef = (float)(0.1*val/cutoff) (f64), C = cutoff*coef, and every output
// pixel gets += C/(0.25+r)/(0.25+r) (float) with r = (float)hypot(dx, dy);
// then out.cut(0, cutoff). Per output pixel the halos are added in the
// bright pixels' raster order, so one thread per output pixel walking the
// bright list (staged through LDS) reproduces the sequence. (float)hypot of
// two ints equals sqrtf((float)(dx^2+dy^2)) while the sum < 2^24 and
// (float)sqrt((double)sum) above (checked against glibc for all |dx|,|dy| <
// 4096, tests/test_post.py); images are limited to 4096 x 4096 accordingly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/ipt_capi.h"
#include "ipt_internal.h"
#include "ipt_math.h"

namespace {

using namespace ipt;

constexpr int kPostBlock = 256;

__global__ __launch_bounds__(kPostBlock) void smooth_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                            int W, int H, int side, unsigned int* max_bits) {
    const int x = blockIdx.x * kPostBlock + threadIdx.x, y = blockIdx.y;
    float cand = 0.0f;
    if (x < W && x >= side - 1 && y >= side - 1) {
        float accum = 0.0f;
        for (int yy = 0; yy < side; ++yy) {
            const float* row = in + (size_t)(y - yy) * W + x;
            for (int xx = 0; xx < side; ++xx) accum += row[-xx];
        }
        accum = accum / (float)((unsigned)side * (unsigned)side);  // size_t -> float, exact below 2^24
        if (out) out[(size_t)y * W + x] = accum;
        cand = accum > 0.0f ? accum : 0.0f;  // `if (accum > max_value)` with max_value >= 0
    }
    // block max of non-negative floats: their bit patterns order as integers
    __shared__ unsigned int red[kPostBlock / 64];
    unsigned int m = __float_as_uint(cand);
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned int b = red[0];
        for (int i = 1; i < kPostBlock / 64; ++i) b = max(b, red[i]);
        if (b) atomicMax(max_bits, b);
    }
}

struct Bright {
    int x, y;
    float c;  // C = cutoff * coef
    int pad;
};

constexpr int kGlareChunk = 512;

__global__ __launch_bounds__(kPostBlock) void glare_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                           int W, int H, const Bright* __restrict__ bright, int nb,
                                                           float cutoff) {
    __shared__ Bright tile[kGlareChunk];
    const int x = blockIdx.x * kPostBlock + threadIdx.x, y = blockIdx.y;
    const bool live = x < W;
    float v = live ? in[(size_t)y * W + x] : 0.0f;
    const float r0 = 0.25f;
    for (int base = 0; base < nb; base += kGlareChunk) {
        const int n = min(kGlareChunk, nb - base);
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += kPostBlock) tile[i] = bright[base + i];
        __syncthreads();
        if (live)
            for (int i = 0; i < n; ++i) {
                const int dx = x - tile[i].x, dy = y - tile[i].y;  // |dx|, |dy| < 4096
                const unsigned int s = (unsigned int)(dx * dx + dy * dy);
                const float r = s < (1u << 24) ? __builtin_sqrtf((float)s) : (float)__builtin_sqrt((double)s);
                const float val = (tile[i].c / (r0 + r)) / (r0 + r);
                v = v + val;
            }
    }
    if (live) out[(size_t)y * W + x] = v < 0.0f ? 0.0f : (v > cutoff ? cutoff : v);  // cimg::cut
}

using ipt_internal::DevBuf;

#define POSTCHECK(ctx, expr)                                                                             \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            return ipt_internal::ctx_fail(ctx, IPT_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

extern "C" {

int ipt_smooth(ipt_ctx* ctx, float* pixels, int width, int height, int side, int in_place, float* max_value) {
    if (!ctx) return IPT_E_INVALID;
    if (!pixels || !max_value || width <= 0 || height <= 0 || side < 0 || side > 4096)
        return ipt_internal::ctx_fail(ctx, IPT_E_INVALID, "ipt_smooth: bad arguments");
    if (side == 1)  // GridRenderPlane.cpp:14: `y >= side-1` with size_t never fails, the loop runs past row 0
        return ipt_internal::ctx_fail(ctx, IPT_E_UNSUPPORTED,
                                      "ipt_smooth: side 1 is undefined behaviour in the reference");
    (void)hipSetDevice(ipt_internal::ctx_device(ctx));
    hipStream_t st = ipt_internal::ctx_stream(ctx);
    const size_t n = (size_t)width * height;
    DevBuf<float> din, dout;
    DevBuf<unsigned int> dmax;
    POSTCHECK(ctx, hipMalloc(&din.p, n * sizeof(float)));
    POSTCHECK(ctx, hipMalloc(&dmax.p, sizeof(unsigned int)));
    if (in_place) POSTCHECK(ctx, hipMalloc(&dout.p, n * sizeof(float)));
    POSTCHECK(ctx, hipMemcpyAsync(din.p, pixels, n * sizeof(float), hipMemcpyHostToDevice, st));
    if (in_place) POSTCHECK(ctx, hipMemcpyAsync(dout.p, din.p, n * sizeof(float), hipMemcpyDeviceToDevice, st));
    POSTCHECK(ctx, hipMemsetAsync(dmax.p, 0, sizeof(unsigned int), st));
    if (side >= 2 && side <= width && side <= height) {
        dim3 grid((width + kPostBlock - 1) / kPostBlock, height);
        hipLaunchKernelGGL(smooth_kernel, grid, dim3(kPostBlock), 0, st, din.p, dout.p, width, height, side, dmax.p);
        POSTCHECK(ctx, hipGetLastError());
    }
    unsigned int mb = 0;
    POSTCHECK(ctx, hipMemcpyAsync(&mb, dmax.p, sizeof mb, hipMemcpyDeviceToHost, st));
    if (in_place) POSTCHECK(ctx, hipMemcpyAsync(pixels, dout.p, n * sizeof(float), hipMemcpyDeviceToHost, st));
    POSTCHECK(ctx, hipStreamSynchronize(st));
    *max_value = __builtin_bit_cast(float, mb);
    return IPT_OK;
}

int ipt_glare(ipt_ctx* ctx, const float* in, float* out, int width, int height, float cutoff) {
    if (!ctx) return IPT_E_INVALID;
    if (!in || !out || width <= 0 || height <= 0)
        return ipt_internal::ctx_fail(ctx, IPT_E_INVALID, "ipt_glare: bad arguments");
    if (width > 4096 || height > 4096)  // the hypot equivalence is proven for |dx|, |dy| < 4096
        return ipt_internal::ctx_fail(ctx, IPT_E_UNSUPPORTED, "ipt_glare: images up to 4096 x 4096");
    (void)hipSetDevice(ipt_internal::ctx_device(ctx));
    hipStream_t st = ipt_internal::ctx_stream(ctx);
    // bright pixels in raster order (gui.cpp:40-47); `val <= cutoff` false for NaN too
    std::vector<Bright> b;
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) {
            const float val = in[(size_t)y * width + x];
            if (val <= cutoff) continue;
            const float coef = (float)(0.1 * (double)val / (double)cutoff);
            b.push_back(Bright{x, y, cutoff * coef, 0});
        }
    const size_t n = (size_t)width * height;
    DevBuf<float> din, dout;
    DevBuf<Bright> db;
    POSTCHECK(ctx, hipMalloc(&din.p, n * sizeof(float)));
    POSTCHECK(ctx, hipMalloc(&dout.p, n * sizeof(float)));
    POSTCHECK(ctx, hipMalloc(&db.p, std::max<size_t>(b.size(), 1) * sizeof(Bright)));
    POSTCHECK(ctx, hipMemcpyAsync(din.p, in, n * sizeof(float), hipMemcpyHostToDevice, st));
    if (!b.empty())
        POSTCHECK(ctx, hipMemcpyAsync(db.p, b.data(), b.size() * sizeof(Bright), hipMemcpyHostToDevice, st));
    dim3 grid((width + kPostBlock - 1) / kPostBlock, height);
    hipLaunchKernelGGL(glare_kernel, grid, dim3(kPostBlock), 0, st, din.p, dout.p, width, height, db.p, (int)b.size(),
                       cutoff);
    POSTCHECK(ctx, hipGetLastError());
    POSTCHECK(ctx, hipMemcpyAsync(out, dout.p, n * sizeof(float), hipMemcpyDeviceToHost, st));
    POSTCHECK(ctx, hipStreamSynchronize(st));
    return IPT_OK;
}

}  // extern "C"
