// ipt_math.h — portable, bit-reproducible arithmetic for the ipt path tracer.
//
// Compiled by hipcc for BOTH the gfx950 device code and the host side of the
// product library (same source, same operation order, -ffp-contract=off), so
// a value computed on the GPU is bit-identical to the value the host side of
// the library computes for the exhaustive math tests.
//
// What it reproduces:
//  * glm 0.9.9.7 vec3/mat3 arithmetic in glm's operation order
//    (reference include/glm/detail/func_geometric.inl:8-90,
//     detail/type_mat3x3.inl:468-474, detail/func_matrix.inl:268-291,
//     ext/matrix_transform.inl:18-47).
//  * the libm functions the reference calls on its hot path, as shipped in the
//    image's glibc 2.35 (x86_64, FMA/AVX2 ifunc variants that the reference
//    binary binds to on any FMA-capable host):
//      acosf  -> fdlibm __ieee754_acosf   (float ops, no FMA)
//      sinf/cosf/sincosf -> ARM optimized-routines sinf/cosf (__sinf_fma,
//                 __cosf_fma: double-precision polynomial, FMA-contracted
//                 exactly where GCC contracted glibc's source)
//      (float)acos((double)x) -> fdlibm __ieee754_acos restated in double;
//                 only its rounding to float is used by the reference
//                 (libddf/ddf_detail.h:82) and that rounding is verified equal
//                 to glibc's for every float input in tests/.
//    Constants were read from the image's libm.so.6 .rodata and the operation
//    graphs from its disassembly; tests/test_math_exhaustive.py checks every
//    float input of each function's reachable domain against the host libm.
#pragma once

#include <stdint.h>

#ifndef IPT_HD
#define IPT_HD __host__ __device__ inline
#endif

namespace ipt {

// ---------------------------------------------------------------- bit casts
IPT_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
IPT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
IPT_HD uint64_t d2u(double d) { return __builtin_bit_cast(uint64_t, d); }
IPT_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

IPT_HD float fabs_(float x) { return u2f(f2u(x) & 0x7fffffffu); }
IPT_HD bool isfinite_(float x) { return (f2u(x) & 0x7f800000u) != 0x7f800000u; }
IPT_HD float inf_() { return u2f(0x7f800000u); }
IPT_HD double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
IPT_HD double sqrtd_(double x) { return __builtin_sqrt(x); }

// IEEE f32 sqrt and division: the device compiler's own sequences. (Wave-
// guarded variants that drop their range handling measured neutral (sqrt) and
// -12 % (division: the guard and its branch cost more than v_div_scale /
// v_div_fixup); the range-free cores below are used only where a host or
// algebraic proof bounds the operands.)
IPT_HD float sqrt_(float x) { return __builtin_sqrtf(x); }
IPT_HD float div_(float a, float b) { return a / b; }

// a/b without the range handling of the compiler's sequence (no v_div_scale /
// v_div_fmas / v_div_fixup): the reciprocal, one Newton step and ONE quotient
// residual step (round 5; two before). Bit-identical to a/b when |a| in
// [2^-40, 2^41) or a = +-0 (then a signed zero, whose sign the callers never
// observe) and |b| in [2^-40, 2^41). Why one residual step suffices: the
// Newton step makes y = RN(1/b) (exhaustively, fn 17 below), and with y the
// correctly rounded reciprocal and q0 = RN(a*y) within an ulp of a/b, q0 +
// y*RN(a - b*q0) (the residual exact by fma) is the correctly rounded quotient
// in the absence of over/underflow (Markstein's theorem for fma division).
// Device checks: ipt_math_selfcheck fn 10 (2^32 hashed pairs over the range)
// and fn 20 (2^32 pairs with divisors of all-ones-like significands, the
// theorem's hard case), 0 mismatches. Callers must guarantee the range.
IPT_HD float div_inrange_(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
    float y = __builtin_amdgcn_rcpf(b);
    y = __builtin_fmaf(__builtin_fmaf(-b, y, 1.0f), y, y);
    const float q0 = a * y;
    return __builtin_fmaf(__builtin_fmaf(-b, q0, a), y, q0);
#else
    return a / b;
#endif
}

// 1/b by the hardware reciprocal and Newton corrections: STEPS = 1 (y1) or 2
// (y2) of the corrections that the round-4 div_inrange_(1.0f, b) applied (y1,
// then q1 == y2, then q2). ipt_math_selfcheck fn 17 / 18 compare them with
// that three-correction sequence over all 2^32 floats: both are identical to
// it bit for bit everywhere (round 5, `profiles/round5_rcp_check.txt`), so
// rcp_inrange_ below takes one correction instead of three.
template <int STEPS>
IPT_HD float rcp_newton_(float b) {
#if defined(__HIP_DEVICE_COMPILE__)
    float y = __builtin_amdgcn_rcpf(b);
    y = __builtin_fmaf(__builtin_fmaf(-b, y, 1.0f), y, y);
    if (STEPS >= 2) y = __builtin_fmaf(__builtin_fmaf(-b, y, 1.0f), y, y);
    return y;
#else
    return 1.0f / b;
#endif
}
// == the three-correction 1.0f / b for every float b (exhaustive device check above)
IPT_HD float rcp_inrange_(float b) { return rcp_newton_<1>(b); }

// Correctly rounded sqrtf for x = +0 or in [2^-96, 2^126): the hardware root (within
// one ulp, no denormal scaling needed in this range) corrected by the signs of
// the residuals of its two neighbours (the sequence of the IEEE expansion
// without its range handling). Equal to sqrtf on every float of the range
// (exhaustive GPU check, math probe 13).
IPT_HD float sqrt_inrange_(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = u2f(f2u(s) - 1u), su = u2f(f2u(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    const float s1 = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : s1;
#else
    return __builtin_sqrtf(x);
#endif
}

// ------------------------------------------------------------------ vec3
// glm::vec3 with glm's component-wise operators; no FMA anywhere.
struct vec3 {
    float x, y, z;
};
IPT_HD vec3 v3(float x, float y, float z) { vec3 r; r.x = x; r.y = y; r.z = z; return r; }
IPT_HD vec3 operator+(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
IPT_HD vec3 operator-(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
IPT_HD vec3 operator-(vec3 a) { return v3(-a.x, -a.y, -a.z); }
IPT_HD vec3 operator*(vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
IPT_HD vec3 operator*(float s, vec3 a) { return v3(s * a.x, s * a.y, s * a.z); }
IPT_HD bool is_zero(vec3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
// glm compute_dot<vec3>: tmp = a*b; tmp.x + tmp.y + tmp.z   (func_geometric.inl:48-55)
IPT_HD float dot(vec3 a, vec3 b) {
    float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
    return (tx + ty) + tz;
}
// glm compute_cross (func_geometric.inl:68-79)
IPT_HD vec3 cross(vec3 x, vec3 y) {
    return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
// glm length = sqrt(dot(v,v)) (func_geometric.inl:8-14)
IPT_HD float length(vec3 v) { return sqrt_(dot(v, v)); }
// glm normalize = v * inversesqrt(dot(v,v)), inversesqrt = 1/sqrt (func_exponential.inl:136-139)
IPT_HD vec3 normalize(vec3 v) {
    float s = div_(1.0f, sqrt_(dot(v, v)));
    return v * s;
}

// normalize for dot(v, v) in [2^-80, 2^80] (root in [2^-40, 2^40]): the same
// roundings as normalize() through the range-free root and quotient
IPT_HD vec3 normalize_inrange_(vec3 v) {
    const float s = rcp_inrange_(sqrt_inrange_(dot(v, v)));
    return v * s;
}

// column-major mat3, m[c][r] as glm
struct mat3 {
    vec3 c[3];
};
// glm mat3 * vec3 (type_mat3x3.inl:468-474): row i = (m0i*vx + m1i*vy) + m2i*vz
IPT_HD vec3 mul(const mat3& m, vec3 v) {
    return v3(m.c[0].x * v.x + m.c[1].x * v.y + m.c[2].x * v.z,
              m.c[0].y * v.x + m.c[1].y * v.y + m.c[2].y * v.z,
              m.c[0].z * v.x + m.c[1].z * v.y + m.c[2].z * v.z);
}
IPT_HD float el(const mat3& m, int c, int r) {
    const vec3& v = m.c[c];
    return r == 0 ? v.x : (r == 1 ? v.y : v.z);
}
// glm compute_inverse<3,3> (func_matrix.inl:268-291), cofactor / determinant
template <bool INRANGE = false>
IPT_HD mat3 inverse(const mat3& M) {
    const float m00 = M.c[0].x, m01 = M.c[0].y, m02 = M.c[0].z;
    const float m10 = M.c[1].x, m11 = M.c[1].y, m12 = M.c[1].z;
    const float m20 = M.c[2].x, m21 = M.c[2].y, m22 = M.c[2].z;
    float det = m00 * (m11 * m22 - m21 * m12);
    det = det - m10 * (m01 * m22 - m21 * m02);
    det = det + m20 * (m01 * m12 - m11 * m02);
    // glm writes "+ m00*(..) - m10*(..) + m20*(..)"; unary + is exact
    const float o = INRANGE ? rcp_inrange_(det) : div_(1.0f, det);  // INRANGE: det in [2^-40, 2^41)
    mat3 I;
    I.c[0].x = (m11 * m22 - m21 * m12) * o;
    I.c[1].x = -(m10 * m22 - m20 * m12) * o;
    I.c[2].x = (m10 * m21 - m20 * m11) * o;
    I.c[0].y = -(m01 * m22 - m21 * m02) * o;
    I.c[1].y = (m00 * m22 - m20 * m02) * o;
    I.c[2].y = -(m00 * m21 - m20 * m01) * o;
    I.c[0].z = (m01 * m12 - m11 * m02) * o;
    I.c[1].z = -(m00 * m12 - m10 * m02) * o;
    I.c[2].z = (m00 * m11 - m10 * m01) * o;
    return I;
}

// ------------------------------------------------------------------ acosf
// glibc 2.35 sysdeps/ieee754/flt-32/e_acosf.c (fdlibm), constants verified
// against libm.so.6 .rodata (0x9c958..0x9c98c).
// Branch-free over fdlibm's three argument ranges: every lane evaluates the
// exact operation sequence of its own branch (selects only pick results), so
// the value is the glibc one while a wave pays one division/sqrt chain, not
// three (the |x|<0.5 and x>0.5 ranges both occur within every wave).
IPT_HD float acosf_(float x) {
    const float one = 1.0f;
    const float pi = u2f(0x40490fdau);
    const float pio2_hi = u2f(0x3fc90fdau);
    const float pio2_lo = u2f(0x33a22168u);
    const float two_pio2_lo = u2f(0x34222168u);  // (float)2.0*pio2_lo, folded by GCC
    const float pS0 = u2f(0x3e2aaaabu), pS1 = -u2f(0x3ea6b090u), pS2 = u2f(0x3e4e0aa8u),
                pS3 = -u2f(0x3d241146u), pS4 = u2f(0x3a4f7f04u), pS5 = u2f(0x3811ef08u);
    const float qS1 = -u2f(0x4019d139u), qS2 = u2f(0x4001572du), qS3 = -u2f(0x3f303361u),
                qS4 = u2f(0x3d9dc62eu);
    const uint32_t hx = f2u(x);
    const uint32_t ix = hx & 0x7fffffffu;
    const bool small = ix < 0x3f000000u;  // |x| < 0.5
    const bool neg = (int32_t)hx < 0;     // x < -0.5 when !small
    const float z = small ? x * x : (neg ? (one + x) * 0.5f : (one - x) * 0.5f);
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = div_(p, q);
    const float sq = sqrt_(z);
    const float r_small = pio2_hi - (x - (pio2_lo - x * r));
    const float r_neg = pi - 2.0f * (sq + (r * sq - pio2_lo));
    const float df = u2f(f2u(sq) & 0xfffff000u);
    const float c = div_(z - df * df, sq + df);
    const float r_pos = 2.0f * (df + (r * sq + c));
    float res = small ? r_small : (neg ? r_neg : r_pos);
    if (small && ix <= 0x32800000u) res = pio2_hi + pio2_lo;
    if (ix == 0x3f800000u) res = (int32_t)hx > 0 ? 0.0f : pi + two_pio2_lo;
    if (ix > 0x3f800000u) res = (x - x) * inf_();  // |x|>1 or NaN: NaN
    return res;
}

// ------------------------------------------------------------ sinf / cosf
// ARM optimized-routines single-precision sin/cos as built into glibc 2.35
// (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h) in its FMA ifunc
// variant. Table __sincosf_table read from libm .rodata 0xb30c0.
struct sincos_tab {
    double c0, c1, s1, c2, s2, c3, s3, c4;
};
IPT_HD sincos_tab sincos_table(int which) {
    sincos_tab t;
    const double sg = which ? -1.0 : 1.0;
    t.c0 = sg * 1.0;
    t.c1 = sg * u2d(0xbfdffffffd0c621cull);
    t.s1 = u2d(0xbfc555545995a603ull);
    t.c2 = sg * u2d(0x3fa55553e1068f19ull);
    t.s2 = u2d(0x3f81107605230bc4ull);
    t.c3 = sg * u2d(0xbf56c087e89a359dull);
    t.s3 = u2d(0xbf2994eb3774cf24ull);
    t.c4 = sg * u2d(0x3ef99343027bf8c3ull);
    return t;
}
IPT_HD double sincos_sign(int q) { return (q == 1 || q == 2) ? -1.0 : 1.0; }
IPT_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ffu; }

// sin polynomial on reduced x (n even) — __sinf_fma @7b359 / @7b2e0
IPT_HD float sin_poly_(double x, double x2, const sincos_tab& p) {
    double s1 = fma_(x2, p.s3, p.s2);
    double x3 = x2 * x;
    double x7 = x2 * x3;
    double s = fma_(x3, p.s1, x);
    return (float)fma_(s1, x7, s);
}
// cos polynomial on reduced x (n odd for sin) — __sinf_fma @7b388
IPT_HD float cos_poly_(double x2, const sincos_tab& p) {
    double x4 = x2 * x2;
    double c1 = fma_(x2, p.c1, p.c0);
    double c2 = fma_(x2, p.c4, p.c3);
    double x6 = x2 * x4;
    double c = fma_(x4, p.c2, c1);
    return (float)fma_(c2, x6, c);
}

// reduce_large (sincosf.h) with __inv_pio4 (libm .rodata 0xb3060)
IPT_HD double reduce_large_(uint32_t xi, int* np) {
    const uint32_t inv_pio4[24] = {
        0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
        0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
        0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
        0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
    const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * u2d(0x3c1921fb54442d18ull);  // pi * 2^-62
}

// fast reduction: n = round(x*2/pi) via (int)(x*hpi_inv*2^24) + 2^23 >> 24; x - n*hpi (one FMA)
IPT_HD double reduce_fast_(double x, int* np) {
    const double hpi_inv = u2d(0x41645f306dc9c883ull);  // 0x1.45f306dc9c883p+23
    double r = x * hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma_(-(double)n, u2d(0x3ff921fb54442d18ull), x);
}

IPT_HD void sincosf_small_(float y, float* sp, float* cp);
IPT_HD float sinf_(float y) {
    double x = y;
    if (abstop12(y) < abstop12(120.0f)) {
        float sv, cv;
        sincosf_small_(y, &sv, &cv);
        return sv;
    } else if (abstop12(y) < abstop12(u2f(0x7f800000u))) {
        uint32_t xi = f2u(y);
        int sign = xi >> 31;
        int n;
        x = reduce_large_(xi, &n);
        double s = sincos_sign((n + sign) & 3);
        sincos_tab p = sincos_table(((n + sign) & 2) ? 1 : 0);
        double x2 = x * x;
        if ((n & 1) == 0) return sin_poly_(x * s, x2, p);
        return cos_poly_(x2, p);
    }
    return (y - y) / (y - y);
}

IPT_HD float cosf_(float y) {
    double x = y;
    if (abstop12(y) < abstop12(120.0f)) {
        float sv, cv;
        sincosf_small_(y, &sv, &cv);
        return cv;
    } else if (abstop12(y) < abstop12(u2f(0x7f800000u))) {
        uint32_t xi = f2u(y);
        int sign = xi >> 31;
        int n;
        x = reduce_large_(xi, &n);
        double s = sincos_sign((n + sign) & 3);
        sincos_tab p = sincos_table(((n + sign) & 2) ? 1 : 0);
        double x2 = x * x;
        if (n & 1) return sin_poly_(x * s, x2, p);
        return cos_poly_(x2, p);
    }
    return (y - y) / (y - y);
}

// sin and cos of the same argument sharing one reduction, for |y| < 120
// (every argument the path tracer produces: rotation angles in [0,pi],
// CosineDdf angles in [0,pi/2] and [0,2pi)). Equal bit-for-bit to
// sinf_/cosf_ there (glibc's __sincosf_fma SLP-vectorises the same FMA graph;
// tests/test_math_exhaustive.py checks the equality against host sincosf).
// Branch-free: for |y| < pi/4 glibc skips the reduction, but reduce_fast_
// then yields n = 0 and x - 0*hpi == x exactly (fma with a -0 product), i.e.
// the same polynomial inputs; only |y| < 2^-12 needs a select.
//
// The quadrant's signs are applied last: glibc selects sign-flipped cosine
// coefficients (sg * c_i, sincos_table) and multiplies x by s = +-1; every
// FMA of the cosine polynomial has all-sign-flipped operands and the sine
// polynomial is odd in x, and round-to-nearest is symmetric, so the results
// are exactly sg * cos_poly(c_i) and s * sin_poly(x): two sign flips of the
// float results instead of selected f64 constants (same bits for every input).
IPT_HD void sincosf_small_(float y, float* sp, float* cp) {
    int n;
    const double x = reduce_fast_((double)y, &n);
    const sincos_tab p = sincos_table(0);
    const double x2 = x * x;
    const uint32_t s_neg = ((n & 3) == 1 || (n & 3) == 2) ? 0x80000000u : 0u;  // sincos_sign(n & 3)
    const uint32_t g_neg = (n & 2) ? 0x80000000u : 0u;                         // sincos_table's sg
    const float a = u2f(f2u(sin_poly_(x, x2, p)) ^ s_neg);
    const float b = u2f(f2u(cos_poly_(x2, p)) ^ g_neg);
    const bool tiny = abstop12(y) < abstop12(0x1p-12f);
    *sp = tiny ? y : ((n & 1) ? b : a);
    *cp = tiny ? 1.0f : ((n & 1) ? a : b);
}
IPT_HD void sincosf_(float y, float* sp, float* cp) {
    if (abstop12(y) < abstop12(120.0f)) {
        sincosf_small_(y, sp, cp);
        return;
    }
    *sp = sinf_(y);
    *cp = cosf_(y);
}
// sinf for |y| < 120 (same arithmetic as sinf_ there)
IPT_HD float sinf_small_(float y) {
    float sv, cv;
    sincosf_small_(y, &sv, &cv);
    return sv;
}

// ------------------------------------------------- (float)acos((double)x)
// fdlibm e_acos.c (double). Used only through its rounding to float; the
// equality of that rounding with glibc's acos for all float inputs in [-1,1]
// is checked exhaustively in tests/test_math_exhaustive.py.
IPT_HD double acos_d_(double x) {
    const double pi = u2d(0x400921fb54442d18ull);
    const double pio2_hi = u2d(0x3ff921fb54442d18ull);
    const double pio2_lo = u2d(0x3c91a62633145c07ull);
    const double pS0 = u2d(0x3fc5555555555555ull), pS1 = u2d(0xbfd4d61203eb6f7dull),
                 pS2 = u2d(0x3fc9c1550e884455ull), pS3 = u2d(0xbfa48228b5688f3bull),
                 pS4 = u2d(0x3f49efe07501b288ull), pS5 = u2d(0x3f023de10dfdf709ull);
    const double qS1 = u2d(0xc0033a271c8a2d4bull), qS2 = u2d(0x40002ae59c598ac8ull),
                 qS3 = u2d(0xbfe6066c1b8d0159ull), qS4 = u2d(0x3fb3b8c5b12e9282ull);
    const uint64_t hx64 = d2u(x);
    const uint32_t hx = (uint32_t)(hx64 >> 32);
    const uint32_t ix = hx & 0x7fffffffu;
    // branch-free over fdlibm's three ranges (see acosf_)
    const bool small = ix < 0x3fe00000u;
    const bool neg = (int32_t)hx < 0;
    const double z = small ? x * x : (neg ? (1.0 + x) * 0.5 : (1.0 - x) * 0.5);
    const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const double r = p / q;
    const double sq = sqrtd_(z);
    const double r_small = pio2_hi - (x - (pio2_lo - x * r));
    const double r_neg = pi - 2.0 * (sq + (r * sq - pio2_lo));
    const double df = u2d(d2u(sq) & 0xffffffff00000000ull);
    const double c = (z - df * df) / (sq + df);
    const double r_pos = 2.0 * (df + (r * sq + c));
    double res = small ? r_small : (neg ? r_neg : r_pos);
    if (small && ix <= 0x3c600000u) res = pio2_hi + pio2_lo;
    if (ix >= 0x3ff00000u) {
        if (((ix - 0x3ff00000u) | (uint32_t)hx64) == 0)
            res = (int32_t)hx > 0 ? 0.0 : pi + 2.0 * pio2_lo;
        else
            res = (x - x) * (double)inf_();
    }
    return res;
}
IPT_HD float acos_f64_to_f32_exact(float x) { return (float)acos_d_((double)x); }

// RotateDdf's angle (float)acos((double)x) (ddf_detail.h:82), fast device path.
// acos_d_ costs two IEEE f64 divisions and an IEEE f64 sqrt, each a long
// correction sequence on gfx950. Here fdlibm's formulas are evaluated with the
// hardware f64 reciprocal / reciprocal-sqrt refined by Newton steps (relative
// error of A a few 1e-16), and the float rounding of A is accepted when A(1-d)
// and A(1+d), d = 2^-44, round to the same float: rounding is monotonic, so
// the exact value and fdlibm's (both within d of A) round there too (Ziv's
// test). Otherwise, and for |x| >= 1, the exact restatement decides. Equal to
// acos_f64_to_f32_exact on every float (device self-check over all 2^32
// inputs, tests/test_gpu_parity.py::test_fast_acos_exhaustive).
IPT_HD float acos_f64_to_f32(float xf) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double x = (double)xf;
    const double ax = __builtin_fabs(x);
    const double pi = u2d(0x400921fb54442d18ull);
    const double pio2_hi = u2d(0x3ff921fb54442d18ull);
    const double pio2_lo = u2d(0x3c91a62633145c07ull);
    const double pS0 = u2d(0x3fc5555555555555ull), pS1 = u2d(0xbfd4d61203eb6f7dull),
                 pS2 = u2d(0x3fc9c1550e884455ull), pS3 = u2d(0xbfa48228b5688f3bull),
                 pS4 = u2d(0x3f49efe07501b288ull), pS5 = u2d(0x3f023de10dfdf709ull);
    const double qS1 = u2d(0xc0033a271c8a2d4bull), qS2 = u2d(0x40002ae59c598ac8ull),
                 qS3 = u2d(0xbfe6066c1b8d0159ull), qS4 = u2d(0x3fb3b8c5b12e9282ull);
    const bool small = ax < 0.5;
    const double z = small ? x * x : (1.0 - ax) * 0.5;
    const double p = z * __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                         __builtin_fma(z, pS5, pS4), pS3), pS2), pS1), pS0);
    const double q = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, qS4, qS3), qS2), qS1), 1.0);
    double y = __builtin_amdgcn_rcp(q);
    y = __builtin_fma(y, __builtin_fma(-q, y, 1.0), y);
    y = __builtin_fma(y, __builtin_fma(-q, y, 1.0), y);
    const double r = p * y;
    // sqrt(z) by Goldschmidt from rsq (z in (0, 0.25] off the small branch)
    const double zs = small ? 0.25 : z;
    const double g0 = __builtin_amdgcn_rsq(zs);
    double sg = zs * g0, h = 0.5 * g0;
    double t = __builtin_fma(-sg, h, 0.5);
    sg = __builtin_fma(sg, t, sg);
    h = __builtin_fma(h, t, h);
    t = __builtin_fma(-sg, sg, zs);
    sg = __builtin_fma(t, h, sg);
    double A;
    if (small)
        A = pio2_hi - (x - (pio2_lo - x * r));
    else if (x < 0.0)
        A = pi - 2.0 * (sg + (r * sg - pio2_lo));
    else
        A = 2.0 * (sg + r * sg);
    const double d = u2d(0x3d30000000000000ull);  // 2^-44
    const float lo = (float)(A * (1.0 - d)), hi = (float)(A * (1.0 + d));
    if (lo == hi && ax < 1.0) return lo;
    return (float)acos_d_(x);
#else
    return acos_f64_to_f32_exact(xf);
#endif
}

// --------------------------------------------------- mixed-precision helpers
// The reference compares floats against the double literal 1e-6
// (geometric_utils.cpp:14,23,45-48; lighting.cpp:116,120). For a float f,
// (double)f < 1e-6 <=> f < 0x358637be (the smallest float above 1e-6 is
// 0x358637be; float(1e-6) = 0x358637bd < 1e-6).
IPT_HD bool lt_1em6(float f) { return f < u2f(0x358637beu); }

// CosineDdf::value (ddf.cpp:232-238): (float)((double)z / M_PI).
// For every float z in [0, 2], (float)(z * (double)(1/M_PI)) rounds to the
// same float as the f64 quotient (checked exhaustively against host libm in
// tests/test_math_exhaustive.py::test_mixed_precision_helpers), so the f64
// division is a multiply. The reference only reaches z in [0, 1+2^-22]
// (z = (inverse*d).z with |d| = 1 and an orthonormal inverse).
IPT_HD float div_pi_to_f32(float z) { return (float)((double)z * u2d(0x3fd45f306dc9c883ull)); }

// CosineDdf::sample phi (ddf.cpp:228): (float)(2*M_PI*(double)u2)
IPT_HD float two_pi_times(float u) { return (float)(u2d(0x401921fb54442d18ull) * (double)u); }
// two_pi_times(u01(g << 8)) for a 24-bit g: u = g 2^-24 exactly, so the double
// product 2pi * u is RN(2pi * g * 2^-24) = RN((2pi 2^-24) * g) -- the same
// real product, the constant scaled by a power of two -- from g directly
IPT_HD float two_pi_times_u24(uint32_t g) { return (float)(u2d(0x3e9921fb54442d18ull) * (double)g); }

// ------------------------------------------------------------ RNG (Philox)
// Philox4x32-10 (Salmon et al., SC'11; Random123 constants).
struct u32x4 {
    uint32_t v[4];
};
IPT_HD void mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    *lo = (uint32_t)p;
}
// a ^ b ^ c: one v_bitop3_b32 (truth table 0x96) on gfx950
IPT_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}
IPT_HD u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                           uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#if defined(__HIP_DEVICE_COMPILE__)
    // the round keys are two scalar adds each: keep them in the loop, where
    // they cost SALU slots, instead of hoisted and spilled to VGPR lanes
    // (every reload a v_readlane + hazard nops on the VALU)
    asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo32(M0, c0, &hi0, &lo0);
        mulhilo32(M1, c2, &hi1, &lo1);
        uint32_t n0 = xor3(hi1, c1, k0);
        uint32_t n2 = xor3(hi0, c3, k1);
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += W0;
        k1 += W1;
    }
    u32x4 out;
    out.v[0] = c0;
    out.v[1] = c1;
    out.v[2] = c2;
    out.v[3] = c3;
    return out;
}
// uniform float in [0,1): top 24 bits * 2^-24 (never 1.0, so randf.h's retry
// loop at include/randf.h:8-9 never fires)
IPT_HD float u01(uint32_t w) { return (float)(w >> 8) * 5.9604644775390625e-08f; }

}  // namespace ipt
