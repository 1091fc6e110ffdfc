// ipt_path.h — per-ray building blocks of the reference estimator, restated
// for the gfx950 megakernel (and compiled for the host side of the library,
// which uses them to precompute scene constants with identical arithmetic).
//
// Every function cites the reference lines it reproduces. All arithmetic is
// in the reference's order; the build uses -ffp-contract=off.
#pragma once

#include "ipt_math.h"

#include <vector>

namespace ipt {

constexpr int kMaxLights = 1024;

// ------------------------------------------------------------- scene (device)
struct LightDev {
    vec3 P;        // Light::position (corner)
    vec3 x, y;     // x_axis, y_axis
    vec3 n;        // normalize(cross(x_axis, y_axis))         lighting.cpp:126,141
    mat3 inv;      // inverse(mat3(x, y, cross(x,y)))          lighting.cpp:87-89
    float area;    // |cross| or |cross|/2                     lighting.cpp:84-85
    float spow;    // power/area                               lighting.cpp:102,142
    int type;      // 0 diamond, 1 triangle
    int pad;
};

// Rotation frame of a RotateDdf(CosineDdf, to) (ddf_detail.h:72-85):
// sample = M * x, value = CosineDdf::value(inverse * d) needs only row 2 of
// the inverse.
struct Frame {
    vec3 m0, m1, m2;  // columns of M
    vec3 iz;          // (inv[0][2], inv[1][2], inv[2][2])
};

// RotateDdf constructor (ddf_detail.h:73-84) incl. glm::rotate
// (ext/matrix_transform.inl:18-47) applied to identity and mat3(mat4):
// make_frame = frame_angle_sc + make_frame_sc.
//
// glm::rotate's cos(a), sin(a) of a = (float)acos((double)dot(z, to))
// (ddf_detail.h:82), a in [0, pi]
IPT_HD void frame_angle_sc(vec3 to, float* s, float* c) {
    const float cosinus = dot(v3(0.0f, 0.0f, 1.0f), to);
    const float a = acos_f64_to_f32(cosinus);
    sincosf_small_(a, s, c);
}
// The frame from `to` and the angle's (s, c) (make_frame below, or an exact
// table of frame_angle_sc by to.z's bits in the path kernel).
// INRANGE: `to` has unit length up to rounding (a normalized vector), so the
// axis test, both roots and both quotients (|axis| = 1 or >= 1e-6, det ~ 1)
// take the range-free sequences (same roundings, see sqrt_inrange_).
template <bool INRANGE = false>
IPT_HD Frame make_frame_sc(vec3 to, float s, float c) {
    const vec3 z = v3(0.0f, 0.0f, 1.0f);
    vec3 axis = cross(z, to);
    vec3 ax;
    if (INRANGE) {
        // length(axis) < 1e-6 is certain below 2^-80 (root 2^-40), where the
        // range-free root is not used; normalize(axis) reuses the root (the
        // replacement (1,0,0) has dot 1 and root 1)
        const float q = dot(axis, axis);
        const float r = sqrt_inrange_(q);
        const bool rep = (q < 0x1p-80f) | lt_1em6(r);
        axis = rep ? v3(1.0f, 0.0f, 0.0f) : axis;
        ax = axis * rcp_inrange_(rep ? 1.0f : r);
    } else {
        if (lt_1em6(length(axis))) axis = v3(1.0f, 0.0f, 0.0f);
        ax = normalize(axis);
    }
    const vec3 temp = (1.0f - c) * ax;
    float R[3][3];
    R[0][0] = c + temp.x * ax.x;
    R[0][1] = temp.x * ax.y + s * ax.z;
    R[0][2] = temp.x * ax.z - s * ax.y;
    R[1][0] = temp.y * ax.x - s * ax.z;
    R[1][1] = c + temp.y * ax.y;
    R[1][2] = temp.y * ax.z + s * ax.x;
    R[2][0] = temp.z * ax.x + s * ax.y;
    R[2][1] = temp.z * ax.y - s * ax.x;
    R[2][2] = c + temp.z * ax.z;
    // Result[k] = m[0]*R[k][0] + m[1]*R[k][1] + m[2]*R[k][2] with m = identity(4)
    mat3 M;
    for (int k = 0; k < 3; ++k) {
        float e0 = (1.0f * R[k][0] + 0.0f * R[k][1]) + 0.0f * R[k][2];
        float e1 = (0.0f * R[k][0] + 1.0f * R[k][1]) + 0.0f * R[k][2];
        float e2 = (0.0f * R[k][0] + 0.0f * R[k][1]) + 1.0f * R[k][2];
        M.c[k] = v3(e0, e1, e2);
    }
    const mat3 I = inverse<INRANGE>(M);
    Frame f;
    f.m0 = M.c[0];
    f.m1 = M.c[1];
    f.m2 = M.c[2];
    f.iz = v3(I.c[0].z, I.c[1].z, I.c[2].z);
    return f;
}
// make_frame_sc<true> without its zero terms. glm's cross((0,0,1), to) has
// z = 0*to.y - to.x*0, so ax.z and temp.z are signed zeros; glm::rotate's
// product with the identity adds 0*R terms to every entry. For finite x,
// x + (+-0) == x and (+-0) - x == -x whenever x != 0, so when all nine
// rotation entries R are non-zero (and `to` is finite) every dropped term only
// met a non-zero partner and the frame is bit-identical to make_frame_sc<true>.
// `ok` reports that condition; the caller takes the exact path otherwise
// (axis replaced by (1,0,0), to.x or to.y zero, an underflowed product).
IPT_HD Frame make_frame_sc_fast(vec3 to, float s, float c, bool& ok) {
    const float axx = -to.y, axy = to.x;  // cross((0,0,1), to).xy when non-zero
    const float q = axx * axx + axy * axy;
    const float r = sqrt_inrange_(q);
    const float inv = rcp_inrange_(r);
    const float ax = axx * inv, ay = axy * inv;
    const float omc = 1.0f - c;
    const float tx = omc * ax, ty = omc * ay;
    const float r00 = c + tx * ax, r01 = tx * ay, r02 = -(s * ay);
    const float r10 = ty * ax, r11 = c + ty * ay, r12 = s * ax;
    const float r20 = s * ay, r21 = -(s * ax), r22 = c;
    // q >= 2^-80 and r >= 1e-6: the exact path's axis is not replaced; q
    // finite: `to` is finite (a NaN/inf component reaches q)
    // (|r20| = |r02| and |r21| = |r12|: negations of the same products)
    const float mn = fminf(fminf(fminf(fabs_(r00), fabs_(r01)), fminf(fabs_(r02), fabs_(r10))),
                           fminf(fminf(fabs_(r11), fabs_(r12)), fabs_(r22)));
    ok = (mn > 0.0f) & (q >= 0x1p-80f) & (q < inf_()) & !lt_1em6(r);
    mat3 M;
    M.c[0] = v3(r00, r01, r02);
    M.c[1] = v3(r10, r11, r12);
    M.c[2] = v3(r20, r21, r22);
    const mat3 I = inverse<true>(M);
    Frame f;
    f.m0 = M.c[0];
    f.m1 = M.c[1];
    f.m2 = M.c[2];
    f.iz = v3(I.c[0].z, I.c[1].z, I.c[2].z);
    return f;
}
template <bool INRANGE = false>
IPT_HD Frame make_frame(vec3 to) {
    float s, c;
    frame_angle_sc(to, &s, &c);
    return make_frame_sc<INRANGE>(to, s, c);
}
IPT_HD vec3 frame_apply(const Frame& f, vec3 v) {
    return v3(f.m0.x * v.x + f.m1.x * v.y + f.m2.x * v.z,
              f.m0.y * v.x + f.m1.y * v.y + f.m2.y * v.z,
              f.m0.z * v.x + f.m1.z * v.y + f.m2.z * v.z);
}
// TransformDdf::value -> CosineDdf::value (ddf_detail.h:74-76, ddf.cpp:232-238)
IPT_HD float frame_cosine_value(const Frame& f, vec3 d) {
    const float z = f.iz.x * d.x + f.iz.y * d.y + f.iz.z * d.z;
    if (z < 0.0f) return 0.0f;
    return div_pi_to_f32(z);
}

// CosineDdf::sample (ddf.cpp:223-231) in local coordinates
IPT_HD vec3 cosine_sample_local(float u1, float u2) {
    const float cos_alpha = sqrt_(u1);
    const float alpha = acosf_(cos_alpha);
    const float phi = two_pi_times(u2);
    const float r = sinf_small_(alpha);
    float sp, cp;
    sincosf_small_(phi, &sp, &cp);
    return v3(r * cp, r * sp, cos_alpha);
}

// --------------------------------------------------------------- geometry
// intersection_with_box_plane (geometric_utils.cpp:8-26) for plane = sgn*e_a.
// dot(d, sgn*e_a) == sgn*d_a and dot(o, sgn*e_a) == sgn*o_a exactly whenever
// the result is used (the discarded zero products only change the sign of a
// zero, and a zero dot is rejected by the |.|<1e-6 test); d is finite.
// INRANGE: the caller guarantees |o| < 2^39 componentwise; then the numerator
// 1 - sgn*oa is 0 or in [2^-24, 2^40) (1 - oa is exact near 1) and the divisor
// in [1e-6, 2): the range-free division is exact (div_inrange_); a zero
// numerator gives t = +-0, rejected below either way.
// Branch-free: the reference's early returns (here and in the area-light
// test and pdf below) are one select over every test (same comparisons, same
// arithmetic, so the same result for every input incl. NaN); in a wave that
// mixes passing and failing lanes the branches only cost exec-mask
// bookkeeping (+3.3 % C2 when introduced).
template <bool INRANGE = false>
IPT_HD float box_plane_t(float oa, float da, float sgn, vec3 o, vec3 d) {
    const float dp = sgn * da;
    const float t = INRANGE ? div_inrange_(1.0f - sgn * oa, dp) : div_(1.0f - sgn * oa, dp);
    const float px = o.x + d.x * t, py = o.y + d.y * t, pz = o.z + d.z * t;
    const bool miss = lt_1em6(fabs_(dp)) | (fabs_(px) > 1.0f) | (fabs_(py) > 1.0f) | (fabs_(pz) > 1.0f) |
                      (dp < 0.0f) | lt_1em6(t);
    return miss ? inf_() : t;
}

// intersection_with_sphere (geometric_utils.cpp:28-55). The f64 expression
// (float)((-2.0*b -+ sqrt_desc)/2.0) equals (-2b -+ sqrt_desc)*0.5f in f32:
// both operands are floats, so the f64 difference is exact whenever it can
// affect the f32 rounding (see DESIGN.md "mixed precision").
// BF: branch-free (the box's one sphere, hit by a large share of rays); the
// sphere lists' tests stay branchy (most miss at the discriminant)
// INR (the box sphere, r = 0.5, |o| < 2^39): desc = 4*fl(A - B), A = fl(b*b),
// B = fl(dot(o,o) - 0.25), and sd through the range-free root. B is 0 or
// |B| >= 2^-26 (for dot(o,o) in [1/8, 1/2] the difference is exact and a
// multiple of 2^-26), so a nonzero A - B is >= 2^-49 unless B = 0: 4*(A - B)
// is then never subnormal and equals the reference's fl(4A - 4B). desc lies in
// (0, 2^-96), outside the root's range, only when B = 0 and A < 2^-98, i.e.
// |b| < 2^-48: sd < 2^-45 with either root, both roots fall below 1e-6 and the
// test misses either way. desc is never -0 (A >= +0); desc < 2^84.
template <bool BF = false, bool INR = false>
IPT_HD float sphere_t(float radius, vec3 o, vec3 d) {
    const float b = dot(o, d);
    const float desc = INR ? 4.0f * (b * b - (dot(o, o) - radius * radius))
                                               : 4.0f * (b * b) - 4.0f * (dot(o, o) - radius * radius);
    if (BF) {
        const float sd = INR ? sqrt_inrange_(desc) : sqrt_(desc);
        const float m2b = -2.0f * b;
        float t1 = (m2b - sd) * 0.5f;
        float t2 = (m2b + sd) * 0.5f;
        t1 = lt_1em6(t1) ? inf_() : t1;
        t2 = lt_1em6(t2) ? inf_() : t2;
        const float t = (t2 < t1) ? t2 : t1;
        const vec3 pos = o + d * t;
        const bool back = dot(pos, o - pos) <= 0.0f;
        return (desc < 0.0f) ? inf_() : ((t == inf_()) ? t : (back ? inf_() : t));
    }
    if (desc < 0.0f) return inf_();
    const float sd = sqrt_(desc);
    const float m2b = -2.0f * b;
    float t1 = (m2b - sd) * 0.5f;
    float t2 = (m2b + sd) * 0.5f;
    if (lt_1em6(t1)) t1 = inf_();
    if (lt_1em6(t2)) t2 = inf_();
    const float t = (t2 < t1) ? t2 : t1;  // std::min(t1, t2)
    if (t == inf_()) return t;            // pos would be inf/nan; the test then keeps t
    const vec3 pos = o + d * t;
    if (dot(pos, o - pos) <= 0.0f) return inf_();
    return t;
}

// The facing plane of axis a (sgn chosen so that sgn*d_a > 0 unless d_a is a
// zero): dp = sgn*d_a equals |d_a| whenever |dp| >= 1e-6 (otherwise the test
// misses either way), so `dp < 0` never decides, and 1 - sgn*o_a is one
// rounding of an exact product, i.e. fma(-sgn, o_a, 1). Same t, same miss.
template <bool INRANGE>
IPT_HD float facing_plane_t(float oa, float da, float sgn, vec3 o, vec3 d) {
    const float dp = fabs_(da);
    const float num = __builtin_fmaf(-sgn, oa, 1.0f);
    const float t = INRANGE ? div_inrange_(num, dp) : div_(num, dp);
    const float px = o.x + d.x * t, py = o.y + d.y * t, pz = o.z + d.z * t;
    const bool miss =
        lt_1em6(dp) | (fabs_(px) > 1.0f) | (fabs_(py) > 1.0f) | (fabs_(pz) > 1.0f) | lt_1em6(t);
    return miss ? inf_() : t;
}

// GeometrySphereInBox::traceRay (GeometrySphereInBox.cpp:10-81) nearest hit:
// returns t (inf = miss) and the hit primitive: 0..4 = plane index in the
// reference's order {+x,+y,+z,-x,-z}, 5 = the r=0.5 sphere.
template <bool INRANGE = false>
IPT_HD float trace_box_planes_only(vec3 o, vec3 d, int* prim) {
    // a NaN direction fails every test (the reference returns no hit); the
    // planes are computed regardless and the result selected at the end
    const bool dnan = d.x + d.y + d.z != d.x + d.y + d.z;
    // x: the facing plane is +x (index 0) for d.x>0 and -x (index 3) otherwise
    const bool xp = d.x > 0.0f, zp = d.z > 0.0f;
    float best = facing_plane_t<INRANGE>(o.x, d.x, xp ? 1.0f : -1.0f, o, d);
    int bi = xp ? 0 : 3;
    const float ty0 = facing_plane_t<INRANGE>(o.y, d.y, 1.0f, o, d);
    const float ty = d.y > 0.0f ? ty0 : inf_();
    // the scan's "nearer, or as near with a lower index" as selects (bitwise
    // on the comparisons: no short-circuit control flow)
    const bool take_y = (ty < best) | ((ty == best) & (1 < bi) & (ty != inf_()));
    best = take_y ? ty : best;
    bi = take_y ? 1 : bi;
    const float tz = facing_plane_t<INRANGE>(o.z, d.z, zp ? 1.0f : -1.0f, o, d);
    const int iz = zp ? 2 : 4;
    const bool take_z = (tz < best) | ((tz == best) & (iz < bi) & (tz != inf_()));
    best = take_z ? tz : best;
    bi = take_z ? iz : bi;
    const bool none = dnan | (best == inf_());
    *prim = none ? -1 : bi;
    return dnan ? inf_() : best;
}
template <bool INRANGE = false>
IPT_HD float trace_box(vec3 o, vec3 d, int* prim) {
    int bi;
    float best = trace_box_planes_only<INRANGE>(o, d, &bi);
    const float ts = sphere_t<true, INRANGE>(0.5f, o, d);
    if (ts < best) { best = ts; bi = 5; }
    *prim = bi;
    return best;
}
// FractalSpheres' acceptance "std::abs(dist) > 1e-6" (double literal):
// |t| > 1e-6 <=> |t| > float(1e-6) = 0x358637bd.
IPT_HD bool gt_1em6(float f) { return f > u2f(0x358637bdu); }

// ----------------------------------------------------------------- lights
// Light types: 0 AreaLight diamond, 1 AreaLight triangle (lighting.cpp:79-144),
// 2 SphereLight, 3 PointLight, 4 InvertedSphereLight (lighting.h:31-73,
// lighting.cpp:146-207). Round lights keep the centre in P and the radius in x.x.

// SphereLight's own intersection_with_sphere (lighting.cpp:11-36), in the
// light's frame (o = origin - centre): float discriminant with dot(d, d), the
// roots in f64 from sqrtf(desc), rejection below 1e-6, and the front/back sign
// test. Returns t (inf = miss).
IPT_HD float round_light_t(float radius, vec3 o, vec3 d) {
    const float b = dot(o, d);
    const float dd = dot(d, d);
    const float desc = 4.0f * (b * b) - 4.0f * dd * (dot(o, o) - radius * radius);
    if (desc < 0.0f) return inf_();
    const double sd = (double)sqrt_(desc);
    float t1 = (float)((-2.0 * (double)b - sd) / 2.0 / (double)dd);
    float t2 = (float)((-2.0 * (double)b + sd) / 2.0 / (double)dd);
    if (lt_1em6(t1)) t1 = inf_();
    if (lt_1em6(t2)) t2 = inf_();
    const float t = (t2 < t1) ? t2 : t1;  // std::min(t1, t2)
    const vec3 pos = o + d * t;
    const vec3 outer_normal = normalize(pos);
    const float direction_sign = dot(outer_normal, o - pos);
    const float position_sign = length(o) - radius;
    if (direction_sign * position_sign <= 0.0f) return inf_();
    return t;  // inf when both roots were rejected (the NaN sign test passes it through)
}

// Light::traceRay: hit flag, position and the light's normal there.
//   AreaLight::traceRay (lighting.cpp:107-144);
//   SphereLight::traceRay (lighting.cpp:161-173), InvertedSphereLight flips
//   the normal (lighting.h:61-66), PointLight never hits (lighting.h:39-41).
// ROUND = false compiles the AreaLight code alone (scenes without round lights:
// the extra branch costs the C2 path kernel 12 % even when never taken).
template <bool ROUND = true>
IPT_HD bool light_trace(const LightDev& L, vec3 o, vec3 d, vec3* hit, vec3* nrm) {
    if (ROUND && L.type >= 2) {
        if (L.type == 3) return false;
        const float t = round_light_t(L.x.x, o - L.P, d);
        if (t == inf_()) return false;
        *hit = o + d * t;
        const vec3 n = normalize(*hit - L.P);
        *nrm = L.type == 4 ? -n : n;
        return true;
    }
    const float n_dir = dot(L.n, d);
    const float t = div_(dot(L.n, L.P - o), n_dir);
    const vec3 rel = (o + d * t) - L.P;
    const vec3 coord = mul(L.inv, rel);
    const bool in = L.type == 0 ? (coord.x >= 0.0f) & (coord.x <= 1.0f) & (coord.y >= 0.0f) & (coord.y <= 1.0f)
                                : (coord.x >= 0.0f) & (coord.y >= 0.0f) & (coord.x + coord.y <= 1.0f);
    *hit = L.P + rel;
    *nrm = L.n;
    return !(lt_1em6(fabs_(n_dir)) | (n_dir > 0.0f)) & !lt_1em6(t) & in;
}

// DdfFromLight::value for a direction whose light trace is `has`/`hit`/`nrm`
// (lighting.cpp:136-148).
IPT_HD float light_pdf(const LightDev& L, vec3 o, bool has, vec3 hit, vec3 nrm) {
    if (!has) return 0.0f;
    const vec3 dir = normalize(hit - o);
    const float cosinus = dot(nrm, -dir);
    const vec3 ho = hit - o;
    const float decay = dot(ho, ho);
    const float p = div_(div_(decay, cosinus), L.area);
    return cosinus < 0.0f ? 0.0f : p;  // the facing test as a select
}

// DdfFromLight::sample (lighting.cpp:125-134) via Light::sample:
//   AreaLight::sample (lighting.cpp:93-104);
//   SphereLight::sample (lighting.cpp:176-193): u1 = 2*randf()-1, acosf,
//   phi = (float)(2*M_PI*u2), sin/cos of phi fused to sincosf by GCC;
//   InvertedSphereLight flips the normal; PointLight::sample (lighting.cpp:
//   196-212): the normal is (sin a cos p, sin a sin p, u1), the point fixed.
// Returns vec3() when the sampled point faces away (cosinus < 1e-5f).
template <bool ROUND = true>
IPT_HD vec3 light_sample_dir(const LightDev& L, vec3 o, float u1, float u2raw) {
    vec3 pos, nrm;
    if (ROUND && L.type >= 2) {
        const float uc = u1 * 2.0f - 1.0f;
        const float alpha = acosf_(uc);
        const float phi = two_pi_times(u2raw);
        float sp, cp;
        sincosf_small_(phi, &sp, &cp);
        if (L.type == 3) {
            const float r = sinf_small_(alpha);
            nrm = v3(r * cp, r * sp, uc);
            pos = L.P;
        } else {
            const float r = L.x.x * sinf_small_(alpha);
            const vec3 q = v3(r * cp, r * sp, L.x.x * uc);
            pos = q + L.P;
            nrm = normalize(q);
            if (L.type == 4) nrm = -nrm;
        }
    } else {
        const float u2 = u2raw * (L.type == 1 ? 1.0f - u1 : 1.0f);
        pos = (L.x * u1 + L.y * u2) + L.P;
        nrm = L.n;
    }
    const vec3 dir = normalize(pos - o);
    const float cosinus = dot(nrm, -dir);
    if (cosinus < 1e-5f) return v3(0.0f, 0.0f, 0.0f);
    return dir;
}

// ---------------------------------------------- axis-aligned single AreaLight
// An AreaLight whose x_axis lies along coordinate axis XA, y_axis along YA and
// whose normal (hence cross(x, y)) lies along NA = 3 - XA - YA, with every
// other component of x, y, n and of the inverse matrix's coordinate rows an
// exact (signed) zero and every component of the corner P non-zero (host-
// checked: axis_aligned_light). Then every product with a zero component in the
// reference's dot/mul/sample expressions is a signed zero added to a term
// that is either non-zero (so it is an exact no-op) or compared against 0/1
// only (so the zero's sign cannot matter): the terms below are exactly the
// generic functions' results wherever those are observed.
template <int I>
IPT_HD float comp(vec3 v) {
    return I == 0 ? v.x : (I == 1 ? v.y : v.z);
}
// light_trace (AreaLight::traceRay, lighting.cpp:107-144), n.d and n.(P-o)
// reduced to their one non-zero term (a zero's sign only meets the |.| < 1e-6,
// > 0 and t < 1e-6 rejections), coord = inverse*rel reduced to the rows' one
// non-zero term each (compared with 0 and 1 only)
//
// INR: the scene's ranges are host-proven (light_ranges_box below), so these
// quotients and roots take the range-free sequences (div_inrange_,
// sqrt_inrange_: bit-identical in range, ipt_math.h). Where a quotient is out
// of range its result is never observed (the hit is rejected or the lane's
// pdf is not used), exactly as its IEEE value would not be.
// (light_trace_ax_q: the same test from the light's n_dir, t and plane point
// q = o + d*t, which every light of a coplanar lattice shares -- the lattice
// lookup computes them once with these operations)
template <int XA, int YA>
IPT_HD bool light_trace_ax_q(const LightDev& L, float n_dir, float t, vec3 q, vec3* hit, vec3* nrm);
template <int XA, int YA, bool INR = false>
IPT_HD bool light_trace_ax(const LightDev& L, vec3 o, vec3 d, vec3* hit, vec3* nrm) {
    constexpr int NA = 3 - XA - YA;
    const float n_dir = comp<NA>(L.n) * comp<NA>(d);
    // INR: |num| is 0 or in [2^-40, 2^41); |n_dir| >= 1e-6 wherever t is used
    const float num = comp<NA>(L.n) * (comp<NA>(L.P) - comp<NA>(o));
    const float t = INR ? div_inrange_(num, n_dir) : div_(num, n_dir);
    return light_trace_ax_q<XA, YA>(L, n_dir, t, o + d * t, hit, nrm);
}
template <int XA, int YA>
IPT_HD bool light_trace_ax_q(const LightDev& L, float n_dir, float t, vec3 q, vec3* hit, vec3* nrm) {
    const vec3 rel = q - L.P;
    const float cx = comp<0>(L.inv.c[XA]) * comp<XA>(rel);
    const float cy = comp<1>(L.inv.c[YA]) * comp<YA>(rel);
    const bool in = L.type == 0 ? (cx >= 0.0f) & (cx <= 1.0f) & (cy >= 0.0f) & (cy <= 1.0f)
                                : (cx >= 0.0f) & (cy >= 0.0f) & (cx + cy <= 1.0f);
    *hit = L.P + rel;
    *nrm = L.n;
    return !(lt_1em6(fabs_(n_dir)) | (n_dir > 0.0f)) & !lt_1em6(t) & in;
}
// light_pdf (DdfFromLight::value) with cosinus = dot(n, -normalize(hit - o))
// reduced to its one term (never a zero on a hit: |n.d| >= 1e-6 there)
template <int NA, bool INR = false>
IPT_HD float light_pdf_ax(const LightDev& L, vec3 o, bool has, vec3 hit, vec3 nrm) {
    if (!has) return 0.0f;
    const vec3 ho = hit - o;
    const float decay = dot(ho, ho);
    // INR on a hit: decay in [dmin^2, dmax^2], cosinus in [~1e-6, 1], area in range
    const float s = INR ? rcp_inrange_(sqrt_inrange_(decay))
                        : div_(1.0f, sqrt_(decay));  // normalize's 1/sqrt(dot(v,v)) (same dot)
    const float cosinus = comp<NA>(nrm) * -(comp<NA>(ho) * s);
    const float p = INR ? div_inrange_(div_inrange_(decay, cosinus), L.area) : div_(div_(decay, cosinus), L.area);
    return cosinus < 0.0f ? 0.0f : p;
}
// light_sample_dir (DdfFromLight::sample via AreaLight::sample): pos =
// (x*u1 + y*u2) + P keeps one product per component (P's components are
// non-zero, so a zero product is an exact no-op), cosinus one term (compared
// with 1e-5 only)
// light_sample_dir_ax from the light's fields it reads (P, x[XA], y[YA],
// n[NA], type), for callers that gathered them ahead (same operations)
template <int XA, int YA, bool INR = false>
IPT_HD vec3 light_sample_dir_axf(vec3 P, float xa, float ya, float nn, int type, vec3 o, float u1, float u2raw) {
    constexpr int NA = 3 - XA - YA;
    const float u2 = u2raw * (type == 1 ? 1.0f - u1 : 1.0f);
    float pc[3];
    pc[XA] = xa * u1 + comp<XA>(P);
    pc[YA] = ya * u2 + comp<YA>(P);
    pc[NA] = comp<NA>(P);
    // INR: |pos - o| in [dmin, dmax] for every surface point o
    const vec3 dir = INR ? normalize_inrange_(v3(pc[0], pc[1], pc[2]) - o) : normalize(v3(pc[0], pc[1], pc[2]) - o);
    const float cosinus = nn * -comp<NA>(dir);
    if (cosinus < 1e-5f) return v3(0.0f, 0.0f, 0.0f);
    return dir;
}
template <int XA, int YA, bool INR = false>
IPT_HD vec3 light_sample_dir_ax(const LightDev& L, vec3 o, float u1, float u2raw) {
    constexpr int NA = 3 - XA - YA;
    const float u2 = u2raw * (L.type == 1 ? 1.0f - u1 : 1.0f);
    float pc[3];
    pc[XA] = comp<XA>(L.x) * u1 + comp<XA>(L.P);
    pc[YA] = comp<YA>(L.y) * u2 + comp<YA>(L.P);
    pc[NA] = comp<NA>(L.P);
    // INR: |pos - o| in [dmin, dmax] for every surface point o
    const vec3 dir = INR ? normalize_inrange_(v3(pc[0], pc[1], pc[2]) - o) : normalize(v3(pc[0], pc[1], pc[2]) - o);
    const float cosinus = comp<NA>(L.n) * -comp<NA>(dir);
    if (cosinus < 1e-5f) return v3(0.0f, 0.0f, 0.0f);
    return dir;
}
// Host check of the conditions above; returns 1 + index of the (XA, YA) pair
// in {(1,0), (0,1)} (normal along z), else 0 (generic code).
inline int axis_aligned_light(const LightDev& L) {
    if (L.type != 0 && L.type != 1) return 0;
    auto z = [](float f) { return (f2u(f) & 0x7fffffffu) == 0u; };
    auto one_nz = [&](vec3 v, int a) {
        const float c[3] = {v.x, v.y, v.z};
        for (int i = 0; i < 3; ++i)
            if ((i == a) == z(c[i])) return false;
        return true;
    };
    if (z(L.P.x) || z(L.P.y) || z(L.P.z)) return 0;
    const int pairs[2][2] = {{1, 0}, {0, 1}};
    for (int k = 0; k < 2; ++k) {
        const int xa = pairs[k][0], ya = pairs[k][1], na = 3 - xa - ya;
        if (!one_nz(L.x, xa) || !one_nz(L.y, ya) || !one_nz(L.n, na)) continue;
        // inverse rows 0 and 1 (coord.x, coord.y): one non-zero term each
        const float r0[3] = {L.inv.c[0].x, L.inv.c[1].x, L.inv.c[2].x};
        const float r1[3] = {L.inv.c[0].y, L.inv.c[1].y, L.inv.c[2].y};
        bool ok = true;
        for (int i = 0; i < 3; ++i) {
            if (i != xa && !z(r0[i])) ok = false;
            if (i != ya && !z(r1[i])) ok = false;
        }
        if (ok) return 1 + k;
    }
    return 0;
}

// Host proof of the INR ranges for an axis-aligned single AreaLight in
// GeometrySphereInBox: every ray origin is the camera, a wall point (a hit of
// the box planes: inside the cube up to rounding) or a sphere point (|p| =
// 0.5 up to rounding). dmin (a lower bound of |light point - origin|) comes
// from the light's bounding box against the wall planes, the sphere and the
// camera; dmax from the cube and camera extents. Required: dmin >= 2^-8
// (decay >= 2^-16; 1/sqrt, decay/cosinus and the sample's normalize in range),
// dmax <= 2^8, area and |n| in [2^-16, 2^16], |P_NA| >= 2^-8 (a non-zero
// P_NA - o_NA is then >= 2^-32, so t's numerator is 0 or in range).
inline bool light_ranges_box(const LightDev& L, int na, const float cam[3]) {
    float lo[3], hi[3];
    const float P[3] = {L.P.x, L.P.y, L.P.z}, X[3] = {L.x.x, L.x.y, L.x.z}, Y[3] = {L.y.x, L.y.y, L.y.z};
    for (int i = 0; i < 3; ++i) {
        lo[i] = P[i] + (X[i] < 0.0f ? X[i] : 0.0f) + (Y[i] < 0.0f ? Y[i] : 0.0f);
        hi[i] = P[i] + (X[i] > 0.0f ? X[i] : 0.0f) + (Y[i] > 0.0f ? Y[i] : 0.0f);
    }
    const double m = 1e-5;  // rounding slack of hit points and of the box above
    double dmin = 1e30;
    // wall planes x = +-1, y = +1, z = +-1 (GeometrySphereInBox.cpp:10-81)
    const double walls[5][2] = {{0, 1}, {1, 1}, {2, 1}, {0, -1}, {2, -1}};
    for (const auto& w : walls) {
        const int a = (int)w[0];
        const double v = w[1];
        const double dd = (lo[a] > v) ? lo[a] - v : ((hi[a] < v) ? v - hi[a] : 0.0);
        dmin = dd < dmin ? dd : dmin;
    }
    auto box_dist = [&](const double q[3]) {
        double s2 = 0.0;
        for (int i = 0; i < 3; ++i) {
            const double dd = q[i] < lo[i] ? lo[i] - q[i] : (q[i] > hi[i] ? q[i] - hi[i] : 0.0);
            s2 += dd * dd;
        }
        return __builtin_sqrt(s2);
    };
    const double origin[3] = {0, 0, 0}, c[3] = {cam[0], cam[1], cam[2]};
    const double ds = box_dist(origin) - 0.5;
    dmin = ds < dmin ? ds : dmin;
    const double dc = box_dist(c);
    dmin = dc < dmin ? dc : dmin;
    dmin -= m;
    double ext = 1.0;
    for (int i = 0; i < 3; ++i) {
        const double e = __builtin_fabs(lo[i]) > __builtin_fabs(hi[i]) ? __builtin_fabs(lo[i]) : __builtin_fabs(hi[i]);
        ext = e > ext ? e : ext;
        ext = __builtin_fabs(cam[i]) > ext ? __builtin_fabs(cam[i]) : ext;
    }
    const double dmax = 2.0 * ext * 1.7320508 + m;
    const float n[3] = {L.n.x, L.n.y, L.n.z};
    const float pn = P[na];
    return dmin >= 0x1p-8 && dmax <= 0x1p8 && L.area >= 0x1p-16f && L.area <= 0x1p16f &&
           __builtin_fabs(n[na]) >= 0x1p-16f && __builtin_fabs(n[na]) <= 0x1p16f && __builtin_fabs(pn) >= 0x1p-8f;
}

// Coplanar light lattice (kLightsGridA10/A01, the many-light C5 scene's 16 x 16
// emitters): every light an axis-aligned diamond AreaLight with the same axis
// pattern, the same normal and the same plane coordinate P[2] (so every
// light's traceRay computes the same t and plane point q), and its rectangle
// in the plane's (u, v) = (q[XA], q[YA]) one cell of a uniform lattice (within
// 2^-12 of a cell on each edge), at most one light per cell. The kernel looks
// a ray up by the cells within e of its cell coordinates (u, v), e the margin
// below, computed per lattice.
//
// The margin. The light test and the lookup see the same float plane point q
// (the same t, the same o + d*t). A light accepts q only within 2^-18 of a
// cell beyond its rectangle: its lower edge is exact (RN(q - P) >= 0 iff
// q >= P), its upper edge moves by the roundings of q - P and of the inverse
// entry times it (relative < 2^-21 of the rectangle). The rectangle lies
// within `dev` cells of its lattice cell (measured here in double). The
// kernel's u = RN(RN(q - u0f) * icwf) is within eps = 2^-24 (|u0|/cw +
// 3.01 (nu + 2)) cells of the exact (q - u0)/cw (u0f, icwf the float
// parameters; three roundings relative to |u| <= nu + 2). So a hit light's
// cell c has u in [c - m, c + 1 + m], m = dev + 2^-18 + eps, and with e >=
// 2m + 2^-15 the kernel's RN(u -+ e) (rounding error < 2^-16 for |u| < 2^9)
// still floors to c on the side where u left the cell. e is that bound
// rounded up to a power of two, at least 2^-14; a lattice that would need more
// than 2^-8 is not used. (C5's 16 x 16 lattice: dev 2^-18.5, e = 2^-14, so a
// ray meets a second candidate cell in ~1 of 8 000 lookups instead of 1 of 64
// with a fixed 2^-8.)
struct LightGrid {
    int pattern = 0;  // axis_aligned_light() of every light; 0 = no lattice
    int nu = 0, nv = 0;
    float u0 = 0.0f, v0 = 0.0f, icw = 0.0f, ich = 0.0f, pn = 0.0f, nn = 0.0f;
    float e = 0x1p-8f;       // candidate margin in cells (above)
    std::vector<int> cells;  // [nv][nu] light index, -1 = empty
};
inline bool light_grid_build(const LightDev* L, int nl, LightGrid& g) {
    if (nl < 2) return false;
    const int pat = axis_aligned_light(L[0]);
    if (pat == 0) return false;
    const int XA = pat == 1 ? 1 : 0, YA = 1 - XA;
    auto c = [](vec3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); };
    std::vector<double> lu(nl), hu(nl), lv(nl), hv(nl);
    for (int i = 0; i < nl; ++i) {
        if (L[i].type != 0 || axis_aligned_light(L[i]) != pat) return false;
        if (f2u(L[i].n.z) != f2u(L[0].n.z) || f2u(L[i].P.z) != f2u(L[0].P.z)) return false;
        const double pu = c(L[i].P, XA), xu = c(L[i].x, XA), pv = c(L[i].P, YA), yv = c(L[i].y, YA);
        lu[i] = pu + (xu < 0.0 ? xu : 0.0);
        hu[i] = pu + (xu > 0.0 ? xu : 0.0);
        lv[i] = pv + (yv < 0.0 ? yv : 0.0);
        hv[i] = pv + (yv > 0.0 ? yv : 0.0);
    }
    const double cw = hu[0] - lu[0], ch = hv[0] - lv[0];
    if (!(cw >= 0x1p-20 && ch >= 0x1p-20)) return false;
    double u0 = lu[0], v0 = lv[0];
    for (int i = 1; i < nl; ++i) {
        u0 = lu[i] < u0 ? lu[i] : u0;
        v0 = lv[i] < v0 ? lv[i] : v0;
    }
    const double tol = 0x1p-12;
    std::vector<int> ci(nl), cj(nl);
    int nu = 0, nv = 0;
    double dev = 0.0;  // largest deviation of a rectangle edge from its lattice line, in cells
    for (int i = 0; i < nl; ++i) {
        const double fi = (lu[i] - u0) / cw, fj = (lv[i] - v0) / ch;
        const double ri = __builtin_floor(fi + 0.5), rj = __builtin_floor(fj + 0.5);
        const double d[4] = {__builtin_fabs(fi - ri), __builtin_fabs((hu[i] - u0) / cw - (ri + 1.0)),
                             __builtin_fabs(fj - rj), __builtin_fabs((hv[i] - v0) / ch - (rj + 1.0))};
        for (double x : d) {
            if (!(x <= tol)) return false;
            dev = x > dev ? x : dev;
        }
        if (ri < 0.0 || rj < 0.0 || ri >= 256.0 || rj >= 256.0) return false;
        ci[i] = (int)ri;
        cj[i] = (int)rj;
        nu = ci[i] + 1 > nu ? ci[i] + 1 : nu;
        nv = cj[i] + 1 > nv ? cj[i] + 1 : nv;
    }
    if (nu * nv > 4096) return false;
    const double umax = u0 + nu * cw, vmax = v0 + nv * ch;
    if (!(__builtin_fabs(u0) <= 0x1p20 && __builtin_fabs(umax) <= 0x1p20 && __builtin_fabs(v0) <= 0x1p20 &&
          __builtin_fabs(vmax) <= 0x1p20 && cw >= 0x1p-12 * (__builtin_fabs(u0) + __builtin_fabs(umax)) &&
          ch >= 0x1p-12 * (__builtin_fabs(v0) + __builtin_fabs(vmax))))
        return false;  // cells small against their coordinates: rounding could exceed the margin
    // the candidate margin (see LightGrid)
    double m = 0.0;
    for (int a = 0; a < 2; ++a) {
        const double org = a == 0 ? u0 : v0, w = a == 0 ? cw : ch;
        const int n = a == 0 ? nu : nv;
        const double eps = 0x1p-24 * (__builtin_fabs(org) / w + 3.01 * (n + 2));
        const double ma = dev + 0x1p-18 + eps;
        m = ma > m ? ma : m;
    }
    double e = 0x1p-14;
    while (e < 2.0 * m + 0x1p-15) e *= 2.0;
    if (e > 0x1p-8) return false;
    g.cells.assign((size_t)nu * nv, -1);
    for (int i = 0; i < nl; ++i) {
        int& cell = g.cells[(size_t)ci[i] + (size_t)nu * cj[i]];
        if (cell >= 0) return false;  // two lights in one cell
        cell = i;
    }
    g.pattern = pat;
    g.nu = nu;
    g.nv = nv;
    g.u0 = (float)u0;
    g.v0 = (float)v0;
    g.icw = (float)(1.0 / cw);
    g.ich = (float)(1.0 / ch);
    g.pn = L[0].P.z;
    g.nn = L[0].n.z;
    g.e = (float)e;
    return true;
}

// A lattice light's fields that its axis-aligned trace / pdf / sample and
// the mixture read, in 48 bytes (three 16-byte loads instead of a 96-byte
// LightDev walked field by field): P[0..1] (P[2] and n[2] are the lattice's
// shared plane, LightGrid::pn / nn), x[XA], y[YA], inverse rows' non-zero
// terms inv.c[XA].x and inv.c[YA].y, area, power/area and the light's
// mixture weight. Every value is copied bit for bit.
struct LightAx {
    float px, py, xa, ya, ix, iy, area, spow, w, pad[3];
};
inline LightAx light_ax_record(const LightDev& L, int pattern, float weight) {
    const int XA = pattern == 1 ? 1 : 0, YA = 1 - XA;
    auto c = [](vec3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); };
    LightAx r{};
    r.px = L.P.x;
    r.py = L.P.y;
    r.xa = c(L.x, XA);
    r.ya = c(L.y, YA);
    r.ix = L.inv.c[XA].x;
    r.iy = L.inv.c[YA].y;
    r.area = L.area;
    r.spow = L.spow;
    r.w = weight;
    return r;
}

// Light constructor derived fields: AreaLight (lighting.cpp:79-90) + the
// per-call normal/power expressions of traceRay/sample; SphereLight /
// InvertedSphereLight: area = 4.0*M_PI*radius*radius in f64 (lighting.h:
// 46-52); PointLight: area 0 (lighting.h:33-37).
IPT_HD LightDev make_light(vec3 P, vec3 x, vec3 y, float power, int type) {
    LightDev L;
    L.P = P;
    L.x = x;
    L.y = y;
    L.type = type;
    L.pad = 0;
    if (type >= 2) {
        const double r = (double)x.x;
        L.area = type == 3 ? 0.0f : (float)(4.0 * u2d(0x400921fb54442d18ull) * r * r);
        L.n = v3(0.0f, 0.0f, 0.0f);
        for (int c = 0; c < 3; ++c) L.inv.c[c] = v3(0.0f, 0.0f, 0.0f);
        L.spow = power / L.area;
        return L;
    }
    const float full_area = length(cross(x, y));
    L.area = type == 0 ? full_area : full_area / 2.0f;
    mat3 m;
    m.c[0] = x;
    m.c[1] = y;
    m.c[2] = cross(x, y);
    L.inv = inverse(m);
    L.n = normalize(cross(x, y));
    L.spow = power / L.area;
    return L;
}

// ------------------------------------------------------------ camera/pixel
// render_sample jitter (main.cpp:192-198) generalised from 640 to W/H.
IPT_HD float jitter_coord(int i, float u, int n) {
    float x = ((float)i + u) / (float)n;
    if (x == 1.0f) x = u2f(0x3f7fffffu);  // nextafter(1.0f, 0.0f)
    return x;
}
// SimpleCamera::sampleRay (SimpleCamera.cpp:15-21)
IPT_HD vec3 camera_dir(vec3 right, vec3 up, vec3 direction, float x, float y) {
    x -= 0.5f;
    y -= 0.5f;
    const vec3 ray = right * x + up * y + direction;
    return normalize(ray);
}
// GridRenderPlane::addRay index mapping (GridRenderPlane.cpp:66-67).
IPT_HD void grid_index(float x, float y, int W, int H, int* xi, int* yi) {
    const float fx = x * (float)W;
    const float fy = ((float)H - y * (float)H) - 1.0f;
    *xi = fx < 0.0f ? 0 : (int)fx;  // (size_t) truncation; values in (-1,0) -> 0
    *yi = fy < 0.0f ? 0 : (int)fy;
}
IPT_HD int nominal_row(int iy, int H) { return H - 2 - iy > 0 ? H - 2 - iy : 0; }

// ---------------------------------------------------------- mixture weights
// CollectionLighting::distributionInPoint + unite (CollectionLighting.cpp:12-21,
// ddf.cpp:169-235) followed by main.cpp:143's unite(light_ddf,1, sdf,1).
// Point-independent: w[0..n-1] lights, w[n] the surface BRDF.
inline void mixture_weights(const float* powers, int n, float* w) {
    float acc_power = 0.0f;
    int cnt = 0;
    for (int l = 0; l < n; ++l) {
        const float ka = acc_power, kb = powers[l];
        if (cnt == 0 && ka != 0.0f) {
            // unite(nullptr,0,b,kb) -> unite(Union(),0,b,1.0f) -> [b : 1/(0+1)]
            w[0] = 1.0f / (0.0f + 1.0f);
            cnt = 1;
        } else {
            for (int k = 0; k < cnt; ++k) w[k] *= ka / (ka + kb);
            w[cnt++] = kb / (ka + kb);
        }
        acc_power += powers[l];
    }
    if (cnt == 0) {
        w[0] = 1.0f / (0.0f + 1.0f);
        return;
    }
    for (int k = 0; k < cnt; ++k) w[k] *= 1.0f / (1.0f + 1.0f);
    w[cnt] = 1.0f / (1.0f + 1.0f);
}

}  // namespace ipt
