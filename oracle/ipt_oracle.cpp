// ORACLE — test infrastructure only, never part of the product.
//
// A plain CPU restatement of dimalit/ipt's hot path (reference snapshot
// 2024-12-23), written independently of ipt_amd/csrc and structured like the
// reference: a recursive ray_power with a Union-of-DDFs mixture built per
// surface hit, glm-order vector arithmetic and the host libm (glibc 2.35
// acosf/sinf/cosf/acos), exactly the calls the reference makes.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
// this library (oracle/libipt_oracle.so), and only as the checker / CPU
// baseline. The reference's own ddf.cpp and main.cpp cannot be compiled in
// this image (they need boost/config.hpp, which is absent — see DESIGN.md),
// so this restatement is pinned (a) bit-exactly against the reference's own
// geometry / lighting / camera / GridRenderPlane / RotateDdf code compiled by
// oracle/build_ref.sh (tests/test_oracle_vs_ref.py), (b) against the
// reference's unit-test known answers (tests/test_reference_kats.py) and
// (c) statistically against the survey's measurements of the real reference
// (image means and per-path event counts, tests/test_oracle_stats.py).
//
// Build: oracle/Makefile  (g++ -O2 -ffp-contract=off, no fast-math)

#include "../include/ipt_capi.h"

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

namespace {

// ------------------------------------------------------------------ glm-ish
struct V3 {
    float x, y, z;
};
inline V3 mk(float x, float y, float z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
inline V3 operator*(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
inline V3 operator*(float s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
inline bool operator==(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
// glm/detail/func_geometric.inl:48-55
inline float dot(V3 a, V3 b) {
    V3 t = mk(a.x * b.x, a.y * b.y, a.z * b.z);
    return t.x + t.y + t.z;
}
// func_geometric.inl:68-79
inline V3 cross(V3 x, V3 y) {
    return mk(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
inline float length(V3 v) { return std::sqrt(dot(v, v)); }
// func_geometric.inl:82-90 + func_exponential.inl:136-139
inline V3 normalize(V3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }

struct M3 {  // column-major, m[c][r]
    float m[3][3];
};
// type_mat3x3.inl:468-474
inline V3 mul(const M3& a, V3 v) {
    return mk(a.m[0][0] * v.x + a.m[1][0] * v.y + a.m[2][0] * v.z,
              a.m[0][1] * v.x + a.m[1][1] * v.y + a.m[2][1] * v.z,
              a.m[0][2] * v.x + a.m[1][2] * v.y + a.m[2][2] * v.z);
}
// func_matrix.inl:268-291
inline M3 inverse(const M3& a) {
    const auto& m = a.m;
    float OneOverDeterminant = 1.0f / (+m[0][0] * (m[1][1] * m[2][2] - m[2][1] * m[1][2]) -
                                       m[1][0] * (m[0][1] * m[2][2] - m[2][1] * m[0][2]) +
                                       m[2][0] * (m[0][1] * m[1][2] - m[1][1] * m[0][2]));
    M3 r;
    r.m[0][0] = +(m[1][1] * m[2][2] - m[2][1] * m[1][2]) * OneOverDeterminant;
    r.m[1][0] = -(m[1][0] * m[2][2] - m[2][0] * m[1][2]) * OneOverDeterminant;
    r.m[2][0] = +(m[1][0] * m[2][1] - m[2][0] * m[1][1]) * OneOverDeterminant;
    r.m[0][1] = -(m[0][1] * m[2][2] - m[2][1] * m[0][2]) * OneOverDeterminant;
    r.m[1][1] = +(m[0][0] * m[2][2] - m[2][0] * m[0][2]) * OneOverDeterminant;
    r.m[2][1] = -(m[0][0] * m[2][1] - m[2][0] * m[0][1]) * OneOverDeterminant;
    r.m[0][2] = +(m[0][1] * m[1][2] - m[1][1] * m[0][2]) * OneOverDeterminant;
    r.m[1][2] = -(m[0][0] * m[1][2] - m[1][0] * m[0][2]) * OneOverDeterminant;
    r.m[2][2] = +(m[0][0] * m[1][1] - m[1][0] * m[0][1]) * OneOverDeterminant;
    return r;
}
// ext/matrix_transform.inl:18-47 on identity(4), truncated to mat3
inline M3 rotate_identity(float angle, V3 v) {
    const float a = angle;
    const float c = std::cos(a);
    const float s = std::sin(a);
    V3 axis = normalize(v);
    V3 temp = (1.0f - c) * axis;
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = temp.x * axis.y + s * axis.z;
    R[0][2] = temp.x * axis.z - s * axis.y;
    R[1][0] = temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = temp.y * axis.z + s * axis.x;
    R[2][0] = temp.z * axis.x + s * axis.y;
    R[2][1] = temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    const float I[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    M3 out;
    for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 3; ++j)
            out.m[k][j] = I[0][j] * R[k][0] + I[1][j] * R[k][1] + I[2][j] * R[k][2];
    return out;
}

const float INF = std::numeric_limits<float>::infinity();

// --------------------------------------------------------------- counters
struct Counters {
    uint64_t paths = 0, traced = 0, surf = 0, light = 0, expanded = 0, iters = 0, lsamp = 0,
             skipped = 0, sframes = 0, ltraces = 0, drifted = 0;
    // SURVEY.md Appendix C's instrumented-reference counts: node sums that are
    // not finite when main.cpp:181 tests them (the NaN-poison), multipliers
    // that are not finite where main.cpp:175 asserts, randf() draws
    uint64_t nf_sums = 0, nf_mults = 0, draws = 0;
};
thread_local Counters* g_cnt = nullptr;

// ------------------------------------------------------------------ RNG
// The randf() replacement (reference include/randf.h:6-11): a per-path
// sequential stream. Draw k of path (pixel p, pass s) is word k%4 of
// Philox4x32-10(counter = {k/4, s, p, 0}, key = seed), mapped to
// (w>>8)*2^-24 in [0,1).
struct Rng {
    uint32_t k0, k1, s, p;
    uint32_t k = 0;
    uint32_t blk[4];
    uint32_t blk_id = 0xffffffffu;
};
thread_local Rng* g_rng = nullptr;

void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}
// Test hook: when set, randf() returns these uniforms in order instead of the
// Philox stream (explicit-uniform sampler checks, ipt_oracle_ddf_sample).
thread_local const float* g_ufeed = nullptr;
float randf() {
    if (g_ufeed) return *g_ufeed++;
    Rng& g = *g_rng;
    if (g_cnt) ++g_cnt->draws;
    uint32_t b = g.k >> 2;
    if (b != g.blk_id) {
        uint32_t c[4] = {b, g.s, g.p, 0u};
        philox(c, g.k0, g.k1);
        std::memcpy(g.blk, c, sizeof c);
        g.blk_id = b;
    }
    uint32_t w = g.blk[g.k & 3];
    ++g.k;
    float res = (float)(w >> 8) * 5.9604644775390625e-08f;
    return res;  // never 1.0f, randf.h:8-9's retry never fires
}


// ------------------------------------------------------------------ scene
struct AreaLightO {
    V3 position, x_axis, y_axis;
    M3 inverse_matrix;
    float power, area;
    int type;
    // lighting.cpp:79-90 (AreaLight); types 2-4: SphereLight, PointLight,
    // InvertedSphereLight (lighting.h:31-73), radius in xa.x
    float radius = 0.0f;
    AreaLightO(V3 origin, V3 xa, V3 ya, float pw, int ty) {
        position = origin;
        x_axis = xa;
        y_axis = ya;
        power = pw;
        type = ty;
        if (type >= 2) {
            radius = xa.x;
            area = type == 3 ? 0.0f : 4.0 * M_PI * radius * radius;  // lighting.h:50
            return;
        }
        float full_area = length(cross(x_axis, y_axis));
        area = type == 0 ? full_area : full_area / 2.0f;
        M3 m;
        V3 c = cross(x_axis, y_axis);
        m.m[0][0] = x_axis.x; m.m[0][1] = x_axis.y; m.m[0][2] = x_axis.z;
        m.m[1][0] = y_axis.x; m.m[1][1] = y_axis.y; m.m[1][2] = y_axis.z;
        m.m[2][0] = c.x; m.m[2][1] = c.y; m.m[2][2] = c.z;
        inverse_matrix = inverse(m);
    }
    // lighting.cpp:176-212 (SphereLight / PointLight ::sample), normal flipped
    // for InvertedSphereLight (lighting.h:67-71)
    void sample_round(V3* pos_out, V3* normal_out, float* sp) const {
        float u1 = randf() * 2.0f - 1.0f;
        float u2 = randf();
        float alpha = std::acos(u1);
        float phi = 2 * M_PI * u2;
        if (type == 3) {
            float r = std::sin(alpha);
            *normal_out = mk(r * std::cos(phi), r * std::sin(phi), u1);
            *pos_out = position;
            *sp = std::numeric_limits<float>::signaling_NaN();
            return;
        }
        float r = radius * std::sin(alpha);
        V3 pos = mk(r * std::cos(phi), r * std::sin(phi), radius * u1);
        *pos_out = pos + position;
        *normal_out = normalize(pos);
        if (type == 4) *normal_out = -*normal_out;
        *sp = power / area;
    }
    // lighting.cpp:11-36: SphereLight's own sphere intersection
    static float round_t(float radius, V3 origin, V3 direction) {
        float desc = 4.0f * (dot(origin, direction) * dot(origin, direction)) -
                     4.0f * dot(direction, direction) * (dot(origin, origin) - radius * radius);
        if (desc < 0.0f) return INF;
        float t1 = (-2.0 * dot(origin, direction) - std::sqrt(desc)) / 2.0 / dot(direction, direction);
        float t2 = (-2.0 * dot(origin, direction) + std::sqrt(desc)) / 2.0 / dot(direction, direction);
        if (t1 < 1e-6) t1 = INF;
        if (t2 < 1e-6) t2 = INF;
        float t = std::min(t1, t2);
        V3 pos = origin + direction * t;
        V3 outer_normal = normalize(pos);
        float direction_sign = dot(outer_normal, origin - pos);
        float position_sign = length(origin) - radius;
        if (direction_sign * position_sign <= 0.0f) return INF;
        return t;
    }
    // lighting.cpp:93-104
    void sample(V3* pos_out, V3* normal_out, float* sp) const {
        if (type >= 2) {
            sample_round(pos_out, normal_out, sp);
            return;
        }
        float u1 = randf();
        float u2 = randf() * (type == 1 ? 1.0f - u1 : 1.0f);
        V3 pos = x_axis * u1 + y_axis * u2;
        *pos_out = pos + position;
        *normal_out = normalize(cross(x_axis, y_axis));
        *sp = power / area;
    }
    // lighting.cpp:107-144
    bool traceRay(V3 origin, V3 direction, V3* pos_out, V3* normal_out, float* sp) const {
        if (g_cnt) ++g_cnt->ltraces;
        if (type == 3) return false;  // PointLight::traceRay (lighting.h:39-41)
        if (type >= 2) {              // SphereLight::traceRay (lighting.cpp:161-173)
            float t = round_t(radius, origin - position, direction);
            if (t == INF) return false;
            *pos_out = origin + direction * t;
            *normal_out = normalize(*pos_out - position);
            if (type == 4) *normal_out = -*normal_out;  // InvertedSphereLight (lighting.h:61-66)
            *sp = power / area;
            return true;
        }
        V3 n = normalize(cross(x_axis, y_axis));
        float n_dir = dot(n, direction);
        if (std::abs(n_dir) < 1e-6 || n_dir > 0.0f) return false;
        float t = dot(n, position - origin) / n_dir;
        if (t < 1e-6) return false;
        V3 relative_pos = origin + direction * t - position;
        V3 coord = mul(inverse_matrix, relative_pos);
        bool hit;
        if (type == 0)
            hit = coord.x >= 0.0f && coord.x <= 1.0f && coord.y >= 0.0f && coord.y <= 1.0f;
        else
            hit = coord.x >= 0.0f && coord.y >= 0.0 && coord.x + coord.y <= 1.0f;
        if (!hit) return false;
        *pos_out = position + relative_pos;
        *normal_out = normalize(cross(x_axis, y_axis));
        *sp = power / area;
        return true;
    }
};

struct SceneO {
    int geometry_kind;
    std::vector<AreaLightO> lights;
    std::vector<float> sph_r;
    std::vector<V3> sph_c;
    V3 cam_pos, cam_dir, cam_right, cam_up;
};

// geometric_utils.cpp:8-26
float intersection_with_box_plane(V3 plane, V3 origin, V3 direction) {
    float dir_plane = dot(direction, plane);
    if (std::abs(dir_plane) < 1e-6) return INF;
    float t = (1.0f - dot(origin, plane)) / dir_plane;
    V3 point = origin + direction * t;
    if (std::abs(point.x) > 1.0f || std::abs(point.y) > 1.0f || std::abs(point.z) > 1.0f)
        return INF;
    if (dot(direction, plane) < 0.0f) return INF;
    if (t < 1e-6) return INF;
    return t;
}
// geometric_utils.cpp:28-55  (pow(b,2.0f) is folded to b*b by the compiler)
float intersection_with_sphere(float radius, V3 origin, V3 direction) {
    float origin_x_dir = dot(origin, direction);
    float desc = 4.0f * (origin_x_dir * origin_x_dir) -
                 4.0f * (dot(origin, origin) - radius * radius);
    if (desc < 0.0f) return INF;
    float sqrt_desc = std::sqrt(desc);
    float t1 = (-2.0 * origin_x_dir - sqrt_desc) / 2.0;
    float t2 = (-2.0 * origin_x_dir + sqrt_desc) / 2.0;
    if (t1 < 1e-6) t1 = INF;
    if (t2 < 1e-6) t2 = INF;
    float t = std::min(t1, t2);
    V3 pos = origin + direction * t;
    if (dot(pos, origin - pos) <= 0.0f) return INF;
    return t;
}

// RotateDdf (ddf_detail.h:72-85) around a CosineDdf (ddf.cpp:223-238)
struct RotatedCosine {
    M3 transformation, inv;
    bool rotated = true;  // false: a plain CosineDdf (GeometryFloor's sdf, GeometryFloor.cpp:19)
    static RotatedCosine plain() {
        RotatedCosine r(mk(0.0f, 0.0f, 1.0f));
        r.rotated = false;
        return r;
    }
    explicit RotatedCosine(V3 to) {
        V3 z = mk(0.0f, 0.0f, 1.0f);
        V3 axis = cross(z, to);
        if (length(axis) < 1e-6) axis = mk(1.0f, 0.0f, 0.0f);
        float cosinus = dot(z, to);
        transformation = rotate_identity((float)::acos((double)cosinus), axis);
        inv = inverse(transformation);
    }
    V3 sample() const {
        float u1 = randf();
        float u2 = randf();
        float cos_alpha = std::sqrt(u1);
        float alpha = std::acos(cos_alpha);
        float phi = 2 * M_PI * u2;
        float r = std::sin(alpha);
        V3 x = mk(r * std::cos(phi), r * std::sin(phi), cos_alpha);
        return rotated ? mul(transformation, x) : x;
    }
    float value(V3 arg) const {
        V3 a = rotated ? mul(inv, arg) : arg;
        if (a.z < 0.0f) return 0.0f;
        return a.z / M_PI;
    }
};

struct SurfHit {
    V3 position, normal;
    bool plain_cosine = false;  // unrotated CosineDdf (GeometryFloor)
};
// GeometrySphereInBox::traceRay (GeometrySphereInBox.cpp:10-81) and the
// 5-planes + N-spheres stress geometry (FractalSpheres.cpp:69-97 acceptance).
bool geometry_trace(const SceneO& sc, V3 origin, V3 direction, SurfHit* out) {
    if (g_cnt) ++g_cnt->traced;
    if (sc.geometry_kind == IPT_GEOM_FLOOR) {  // GeometryFloor.cpp:10-23
        float t = intersection_with_box_plane(mk(0, 0, -1), origin, direction);
        if (t == INF || t < 0.0f || std::abs(t) < 1e-6) return false;
        out->position = origin + direction * t;
        out->normal = mk(0, 0, 1);
        out->plain_cosine = true;
        return true;
    }
    if (sc.geometry_kind == IPT_GEOM_SMALLPT) {  // GeometrySmallPt.cpp:11-58
        double min_t = std::numeric_limits<double>::infinity();
        int min_s = -1;
        for (size_t i = 0; i < sc.sph_r.size(); ++i) {
            // Sphere::intersect (GeometrySmallPt.cpp:16-22), rad a double
            const double rad = sc.sph_r[i];
            V3 op = sc.sph_c[i] - origin;
            double t, eps = 1e-4, b = dot(op, direction), det = b * b - dot(op, op) + rad * rad;
            if (det < 0) {
                t = 0;
            } else {
                det = std::sqrt(det);
                t = (t = b - det) > eps ? t : ((t = b + det) > eps ? t : 0);
            }
            if (t != 0.0) {
                if (t < min_t) {
                    min_t = t;
                    min_s = (int)i;
                }
            }
        }
        if (!std::isfinite(min_t)) return false;
        out->position = origin + direction * (float)min_t;
        const V3 v = normalize(out->position - sc.sph_c[min_s]);
        out->normal = sc.sph_r[min_s] < 100 ? v : -v;
        return true;
    }
    if (sc.geometry_kind == IPT_GEOM_CORNER) {  // GeometryCorner.cpp:10-42
        float tx = intersection_with_box_plane(mk(-1, 0, 0), origin, direction);
        float ty = intersection_with_box_plane(mk(0, -1, 0), origin, direction);
        float tz = intersection_with_box_plane(mk(0, 0, -1), origin, direction);
        float t = tx;
        V3 normal = mk(1, 0, 0);
        if (ty < t) {
            t = ty;
            normal = mk(0, 1, 0);
        }
        if (tz < t) {
            t = tz;
            normal = mk(0, 0, 1);
        }
        if (t == INF || t < 0.0f || std::abs(t) < 1e-6) return false;
        out->position = origin + direction * t;
        out->normal = normal;
        return true;
    }
    static const V3 planes[] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {-1, 0, 0}, {0, 0, -1}};
    float dist = INF;
    int intersected_plane = -1;
    bool intersected_sphere = false;
    for (int i = 0; i < 5; ++i) {
        float t = intersection_with_box_plane(planes[i], origin, direction);
        if (t < dist) {
            dist = t;
            intersected_plane = i;
        }
    }
    V3 sc_center = mk(0, 0, 0);
    if (sc.geometry_kind == IPT_GEOM_SPHERES) {  // FractalSpheres: the list alone
        dist = INF;
        intersected_plane = -1;
    }
    if (sc.geometry_kind == IPT_GEOM_SPHERE_IN_BOX) {
        float t = intersection_with_sphere(0.5f, origin, direction);
        if (t < dist) {
            dist = t;
            intersected_sphere = true;
            intersected_plane = -1;
        }
    } else {
        for (size_t i = 0; i < sc.sph_r.size(); ++i) {
            float t = intersection_with_sphere(sc.sph_r[i], origin - sc.sph_c[i], direction);
            if (std::isfinite(t) && std::abs(t) > 1e-6 && t < dist) {
                dist = t;
                intersected_sphere = true;
                intersected_plane = -1;
                sc_center = sc.sph_c[i];
            }
        }
    }
    if (dist == INF) return false;
    out->position = origin + direction * dist;
    if (intersected_plane >= 0) {
        out->normal = -planes[intersected_plane];
    } else if (intersected_sphere) {
        out->normal = sc.geometry_kind == IPT_GEOM_SPHERE_IN_BOX
                          ? normalize(out->position)
                          : normalize(out->position - sc_center);
    } else {
        return false;
    }
    return true;
}

// CollectionLighting::traceRayToLight (CollectionLighting.cpp:23-34)
bool lighting_trace(const SceneO& sc, V3 origin, V3 direction, V3* pos, float* sp) {
    bool has = false;
    V3 rp{}, rn{};
    float rs = 0;
    for (const auto& l : sc.lights) {
        V3 p, n;
        float s;
        if (!l.traceRay(origin, direction, &p, &n, &s)) continue;
        if (!has || length(rp - origin) > length(p - origin)) {
            has = true;
            rp = p;
            rn = n;
            rs = s;
        }
    }
    *pos = rp;
    *sp = rs;
    return has;
}

// The mixture built at main.cpp:142-143: CollectionLighting::distributionInPoint
// (CollectionLighting.cpp:12-21) united with the surface DDF, with unite()'s
// weight arithmetic (ddf.cpp:169-235).
struct Mixture {
    std::vector<float> weights;  // lights in order, then the surface DDF
};
Mixture build_mixture(const SceneO& sc) {
    // res = unite(): an empty UnionDdf
    std::vector<float> w;
    float acc_power = 0.0f;
    for (const auto& l : sc.lights) {
        float ka = acc_power, kb = l.power;
        if (w.empty() && ka != 0.0f) {
            w.push_back(1.0f / (0.0f + 1.0f));
        } else {
            for (float& k : w) k *= ka / (ka + kb);
            w.push_back(kb / (ka + kb));
        }
        acc_power += l.power;
    }
    Mixture m;
    if (w.empty()) {
        m.weights.push_back(1.0f / (0.0f + 1.0f));
        return m;
    }
    for (float& k : w) k *= 1.0f / (1.0f + 1.0f);
    w.push_back(1.0f / (1.0f + 1.0f));
    m.weights = w;
    return m;
}

struct Ctx {
    const SceneO* sc;
    const Mixture* mix;
    int depth_max;
};

// DdfFromLight::value (lighting.cpp:136-148) for d != vec3()
float light_ddf_value(const AreaLightO& l, V3 origin, V3 direction) {
    V3 p, n;
    float s;
    if (!l.traceRay(origin, direction, &p, &n, &s)) return 0.0f;
    V3 dir = normalize(p - origin);
    float cosinus = dot(n, -dir);
    if (cosinus < 0.0f) return 0.0f;
    float decay = dot(p - origin, p - origin);
    return decay / cosinus / l.area;
}

// main.cpp:98-184
float ray_power(const Ctx& cx, V3 origin, V3 direction, int depth, int n_rays) {
    if (depth == cx.depth_max) return 0.0f;
    const SceneO& sc = *cx.sc;
    SurfHit si;
    bool has_si = geometry_trace(sc, origin, direction, &si);
    V3 lpos;
    float lpow;
    bool has_li = lighting_trace(sc, origin, direction, &lpos, &lpow);
    if (g_cnt) {
        if (has_si) ++g_cnt->surf;
        if (has_li) ++g_cnt->light;
    }
    if (has_li) {
        if (!has_si || length(si.position - origin) > length(lpos - origin)) {
            return std::isfinite(lpow) ? lpow : 1.0f;
        }
    }
    if (!has_si) return 0.0f;
    if (g_cnt) ++g_cnt->expanded;  // distributionInPoint call
    // surface DDF: RotateDdf(CosineDdf, normal), or the floor's plain CosineDdf
    RotatedCosine sdf = si.plain_cosine ? RotatedCosine::plain() : RotatedCosine(si.normal);
    if (g_cnt && !(si.normal.x == 0.0f && si.normal.y == 0.0f) &&
        !(si.normal.y == 0.0f && si.normal.z == 0.0f) && !(si.normal.x == 0.0f && si.normal.z == 0.0f))
        ++g_cnt->sframes;
    const std::vector<float>& w = cx.mix->weights;
    const int nl = (int)sc.lights.size();
    float res = 0.0f;
    for (int i = 0; i < n_rays; ++i) {
        if (g_cnt) ++g_cnt->iters;
#ifdef IPT_ORACLE_ITER_HOOK
        const uint32_t k_at = g_rng ? g_rng->k : 0u;  // analysis builds only (scripts/skip_stats.cpp)
#endif
        // UnionDdf::sample (ddf.cpp:139-154)
        V3 new_direction = mk(0, 0, 0);  // fall-through (sum of weights < 1): defined as vec3()
        float r = randf();
        float acc = 0.0f;
        for (int c = 0; c <= nl; ++c) {
            acc += w[c];
            if (r < acc) {
                if (c < nl) {
                    if (g_cnt) ++g_cnt->lsamp;
                    // DdfFromLight::sample (lighting.cpp:125-134)
                    V3 p, n;
                    float s;
                    sc.lights[c].sample(&p, &n, &s);
                    V3 dir = normalize(p - si.position);
                    float cosinus = dot(n, -dir);
                    new_direction = cosinus < 1e-5f ? mk(0, 0, 0) : dir;
                } else {
                    new_direction = sdf.sample();
                }
                break;
            }
        }
#ifdef IPT_ORACLE_ITER_HOOK
        IPT_ORACLE_ITER_HOOK(depth, i, n_rays, k_at, new_direction == mk(0, 0, 0), si.position);
#endif
        if (new_direction == mk(0, 0, 0)) {
            if (g_cnt) ++g_cnt->skipped;
            continue;
        }
        // UnionDdf::value (ddf.cpp:157-162)
        float mix_val = 0.0f;
        for (int c = 0; c < nl; ++c)
            mix_val += w[c] * light_ddf_value(sc.lights[c], si.position, new_direction);
        mix_val += w[nl] * sdf.value(new_direction);
        float sdf_val = sdf.value(new_direction);
        float multiplier = sdf_val / mix_val;
        if (g_cnt && !std::isfinite(multiplier)) ++g_cnt->nf_mults;  // main.cpp:175's assert
        const float albedo = 1.0f;
        res += multiplier * albedo *
               ray_power(cx, si.position, new_direction, depth + 1, n_rays / 2);
    }
    if (g_cnt && !std::isfinite(res)) ++g_cnt->nf_sums;  // main.cpp:181
    res = std::isfinite(res) ? res / n_rays : 0.0f;
    return res;
}

SceneO make_scene(const ipt_scene* s) {
    SceneO o;
    o.geometry_kind = s->geometry_kind;
    for (int i = 0; i < s->n_lights; ++i) {
        const ipt_area_light& L = s->lights[i];
        o.lights.emplace_back(mk(L.position[0], L.position[1], L.position[2]),
                              mk(L.x_axis[0], L.x_axis[1], L.x_axis[2]),
                              mk(L.y_axis[0], L.y_axis[1], L.y_axis[2]), L.power, L.type);
    }
    for (int i = 0; i < s->n_spheres; ++i) {
        o.sph_r.push_back(s->spheres[i].radius);
        o.sph_c.push_back(mk(s->spheres[i].center[0], s->spheres[i].center[1], s->spheres[i].center[2]));
    }
    const ipt_camera& c = s->camera;
    o.cam_pos = mk(c.position[0], c.position[1], c.position[2]);
    o.cam_dir = mk(c.direction[0], c.direction[1], c.direction[2]);
    o.cam_right = mk(c.right[0], c.right[1], c.right[2]);
    o.cam_up = mk(c.up[0], c.up[1], c.up[2]);
    return o;
}

}  // namespace

extern "C" {

// One sample of render_sample's pixel loop (main.cpp:189-216) generalised to
// W x H; returns the clamped value and the GridRenderPlane::addRay target
// (GridRenderPlane.cpp:66-67).
static float oracle_pixel(const Ctx& cx, const ipt_params* p, int ix, int iy, int s,
                          int* xi_out, int* yi_out) {
    Rng rng;
    rng.k0 = (uint32_t)p->seed;
    rng.k1 = (uint32_t)(p->seed >> 32);
    rng.s = (uint32_t)(p->spp_offset + s);
    rng.p = (uint32_t)(iy * p->width + ix);
    g_rng = &rng;
    float x = ((float)ix + randf()) / (float)p->width;
    float y = ((float)iy + randf()) / (float)p->height;
    if (x == 1.0f) x = std::nextafter(x, 0.0f);
    if (y == 1.0f) y = std::nextafter(y, 0.0f);
    const SceneO& sc = *cx.sc;
    // SimpleCamera::sampleRay (SimpleCamera.cpp:15-21)
    float cxp = x - 0.5f, cyp = y - 0.5f;
    V3 ray = sc.cam_right * cxp + sc.cam_up * cyp + sc.cam_dir;
    V3 direction = normalize(ray);
    if (g_cnt) ++g_cnt->paths;
    float value = ray_power(cx, sc.cam_pos, direction, 0, p->n_rays);
    value = value >= 0.0f ? value : 0.0f;
    // GridRenderPlane::addRay index math
    size_t W = (size_t)p->width, H = (size_t)p->height;
    size_t xi = x * W;
    float fy = H - y * H - 1;
    size_t yi = fy;  // values in (-1,0) truncate to 0
    *xi_out = (int)xi;
    *yi_out = (int)yi;
    g_rng = nullptr;
    return value;
}

// GridRenderPlane target (xi, yi) of source pixel (ix, iy) relative to its
// nominal destination (ix, max(H-2-iy, 0)), as ipt_render_values' codes.
static uint8_t drift_code(int W, int H, int ix, int iy, int xi, int yi) {
    const int yn = H - 2 - iy > 0 ? H - 2 - iy : 0;
    const int dx = xi - ix, dy = yi - yn;
    uint8_t code = 0xff;
    if (dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1 && xi < W && yi < H) code = (uint8_t)((dx + 1) | ((dy + 1) << 2));
    return code;
}

// values/codes: [spp][H][W]; codes as in ipt_render_values. counters may be NULL.
int ipt_oracle_render_values(const ipt_scene* scene, const ipt_params* p, float* values,
                             uint8_t* codes, int n_threads, ipt_counters* counters) {
    if (!scene || !p || !values || !codes || p->width <= 0 || p->height <= 0 || p->spp < 0)
        return IPT_E_INVALID;
    SceneO sc = make_scene(scene);
    Mixture mix = build_mixture(sc);
    Ctx cx{&sc, &mix, p->depth_max};
    const int W = p->width, H = p->height;
    const int64_t rows = (int64_t)p->spp * H;
    std::atomic<int64_t> next{0};
    if (n_threads <= 0) n_threads = (int)std::thread::hardware_concurrency();
    std::vector<Counters> percnt(n_threads);
    auto work = [&](int tid) {
        g_cnt = counters ? &percnt[tid] : nullptr;
        for (;;) {
            int64_t r = next.fetch_add(1);
            if (r >= rows) break;
            int s = (int)(r / H), iy = (int)(r % H);
            for (int ix = 0; ix < W; ++ix) {
                int xi, yi;
                float v = oracle_pixel(cx, p, ix, iy, s, &xi, &yi);
                const uint8_t code = drift_code(W, H, ix, iy, xi, yi);
                if (g_cnt && code != 0x05) ++g_cnt->drifted;
                int64_t idx = ((int64_t)s * H + iy) * W + ix;
                values[idx] = v;
                codes[idx] = code;
            }
        }
        g_cnt = nullptr;
    };
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(work, t);
    for (auto& t : th) t.join();
    if (counters) {
        ipt_counters c{};
        for (auto& q : percnt) {
            c.paths += q.paths; c.traced_rays += q.traced; c.surface_hits += q.surf;
            c.light_hits += q.light; c.expanded_nodes += q.expanded; c.iterations += q.iters;
            c.light_samples += q.lsamp; c.skipped += q.skipped; c.sphere_frames += q.sframes;
            c.light_traces += q.ltraces; c.drifted += q.drifted;
        }
        *counters = c;
    }
    return IPT_OK;
}

// GridRenderPlane::addRay replay (GridRenderPlane.cpp:61-75) in render_sample
// order: passes, then rows, then columns. pixel_max/sums may be NULL.
int ipt_oracle_accumulate(int W, int H, int spp, const float* values, const uint8_t* codes,
                          float* pixels, uint32_t* counters, float* sums, float* pixel_max) {
    for (int s = 0; s < spp; ++s)
        for (int iy = 0; iy < H; ++iy)
            for (int ix = 0; ix < W; ++ix) {
                int64_t idx = ((int64_t)s * H + iy) * W + ix;
                uint8_t c = codes[idx];
                if (c == 0xff) return IPT_E_INVALID;
                int yn = H - 2 - iy > 0 ? H - 2 - iy : 0;
                int xi = ix + (c & 3) - 1, yi = yn + ((c >> 2) & 3) - 1;
                int64_t d = (int64_t)yi * W + xi;
                float v = values[idx];
                size_t cnt = counters[d];
                pixels[d] = (pixels[d] * cnt + v) / (cnt + 1);
                counters[d] = (uint32_t)(cnt + 1);
                if (sums) sums[d] += v;
                if (pixel_max && pixels[d] > pixel_max[d]) pixel_max[d] = pixels[d];
            }
    return IPT_OK;
}

// ---- function-level probes (pinned against oracle/_ref in tests) ---------
float ipt_oracle_box_plane(const float* plane, const float* o, const float* d) {
    return intersection_with_box_plane(mk(plane[0], plane[1], plane[2]), mk(o[0], o[1], o[2]),
                                       mk(d[0], d[1], d[2]));
}
float ipt_oracle_sphere(float r, const float* o, const float* d) {
    return intersection_with_sphere(r, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]));
}
// GeometrySphereInBox hit: returns 0/1, writes position[3], normal[3]
int ipt_oracle_trace_box(const float* o, const float* d, float* out6) {
    SceneO sc;
    sc.geometry_kind = IPT_GEOM_SPHERE_IN_BOX;
    SurfHit h;
    if (!geometry_trace(sc, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), &h)) return 0;
    out6[0] = h.position.x; out6[1] = h.position.y; out6[2] = h.position.z;
    out6[3] = h.normal.x; out6[4] = h.normal.y; out6[5] = h.normal.z;
    return 1;
}
// AreaLight: out = {area, surface_power}; trace: returns hit, writes pos[3]
void ipt_oracle_area_light(const ipt_area_light* L, float* area_sp) {
    AreaLightO l(mk(L->position[0], L->position[1], L->position[2]),
                 mk(L->x_axis[0], L->x_axis[1], L->x_axis[2]),
                 mk(L->y_axis[0], L->y_axis[1], L->y_axis[2]), L->power, L->type);
    area_sp[0] = l.area;
    area_sp[1] = l.power / l.area;
}
int ipt_oracle_light_trace(const ipt_area_light* L, const float* o, const float* d, float* pos) {
    AreaLightO l(mk(L->position[0], L->position[1], L->position[2]),
                 mk(L->x_axis[0], L->x_axis[1], L->x_axis[2]),
                 mk(L->y_axis[0], L->y_axis[1], L->y_axis[2]), L->power, L->type);
    V3 p, n;
    float s;
    if (!l.traceRay(mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), &p, &n, &s)) return 0;
    pos[0] = p.x; pos[1] = p.y; pos[2] = p.z;
    return 1;
}
// RotateDdf(CosineDdf, to): transformation (9, column-major) and inverse (9)
void ipt_oracle_rotate(const float* to, float* m18) {
    RotatedCosine r(mk(to[0], to[1], to[2]));
    for (int c = 0; c < 3; ++c)
        for (int k = 0; k < 3; ++k) {
            m18[c * 3 + k] = r.transformation.m[c][k];
            m18[9 + c * 3 + k] = r.inv.m[c][k];
        }
}
// SimpleCamera ctor (SimpleCamera.cpp:8-13): right, up
void ipt_oracle_camera(const float* pos, const float* dir, const float* up_hint, float* right_up) {
    (void)pos;
    V3 d = mk(dir[0], dir[1], dir[2]);
    V3 r = normalize(cross(d, mk(up_hint[0], up_hint[1], up_hint[2])));
    V3 u = normalize(cross(r, d));
    right_up[0] = r.x; right_up[1] = r.y; right_up[2] = r.z;
    right_up[3] = u.x; right_up[4] = u.y; right_up[5] = u.z;
}
void ipt_oracle_mixture_weights(const float* powers, int n, float* w) {
    SceneO sc;
    for (int i = 0; i < n; ++i)
        sc.lights.emplace_back(mk(0, 0, 0), mk(1, 0, 0), mk(0, 1, 0), powers[i], 0);
    Mixture m = build_mixture(sc);
    for (size_t i = 0; i < m.weights.size(); ++i) w[i] = m.weights[i];
}
// CosineDdf::value (ddf.cpp:232-238) on a local vector
float ipt_oracle_cosine_value(float z) {
    if (z < 0.0f) return 0.0f;
    return z / M_PI;
}
// Draw k of the per-path stream, for RNG fixture tests.
float ipt_oracle_randf(uint64_t seed, uint32_t pass, uint32_t pixel, uint32_t k) {
    Rng rng;
    rng.k0 = (uint32_t)seed;
    rng.k1 = (uint32_t)(seed >> 32);
    rng.s = pass;
    rng.p = pixel;
    rng.k = k;
    g_rng = &rng;
    float v = randf();
    g_rng = nullptr;
    return v;
}
}

extern "C" {
// CPU-baseline leg of bench.py: renders source rows iy = row_phase (mod
// row_step) of every pass in p with n_threads threads and returns the sum of
// the clamped values (so nothing is optimised away); *paths = samples done.
double ipt_oracle_render_rows(const ipt_scene* scene, const ipt_params* p, int row_step,
                              int row_phase, int n_threads, uint64_t* paths) {
    SceneO sc = make_scene(scene);
    Mixture mix = build_mixture(sc);
    Ctx cx{&sc, &mix, p->depth_max};
    const int W = p->width, H = p->height;
    std::vector<int> rows;
    for (int iy = row_phase; iy < H; iy += row_step) rows.push_back(iy);
    const int64_t nrows = (int64_t)p->spp * (int64_t)rows.size();
    std::atomic<int64_t> next{0};
    if (n_threads <= 0) n_threads = (int)std::thread::hardware_concurrency();
    std::vector<double> part(n_threads, 0.0);
    auto work = [&](int tid) {
        double acc = 0.0;
        for (;;) {
            int64_t r = next.fetch_add(1);
            if (r >= nrows) break;
            int s = (int)(r / (int64_t)rows.size());
            int iy = rows[r % (int64_t)rows.size()];
            for (int ix = 0; ix < W; ++ix) {
                int xi, yi;
                acc += oracle_pixel(cx, p, ix, iy, s, &xi, &yi);
            }
        }
        part[tid] = acc;
    };
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(work, t);
    for (auto& t : th) t.join();
    double total = 0.0;
    for (double v : part) total += v;
    if (paths) *paths = (uint64_t)nrows * (uint64_t)W;
    return total;
}

// Full-size parity (tests/test_gpu_parity.py): the clamped root values of the
// source pixels (ix, iy) with iy = row_phase (mod row_step) and
// ix = col_phase (mod col_step) of every pass in p, as values[s][r][c].
int ipt_oracle_render_rows_values(const ipt_scene* scene, const ipt_params* p, int row_step, int row_phase,
                                  int col_step, int col_phase, int n_threads, float* values) {
    if (!scene || !p || !values || row_step <= 0 || row_phase < 0 || col_step <= 0 || col_phase < 0)
        return IPT_E_INVALID;
    SceneO sc = make_scene(scene);
    Mixture mix = build_mixture(sc);
    Ctx cx{&sc, &mix, p->depth_max};
    const int W = p->width, H = p->height;
    std::vector<int> rows;
    for (int iy = row_phase; iy < H; iy += row_step) rows.push_back(iy);
    const int64_t nr = (int64_t)rows.size(), nrows = (int64_t)p->spp * nr;
    const int64_t nc = col_phase < W ? (W - 1 - col_phase) / col_step + 1 : 0;
    // one path per work item: a sparse sample (C3's 128 paths per call) has
    // fewer rows than threads, and path costs vary by orders of magnitude
    std::atomic<int64_t> next{0};
    if (n_threads <= 0) n_threads = (int)std::thread::hardware_concurrency();
    auto work = [&]() {
        for (;;) {
            const int64_t i = next.fetch_add(1);
            if (i >= nrows * nc) break;
            const int64_t r = i / nc;
            const int s = (int)(r / nr), q = (int)(r % nr), c = (int)(i % nc);
            int xi, yi;
            values[i] = oracle_pixel(cx, p, col_phase + c * col_step, rows[q], s, &xi, &yi);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(work);
    for (auto& t : th) t.join();
    return IPT_OK;
}
}

extern "C" {
// AreaLight::sample with explicit draws (lighting.cpp:93-104): pos(3), normal(3)
void ipt_oracle_light_sample_uv(const ipt_area_light* L, float u1, float u2raw, float* out6) {
    AreaLightO l(mk(L->position[0], L->position[1], L->position[2]),
                 mk(L->x_axis[0], L->x_axis[1], L->x_axis[2]),
                 mk(L->y_axis[0], L->y_axis[1], L->y_axis[2]), L->power, L->type);
    float u2 = u2raw * (l.type == 1 ? 1.0f - u1 : 1.0f);
    V3 pos = l.x_axis * u1 + l.y_axis * u2;
    V3 p = pos + l.position;
    V3 n = normalize(cross(l.x_axis, l.y_axis));
    out6[0] = p.x; out6[1] = p.y; out6[2] = p.z;
    out6[3] = n.x; out6[4] = n.y; out6[5] = n.z;
}
// SimpleCamera::sampleRay (SimpleCamera.cpp:15-21): direction(3)
void ipt_oracle_camera_ray(const float* dir, const float* right, const float* up, float x,
                           float y, float* out3) {
    x -= 0.5f;
    y -= 0.5f;
    V3 ray = mk(right[0], right[1], right[2]) * x + mk(up[0], up[1], up[2]) * y +
             mk(dir[0], dir[1], dir[2]);
    V3 d = normalize(ray);
    out3[0] = d.x; out3[1] = d.y; out3[2] = d.z;
}
// CollectionLighting::traceRayToLight over n lights: returns hit, pos(3), power
int ipt_oracle_collection_trace(const ipt_area_light* L, int n, const float* o, const float* d,
                                float* out4) {
    SceneO sc;
    for (int i = 0; i < n; ++i)
        sc.lights.emplace_back(mk(L[i].position[0], L[i].position[1], L[i].position[2]),
                               mk(L[i].x_axis[0], L[i].x_axis[1], L[i].x_axis[2]),
                               mk(L[i].y_axis[0], L[i].y_axis[1], L[i].y_axis[2]), L[i].power,
                               L[i].type);
    V3 p;
    float s;
    if (!lighting_trace(sc, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), &p, &s)) return 0;
    out4[0] = p.x; out4[1] = p.y; out4[2] = p.z; out4[3] = s;
    return 1;
}
// GridRenderPlane::addRay on an explicit (x, y, v) sequence (GridRenderPlane.cpp:61-75)
void ipt_oracle_grid_addray(int W, int H, int n, const float* xyv, float* pixels,
                            uint32_t* counters, float* max_value) {
    float mx = 0.0f;
    for (int i = 0; i < n; ++i) {
        float x = xyv[3 * i], y = xyv[3 * i + 1], v = xyv[3 * i + 2];
        size_t xi = x * (size_t)W;
        float fy = (size_t)H - y * (size_t)H - 1;
        size_t yi = fy;
        size_t d = yi * W + xi;
        size_t c = counters[d];
        pixels[d] = (pixels[d] * c + v) / (c + 1);
        counters[d] = (uint32_t)(c + 1);
        if (pixels[d] > mx) mx = pixels[d];
    }
    *max_value = mx;
}
}

extern "C" {
// n samples of RotateDdf(CosineDdf, to)::sample (ddf_detail.h:69-72, ddf.cpp:223-231)
// drawn from the per-path stream (seed, pass 0, pixel 0); for the chi^2 test.
void ipt_oracle_cosine_samples(uint64_t seed, const float* to, int n, float* out3n) {
    Rng rng;
    rng.k0 = (uint32_t)seed;
    rng.k1 = (uint32_t)(seed >> 32);
    rng.s = 0;
    rng.p = 0;
    g_rng = &rng;
    RotatedCosine r(mk(to[0], to[1], to[2]));
    for (int i = 0; i < n; ++i) {
        V3 v = r.sample();
        out3n[3 * i] = v.x; out3n[3 * i + 1] = v.y; out3n[3 * i + 2] = v.z;
    }
    g_rng = nullptr;
}
// RotateDdf(CosineDdf, to)::value (ddf_detail.h:74-76)
float ipt_oracle_cosine_ddf_value(const float* to, const float* d) {
    RotatedCosine r(mk(to[0], to[1], to[2]));
    return r.value(mk(d[0], d[1], d[2]));
}
}

extern "C" {
// Per-path event counts (SURVEY.md Appendix C vocabulary) for the statistical
// pin of the estimator (tests/test_oracle_stats.py): for every path of
// render_values' order, values[i] (clamped root value) and
// ev[i*IPT_ORACLE_NEV + e] for e = traced rays, geometry hits, light hits,
// expanded nodes, iterations, light-sampled iterations, skipped iterations,
// AreaLight::traceRay calls, non-finite node sums (main.cpp:181), non-finite
// multipliers (main.cpp:175), randf() draws.
#define IPT_ORACLE_NEV 11
int ipt_oracle_nev(void) { return IPT_ORACLE_NEV; }
int ipt_oracle_render_events(const ipt_scene* scene, const ipt_params* p, int n_threads, float* values,
                             uint8_t* codes, uint32_t* ev) {
    if (!scene || !p || !values || !codes || !ev || p->width <= 0 || p->height <= 0 || p->spp < 0) return IPT_E_INVALID;
    SceneO sc = make_scene(scene);
    Mixture mix = build_mixture(sc);
    Ctx cx{&sc, &mix, p->depth_max};
    const int W = p->width, H = p->height;
    const int64_t rows = (int64_t)p->spp * H;
    std::atomic<int64_t> next{0};
    if (n_threads <= 0) n_threads = (int)std::thread::hardware_concurrency();
    auto work = [&]() {
        for (;;) {
            int64_t r = next.fetch_add(1);
            if (r >= rows) break;
            int s = (int)(r / H), iy = (int)(r % H);
            for (int ix = 0; ix < W; ++ix) {
                Counters c;
                g_cnt = &c;
                int xi, yi;
                const float v = oracle_pixel(cx, p, ix, iy, s, &xi, &yi);
                g_cnt = nullptr;
                const int64_t idx = ((int64_t)s * H + iy) * W + ix;
                values[idx] = v;
                codes[idx] = drift_code(W, H, ix, iy, xi, yi);
                const uint64_t e[IPT_ORACLE_NEV] = {c.traced, c.surf, c.light, c.expanded, c.iters, c.lsamp,
                                                    c.skipped, c.ltraces, c.nf_sums, c.nf_mults, c.draws};
                for (int q = 0; q < IPT_ORACLE_NEV; ++q) ev[idx * IPT_ORACLE_NEV + q] = (uint32_t)e[q];
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(work);
    for (auto& t : th) t.join();
    return IPT_OK;
}

// Philox4x32-10 block (the randf() replacement's generator) for known-answer
// tests against Random123's published vectors: out = philox(ctr[4], key[2]).
void ipt_oracle_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    philox(c, key[0], key[1]);
    for (int i = 0; i < 4; ++i) out[i] = c[i];
}
}

// ------------------------------------------------------------ post-process
// Literal restatements of the reference's image post-process (SURVEY.md §8(f)
// row 2), same loop order and types, for tests/test_post.py.
extern "C" {
// GridRenderPlane::smooth (in_place = 1) / computeSmoothedMax (in_place = 0),
// GridRenderPlane.cpp:10-59: y, x downwards from the bottom-right, size_t
// bounds `y >= side-1` (side 0: no iteration; side 1 would wrap: rejected).
int ipt_oracle_smooth(float* pixels, size_t width, size_t height, size_t side, int in_place, float* max_out) {
    if (side == 1) return -1;
    float max_value = 0.0f;
    if (height == 0 || width == 0) { *max_out = 0.0f; return 0; }
    for (size_t y = height - 1; y >= side - 1; --y) {
        for (size_t x = width - 1; x >= side - 1; --x) {
            float accum = 0.0f;
            for (size_t yy = 0; yy < side; ++yy)
                for (size_t xx = 0; xx < side; ++xx) accum += pixels[(y - yy) * width + x - xx];
            accum /= side * side;
            if (in_place) pixels[y * width + x] = accum;
            if (accum > max_value) max_value = accum;
            if (x == 0) break;
        }
        if (y == 0) break;
    }
    *max_out = max_value;
    return 0;
}

// gui.cpp:28-52: draw_halo(img, cx, cy, C, r0) adds C/(r0+r)/(r0+r) with
// r = (float)hypot(x-cx, y-cy) to every pixel; glare copies the image, draws a
// halo of C = cutoff*(float)(0.1*val/cutoff) for every pixel with
// !(val <= cutoff) in raster order, then cuts to [0, cutoff].
void ipt_oracle_glare(const float* img, float* out, int width, int height, float cutoff) {
    std::vector<float> o(img, img + (size_t)width * height);
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) {
            float val = img[(size_t)y * width + x];
            if (val <= cutoff) continue;
            float coef = 0.1 * val / cutoff;
            const float C = cutoff * coef, r0 = 0.25f;
            for (int yy = 0; yy < height; ++yy)
                for (int xx = 0; xx < width; ++xx) {
                    float r = std::hypot(xx - x, yy - y);
                    float v = C / (r0 + r) / (r0 + r);
                    o[(size_t)yy * width + xx] += v;
                }
        }
    for (size_t i = 0; i < o.size(); ++i) {
        const float v = o[i];
        out[i] = v < 0.0f ? 0.0f : (v > cutoff ? cutoff : v);
    }
}
}

// ---------------------------------------------------------------- DDFs
// The three samplers of the path with explicit uniforms (3 per sample: pick,
// u1, u2), for tests/test_ddf_samplers.py (device parity + the reference's
// chi^2 harness check_ddf.cpp:114-203). kind 0: RotateDdf(CosineDdf, to),
// params = to; kind 1: DdfFromLight of light params[3] at origin params[0..2]
// (lighting.cpp:125-148); kind 2: UnionDdf of all lights + RotateDdf(CosineDdf,
// normal) with the scene's unite() weights (ddf.cpp:142-162), origin
// params[0..2], normal params[3..5].
namespace {
V3 light_ddf_sample(const AreaLightO& l, V3 o) {
    V3 pos, n;
    float sp;
    l.sample(&pos, &n, &sp);
    V3 dir = normalize(pos - o);
    if (dot(n, -dir) < 1e-5f) return mk(0.0f, 0.0f, 0.0f);  // lighting.cpp:130-131
    return dir;
}
}  // namespace
extern "C" {
int ipt_oracle_ddf_sample(const ipt_scene* scene, int kind, const float* params, const float* u, int n,
                          float* out3n) {
    SceneO sc = make_scene(scene);
    const V3 o = mk(params[0], params[1], params[2]);
    Mixture mx = build_mixture(sc);
    for (int i = 0; i < n; ++i) {
        V3 v = mk(0.0f, 0.0f, 0.0f);
        if (kind == 0) {
            g_ufeed = u + 3 * i + 1;
            v = RotatedCosine(o).sample();
        } else if (kind == 1) {
            g_ufeed = u + 3 * i + 1;
            v = light_ddf_sample(sc.lights[(int)params[3]], o);
        } else {
            g_ufeed = u + 3 * i;
            const float r = randf();  // UnionDdf::sample: first r < running sum
            float acc = 0.0f;
            size_t c = 0;
            for (; c < mx.weights.size(); ++c) {
                acc += mx.weights[c];
                if (r < acc) break;
            }
            if (c < sc.lights.size()) v = light_ddf_sample(sc.lights[c], o);
            else if (c == sc.lights.size()) v = RotatedCosine(mk(params[3], params[4], params[5])).sample();
        }
        g_ufeed = nullptr;
        out3n[3 * i] = v.x; out3n[3 * i + 1] = v.y; out3n[3 * i + 2] = v.z;
    }
    return 0;
}
int ipt_oracle_ddf_value(const ipt_scene* scene, int kind, const float* params, const float* dirs, int n,
                         float* out) {
    SceneO sc = make_scene(scene);
    const V3 o = mk(params[0], params[1], params[2]);
    Mixture mx = build_mixture(sc);
    for (int i = 0; i < n; ++i) {
        const V3 d = mk(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
        float v;
        if (kind == 0) {
            v = RotatedCosine(o).value(d);
        } else if (kind == 1) {
            v = light_ddf_value(sc.lights[(int)params[3]], o, d);
        } else {
            v = 0.0f;  // UnionDdf::value: sequential sum in component order
            for (size_t c = 0; c < sc.lights.size(); ++c) v += mx.weights[c] * light_ddf_value(sc.lights[c], o, d);
            v += mx.weights.back() * RotatedCosine(mk(params[3], params[4], params[5])).value(d);
        }
        out[i] = v;
    }
    return 0;
}
}
