// ORACLE pinning harness — test infrastructure only.
//
// Linked against the reference's OWN translation units compiled from
// /root/reference by oracle/build_ref.sh (geometric_utils.cpp, lighting.cpp,
// CollectionLighting.cpp, SimpleCamera.cpp, GridRenderPlane.cpp,
// sample_scenes.cpp and the geometry TUs it names). It evaluates those
// functions on deterministic + adversarial inputs and writes the results as
// binary fixtures to tests/golden/ref_*.bin; tests/test_oracle_vs_ref.py
// checks the CPU oracle (oracle/ipt_oracle.cpp) against them bit-for-bit.
//
// Not built/linked: libddf/ddf.cpp and main.cpp (they need boost/config.hpp,
// absent from this image). Code paths of the linked TUs that would call into
// them (Ddf allocation, CosineDdf, unite) are never executed here.
#include "geometric_utils.h"
#include "GridRenderPlane.h"
#include "SimpleCamera.h"
#include "CollectionLighting.h"
#include "lighting/lighting.h"
#include "sample_scenes.h"
#include "geometry/FractalSpheres.h"
#include <functional>
#include "libddf/ddf_detail.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

using glm::vec3;

// FractalSpheres.cpp:16 (a free function the header does not declare)
void generate_spheres(float r1, vec3 c1, float r2, vec3 c2, bool light_from_left,
                      std::function<bool(float r, vec3 c)> callback);

namespace {

std::string g_dir;

void write(const char* name, const std::vector<float>& v) {
    std::string p = g_dir + "/" + name;
    FILE* f = std::fopen(p.c_str(), "wb");
    if (!f) { std::perror(p.c_str()); std::exit(1); }
    std::fwrite(v.data(), sizeof(float), v.size(), f);
    std::fclose(f);
}

std::mt19937 rng(20241223);
float U(float a, float b) { return std::uniform_real_distribution<float>(a, b)(rng); }
vec3 unit() {
    for (;;) {
        vec3 v(U(-1, 1), U(-1, 1), U(-1, 1));
        float l = glm::length(v);
        if (l > 0.1f && l <= 1.0f) return glm::normalize(v);
    }
}
// "snap" a coordinate to a special value now and then (walls, edges, zeros)
float special(float x) {
    switch (rng() % 10) {
        case 0: return 1.0f;
        case 1: return -1.0f;
        case 2: return 0.0f;
        case 3: return std::nextafter(1.0f, 2.0f);
        case 4: return std::nextafter(1.0f, 0.0f);
        default: return x;
    }
}

// A probe origin for RotateDdf: records the vector value() is called with and
// returns a fixed vector from sample(). Owns its allocation (class-specific
// new/delete), so nothing of the unbuilt ddf.cpp is touched.
struct Probe : public Ddf {
    mutable vec3 last;
    vec3 out;
    glm::vec3 sample() const override { return out; }
    float value(glm::vec3 a) const override { last = a; return 0.0f; }
    static void* operator new(size_t n) { return std::malloc(n); }
    static void operator delete(void* p) { std::free(p); }
};

}  // namespace

int main(int argc, char** argv) {
    g_dir = argc > 1 ? argv[1] : ".";
    const int N = 4000;

    // 1. intersection_with_box_plane: plane(3) o(3) d(3) -> t
    {
        static const vec3 planes[] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {-1, 0, 0}, {0, 0, -1}};
        std::vector<float> out;
        for (int i = 0; i < N; ++i) {
            vec3 p = planes[i % 5];
            vec3 o(special(U(-1, 1)), special(U(-1, 1)), special(U(-1, 1)));
            vec3 d = unit();
            if (i % 7 == 0) d[rng() % 3] = 0.0f;
            if (i % 11 == 0) d = glm::normalize(vec3(special(d.x), special(d.y), d.z));
            float t = intersection_with_box_plane(p, o, d);
            float rec[] = {p.x, p.y, p.z, o.x, o.y, o.z, d.x, d.y, d.z, t};
            out.insert(out.end(), rec, rec + 10);
        }
        write("ref_box_plane.bin", out);
    }
    // 2. intersection_with_sphere: r o(3) d(3) -> t
    {
        std::vector<float> out;
        for (int i = 0; i < N; ++i) {
            float r = (i % 3 == 0) ? 0.5f : U(0.01f, 1.0f);
            vec3 o(U(-3, 3), U(-3, 3), U(-3, 3));
            if (i % 5 == 0) o = glm::normalize(o) * r;  // on the sphere
            vec3 d = unit();
            if (i % 4 == 0) d = glm::normalize(-o + vec3(U(-0.3f, 0.3f), U(-0.3f, 0.3f), U(-0.3f, 0.3f)));
            float t = intersection_with_sphere(r, o, d);
            float rec[] = {r, o.x, o.y, o.z, d.x, d.y, d.z, t};
            out.insert(out.end(), rec, rec + 8);
        }
        write("ref_sphere.bin", out);
    }
    // 3. AreaLight ctor + traceRay: P x y power type o d -> area spow hit pos(3)
    {
        std::vector<float> out;
        for (int i = 0; i < N; ++i) {
            vec3 P(U(-1, 1), U(-1, 1), U(-1, 1));
            vec3 x = unit() * U(0.05f, 1.0f), y = unit() * U(0.05f, 1.0f);
            float power = U(0.1f, 4.0f);
            int type = i % 2;
            if (i % 3 == 0) {  // the sample_scenes[0] light
                P = vec3{+0.1f, -0.8f - 0.1f, -0.15f};
                x = vec3{0.0f, 0.2f, 0.0f};
                y = glm::cross(vec3(0.0f, 0.0f, -1.0f), x);
                power = 1.0f;
                type = 0;
            }
            AreaLight L(P, x, y, power, type ? AreaLight::TYPE_TRIANLE : AreaLight::TYPE_DIAMOND);
            vec3 o(U(-1, 1), U(-1, 1), U(-1, 1));
            vec3 target = P + x * U(-0.1f, 1.1f) + y * U(-0.1f, 1.1f);
            vec3 d = glm::normalize(target - o);
            auto h = L.traceRay(o, d);
            float rec[] = {P.x, P.y, P.z, x.x, x.y, x.z, y.x, y.y, y.z, power, (float)type,
                           o.x, o.y, o.z, d.x, d.y, d.z, L.area, L.power / L.area,
                           h ? 1.0f : 0.0f, h ? h->position.x : 0.0f, h ? h->position.y : 0.0f,
                           h ? h->position.z : 0.0f, h ? h->surface_power : 0.0f};
            out.insert(out.end(), rec, rec + 24);
        }
        write("ref_area_light.bin", out);
    }
    // 4. AreaLight::sample with the reference's own randf (drand48 seeded):
    //    P x y type seed -> u1 u2 pos(3) normal(3)
    {
        std::vector<float> out;
        for (int i = 0; i < 1000; ++i) {
            vec3 P(U(-1, 1), U(-1, 1), U(-1, 1));
            vec3 x = unit() * U(0.05f, 1.0f), y = unit() * U(0.05f, 1.0f);
            int type = i % 2;
            AreaLight L(P, x, y, 1.0f, type ? AreaLight::TYPE_TRIANLE : AreaLight::TYPE_DIAMOND);
            long seed = 1000 + i;
            srand48(seed);
            light_intersection s = L.sample();
            srand48(seed);  // replay randf() (include/randf.h:6-11)
            float u1 = drand48();
            while (u1 == 1.0f) u1 = drand48();
            float u2 = drand48();
            while (u2 == 1.0f) u2 = drand48();
            float rec[] = {P.x, P.y, P.z, x.x, x.y, x.z, y.x, y.y, y.z, (float)type, u1, u2,
                           s.position.x, s.position.y, s.position.z, s.normal.x, s.normal.y,
                           s.normal.z};
            out.insert(out.end(), rec, rec + 18);
        }
        write("ref_light_sample.bin", out);
    }
    // 5. SimpleCamera ctor + sampleRay: pos dir up_hint x y -> right(3) up(3) o(3) d(3)
    {
        std::vector<float> out;
        for (int i = 0; i < N; ++i) {
            vec3 pos(U(-4, 4), U(-4, 4), U(-4, 4));
            vec3 dir = unit() * U(0.5f, 2.0f);
            vec3 up = (i % 2) ? vec3(0, 0, 1) : vec3(0, 1, 0);
            float x = U(0, 1), y = U(0, 1);
            SimpleCamera cam(pos, dir, up);
            auto r = cam.sampleRay(x, y);
            float rec[] = {pos.x, pos.y, pos.z, dir.x, dir.y, dir.z, up.x, up.y, up.z, x, y,
                           cam.right.x, cam.right.y, cam.right.z, cam.up.x, cam.up.y, cam.up.z,
                           r.first.x, r.first.y, r.first.z, r.second.x, r.second.y, r.second.z};
            out.insert(out.end(), rec, rec + 23);
        }
        write("ref_camera.bin", out);
    }
    // 6. make_scene_box(): camera fields + light fields (the flattener's input)
    {
        Scene sc = make_scene_box();
        auto cam = std::dynamic_pointer_cast<const SimpleCamera>(sc.camera);
        auto lit = std::dynamic_pointer_cast<const CollectionLighting>(sc.lighting);
        std::vector<float> out = {cam->position.x, cam->position.y, cam->position.z,
                                  cam->direction.x, cam->direction.y, cam->direction.z,
                                  cam->right.x, cam->right.y, cam->right.z,
                                  cam->up.x, cam->up.y, cam->up.z, (float)lit->lights.size()};
        for (auto& l : lit->lights) {
            out.push_back(l->position.x);
            out.push_back(l->position.y);
            out.push_back(l->position.z);
            out.push_back(l->power);
            out.push_back(l->area);
        }
        // probe the box light through its own traceRay from fixed points
        for (int i = 0; i < 200; ++i) {
            vec3 o(U(-0.9f, 0.9f), U(-0.9f, 0.9f), U(-0.9f, 0.9f));
            vec3 t(U(0.05f, 0.35f), U(-0.95f, -0.65f), -0.15f);
            vec3 d = glm::normalize(t - o);
            auto h = sc.lighting->traceRayToLight(o, d);
            float rec[] = {o.x, o.y, o.z, d.x, d.y, d.z, h ? 1.0f : 0.0f,
                           h ? h->position.x : 0.f, h ? h->position.y : 0.f, h ? h->position.z : 0.f,
                           h ? h->surface_power : 0.f};
            out.insert(out.end(), rec, rec + 11);
        }
        write("ref_scene_box.bin", out);
    }
    // 7. CollectionLighting::traceRayToLight with 16 overlapping lights
    {
        CollectionLighting C;
        std::vector<float> out;
        for (int l = 0; l < 16; ++l) {
            vec3 corner(U(-0.5f, 0.3f), U(-0.5f, 0.3f), U(-0.8f, 0.8f));
            vec3 n = unit();
            vec3 xs = glm::normalize(glm::cross(n, unit())) * U(0.1f, 0.6f);
            float pw = U(0.1f, 2.0f);
            C.addSquareLight(corner, n, xs, pw);
            vec3 ys = glm::cross(n, xs);
            float rec[] = {corner.x, corner.y, corner.z, xs.x, xs.y, xs.z, ys.x, ys.y, ys.z, pw};
            out.insert(out.end(), rec, rec + 10);
        }
        for (int i = 0; i < N; ++i) {
            vec3 o(U(-2, 2), U(-2, 2), U(-2, 2));
            vec3 d = glm::normalize(vec3(U(-0.4f, 0.4f), U(-0.4f, 0.4f), U(-0.4f, 0.4f)) - o);
            auto h = C.traceRayToLight(o, d);
            float rec[] = {o.x, o.y, o.z, d.x, d.y, d.z, h ? 1.0f : 0.0f,
                           h ? h->position.x : 0.f, h ? h->position.y : 0.f, h ? h->position.z : 0.f,
                           h ? h->surface_power : 0.f};
            out.insert(out.end(), rec, rec + 11);
        }
        write("ref_collection.bin", out);
    }
    // 8. RotateDdf (libddf/ddf_detail.h, header-only) around a probe:
    //    to(3) -> transformation(9) inverse(9) sample(x) (3) value-arg(3)
    {
        std::vector<float> out;
        for (int i = 0; i < N; ++i) {
            vec3 to = unit();
            switch (i % 8) {
                case 0: to = vec3(0, 0, 1); break;
                case 1: to = -vec3(0, 0, 1); break;
                case 2: to = -vec3(1, 0, 0); break;
                case 3: to = -vec3(0, 1, 0); break;
                case 4: to = vec3(-0.0f, -0.0f, -1.0f); break;
                default: break;
            }
            auto* p = new Probe();
            p->out = unit();
            vec3 probe_out = p->out;
            RotateDdf R(std::unique_ptr<Ddf>(p), to);
            vec3 s = R.sample();
            vec3 arg = unit();
            R.value(arg);
            vec3 va = p->last;
            std::vector<float> rec = {to.x, to.y, to.z};
            for (int c = 0; c < 3; ++c)
                for (int r = 0; r < 3; ++r) rec.push_back(R.transformation[c][r]);
            for (int c = 0; c < 3; ++c)
                for (int r = 0; r < 3; ++r) rec.push_back(R.inverse[c][r]);
            float tail[] = {probe_out.x, probe_out.y, probe_out.z, s.x, s.y, s.z,
                            arg.x, arg.y, arg.z, va.x, va.y, va.z};
            rec.insert(rec.end(), tail, tail + 12);
            out.insert(out.end(), rec.begin(), rec.end());
        }
        write("ref_rotate.bin", out);
    }
    // 9. GridRenderPlane::addRay sequence: W H then (x y v) -> pixels, counters, max
    {
        const int W = 37, H = 23;
        GridRenderPlane g(W, H);
        std::vector<float> in;
        for (int s = 0; s < 3; ++s)
            for (int iy = 0; iy < H; ++iy)
                for (int ix = 0; ix < W; ++ix) {
                    float u = (rng() % 5 == 0) ? 0.0f : U(0, 1);
                    float w = (rng() % 5 == 0) ? std::nextafter(1.0f, 0.0f) : U(0, 1);
                    float x = (ix + u) / (float)W;
                    float y = (iy + w) / (float)H;
                    if (x == 1.0f) x = std::nextafter(x, 0.0f);
                    if (y == 1.0f) y = std::nextafter(y, 0.0f);
                    float v = U(0, 30);
                    g.addRay(x, y, v);
                    in.push_back(x);
                    in.push_back(y);
                    in.push_back(v);
                }
        std::vector<float> out = {(float)W, (float)H, (float)(in.size() / 3)};
        out.insert(out.end(), in.begin(), in.end());
        for (int i = 0; i < W * H; ++i) out.push_back(g.pixels[i]);
        for (int i = 0; i < W * H; ++i) out.push_back((float)g.pixel_counters[i]);
        out.push_back(g.max_value);
        write("ref_grid.bin", out);
    }
    // 10. GridRenderPlane::smooth(side) and computeSmoothedMax(side)
    //     (GridRenderPlane.cpp:10-59) on random planes (some zero pixels):
    //     per case W H side, input pixels, smoothed pixels, smooth's max,
    //     computeSmoothedMax's max (on the unsmoothed input)
    {
        std::vector<float> out;
        const int cases[][3] = {{37, 23, 2}, {37, 23, 3}, {16, 40, 5}, {9, 9, 9}, {8, 6, 7}, {5, 5, 0}};
        out.push_back((float)(sizeof(cases) / sizeof(cases[0])));
        for (const auto& c : cases) {
            const int W = c[0], H = c[1], side = c[2];
            GridRenderPlane g(W, H), h(W, H);
            for (int i = 0; i < W * H; ++i) g.pixels[i] = h.pixels[i] = (rng() % 7 == 0) ? 0.0f : U(0, 30);
            out.push_back((float)W);
            out.push_back((float)H);
            out.push_back((float)side);
            out.insert(out.end(), g.pixels.begin(), g.pixels.end());
            g.smooth(side);
            h.computeSmoothedMax(side);
            out.insert(out.end(), g.pixels.begin(), g.pixels.end());
            out.push_back(g.max_value);
            out.push_back(h.max_value);
        }
        write("ref_smooth.bin", out);
    }
    // 11. the other sample_scenes (sample_scenes.cpp:43-108): camera fields,
    //     per light position/power/area, and light probes through the scene's
    //     own traceRayToLight (AreaLight, triangle AreaLight, SphereLight)
    {
        std::vector<float> out;
        Scene (*makers[])() = {make_scene_square_lit_by_square, make_scene_lit_corner, make_scene_fractal,
                               make_scene_smallpt};
        out.push_back(4.0f);
        for (auto mk_scene : makers) {
            Scene sc = mk_scene();
            auto cam = std::dynamic_pointer_cast<const SimpleCamera>(sc.camera);
            auto lit = std::dynamic_pointer_cast<const CollectionLighting>(sc.lighting);
            float head[] = {cam->position.x, cam->position.y, cam->position.z, cam->direction.x,
                            cam->direction.y, cam->direction.z, cam->right.x, cam->right.y, cam->right.z,
                            cam->up.x, cam->up.y, cam->up.z, (float)lit->lights.size()};
            out.insert(out.end(), head, head + 13);
            for (auto& l : lit->lights) {
                out.push_back(l->position.x);
                out.push_back(l->position.y);
                out.push_back(l->position.z);
                out.push_back(l->power);
                out.push_back(l->area);
            }
            for (int i = 0; i < 200; ++i) {
                // aim at a point of the light (its own sample(), drand48) from a random origin
                const vec3 t = lit->lights[0]->sample().position;
                const float sc_len = glm::length(cam->position - t);
                vec3 o = t + glm::normalize(vec3(U(-1, 1), U(-1, 1), U(-1, 1))) * U(0.05f, 1.0f) * sc_len;
                vec3 d = glm::normalize(t - o);
                auto hh = sc.lighting->traceRayToLight(o, d);
                float rec[] = {o.x, o.y, o.z, d.x, d.y, d.z, hh ? 1.0f : 0.0f,
                               hh ? hh->position.x : 0.f, hh ? hh->position.y : 0.f, hh ? hh->position.z : 0.f,
                               hh ? hh->surface_power : 0.f};
                out.insert(out.end(), rec, rec + 11);
            }
        }
        write("ref_scenes.bin", out);
    }
    // 12. FractalSpheres' sphere list: the reference's generate_spheres
    //     (FractalSpheres.cpp:16-44) driven as FractalSpheres::FractalSpheres
    //     does (FractalSpheres.cpp:46-67: r1 = r2 = 0.5 at (-2,0,0), (2,0,0),
    //     stop below r = 0.001); rs/cs are private, so the harness collects them
    {
        std::vector<float> rs, cs;
        auto add_sphere = [&](float r, vec3 c) -> bool {
            if (r < 0.001) return true;
            rs.push_back(r);
            cs.push_back(c.x);
            cs.push_back(c.y);
            cs.push_back(c.z);
            return false;
        };
        add_sphere(0.5f, vec3(-2, 0, 0));
        add_sphere(0.5f, vec3(2, 0, 0));
        generate_spheres(0.5f, vec3(-2, 0, 0), 0.5f, vec3(2, 0, 0), true, add_sphere);
        std::vector<float> out = {(float)rs.size()};
        for (size_t i = 0; i < rs.size(); ++i) {
            out.push_back(cs[3 * i]);
            out.push_back(cs[3 * i + 1]);
            out.push_back(cs[3 * i + 2]);
            out.push_back(rs[i]);
        }
        write("ref_fractal_spheres.bin", out);
    }
    std::printf("ref_kat: fixtures written to %s\n", g_dir.c_str());
    return 0;
}
