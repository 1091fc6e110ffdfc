// ipt_host.cpp — see ipt_host.h. Host-only C++ (g++), no HIP headers: every
// GPU call goes through the C-ABI of libipt_hip.so.
#define IPT_HD inline
#include "ipt_host.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <thread>

#include "../csrc/ipt_math.h"  // glm-order float arithmetic (vec3, cross, normalize)

namespace ipt {

namespace {

vec3 g(vec3f v) { return v3(v.x, v.y, v.z); }
vec3f h(vec3 v) { return vec3f{v.x, v.y, v.z}; }

[[noreturn]] void unsupported(const std::string& what) {
    throw IptError(IPT_E_UNSUPPORTED, what + ": not on the GPU path yet (SURVEY.md §8(f) row 1)");
}

void check(ipt_ctx* ctx, int rc) {
    if (rc != IPT_OK) throw IptError(rc, ipt_last_error(ctx));
}

// SplitMix64 (the synthetic scenes' generator, ipt_amd/scenes.py)
struct SplitMix64 {
    uint64_t x;
    uint64_t next() {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    float u() { return (float)(next() >> 40) * 0x1p-24f; }  // exact: 24-bit integer * 2^-24
};

std::shared_ptr<SimpleCamera> box_camera() {
    // sample_scenes.cpp:36-38
    const vec3 camera_pos = v3(0.0f, -3.0f, 0.1f);
    const vec3 camera_dir = normalize(v3(0.0f, 1.0f, -1.0f) - camera_pos);
    return std::make_shared<SimpleCamera>(h(camera_pos), h(camera_dir));
}

vec3f box_light_corner() { return vec3f{+0.1f, -0.8f - 0.1f, -0.15f}; }  // sample_scenes.cpp:30

}  // namespace

AreaLight::AreaLight(vec3f corner, vec3f x, vec3f y, float p, type_t t)
    : position(corner), x_axis(x), y_axis(y), type(t) {
    power = p;
}

void CollectionLighting::addSquareLight(vec3f corner, vec3f normal, vec3f x_side, float power) {
    const vec3 y_side = cross(g(normal), g(x_side));
    lights.push_back(std::make_shared<const AreaLight>(corner, x_side, h(y_side), power, AreaLight::TYPE_DIAMOND));
}
void CollectionLighting::addTriangleLight(vec3f corner, vec3f x_side, vec3f y_side, float power) {
    lights.push_back(std::make_shared<const AreaLight>(corner, x_side, y_side, power, AreaLight::TYPE_TRIANLE));
}
SphereLight::SphereLight(vec3f origin, float r, float p) : position(origin), radius(r) { power = p; }
PointLight::PointLight(vec3f origin, float vr, float p) : position(origin), virtual_radius(vr) { power = p; }
InvertedSphereLight::InvertedSphereLight(vec3f origin, float r, float p) : SphereLight(origin, r, p) {}

// CollectionLighting.cpp:36-55
void CollectionLighting::addPointLight(vec3f position, float virtual_radius, float power) {
    lights.push_back(std::make_shared<const PointLight>(position, virtual_radius, power));
}
void CollectionLighting::addSphereLight(vec3f position, float radius, float power) {
    lights.push_back(std::make_shared<const SphereLight>(position, radius, power));
}
void CollectionLighting::addOuterLight(float radius, float power) {
    lights.push_back(std::make_shared<const InvertedSphereLight>(vec3f{0, 0, 0}, radius, power));
}

// FractalSpheres.cpp:16-44 (generate_spheres) and 46-67 (the constructor),
// float arithmetic with glibc asinf/sinf as the reference's build calls them.
namespace {
void generate_spheres(float r1, vec3 c1, float r2, vec3 c2, bool light_from_left,
                      const std::function<bool(float, vec3)>& callback) {
    const float L = length(c1 - c2) - r1 - r2;
    if (L < 0.01) return;
    const float sin_alpha = r1 / (r1 + L);
    const float alpha = std::asin(sin_alpha);
    const float sin_beta = r2 / (r2 + L);
    const float beta = std::asin(sin_beta);
    const float pi = 3.14159265358979323846f;  // M_PIf32
    const float gamma = pi - alpha - beta;
    const float A = L * sin_alpha / std::sin(gamma);
    const float x = A * std::sin(gamma / 2) / std::sin(pi - beta - gamma / 2);
    const vec3 c3 = c1 + normalize(c2 - c1) * (x + r1);
    const float r3 = x * sin_beta;
    if (callback(r3, c3)) return;
    if (light_from_left)
        generate_spheres(r1, c1, r3, c3, !light_from_left, callback);
    else
        generate_spheres(r3, c3, r2, c2, !light_from_left, callback);
}
}  // namespace

FractalSpheres::FractalSpheres() {
    auto add_sphere = [this](float r, vec3 c) -> bool {
        if (r < 0.001) return true;
        rs.push_back(r);
        cs.push_back(h(c));
        return false;
    };
    add_sphere(0.5f, v3(-2, 0, 0));
    add_sphere(0.5f, v3(2, 0, 0));
    generate_spheres(0.5f, v3(-2, 0, 0), 0.5f, v3(2, 0, 0), true, add_sphere);
}

SimpleCamera::SimpleCamera(vec3f pos, vec3f dir, vec3f up_hint) : position(pos), direction(dir) {
    const vec3 r = normalize(cross(g(dir), g(up_hint)));
    right = h(r);
    up = h(normalize(cross(r, g(dir))));
}

GridRenderPlane::GridRenderPlane(size_t w, size_t hh) : width(w), height(hh) {
    pixels.resize(w * hh);
    pixel_counters.resize(w * hh);
}

// ---------------------------------------------------------------- scenes
Scene make_scene_box() {
    auto lighting = std::make_shared<CollectionLighting>();
    lighting->addSquareLight(box_light_corner(), vec3f{0.0f, 0.0f, -1.0f}, vec3f{0.0f, 0.2f, 0.0f}, 1.0f);
    return Scene{std::make_shared<GeometrySphereInBox>(), lighting, box_camera()};
}

Scene make_scene_box_lights(int k) {
    if (k <= 0) throw IptError(IPT_E_INVALID, "make_scene_box_lights: k must be positive");
    auto lighting = std::make_shared<CollectionLighting>();
    const vec3f c0 = box_light_corner();
    const float side = 0.2f / (float)k;
    for (int a = 0; a < k; ++a)
        for (int b = 0; b < k; ++b) {
            const vec3f corner{c0.x + (float)b * side, c0.y + (float)a * side, c0.z};
            lighting->addSquareLight(corner, vec3f{0.0f, 0.0f, -1.0f}, vec3f{0.0f, side, 0.0f},
                                     1.0f / (float)(k * k));
        }
    return Scene{std::make_shared<GeometrySphereInBox>(), lighting, box_camera()};
}

Scene make_scene_spheres(int n, uint64_t seed) {
    if (n < 0) throw IptError(IPT_E_INVALID, "make_scene_spheres: n must be >= 0");
    auto geom = std::make_shared<SpheresInBox>();
    SplitMix64 rng{seed};
    geom->spheres.reserve(n);
    for (int i = 0; i < n; ++i) {
        SpheresInBox::Sphere s;
        s.center.x = -0.9f + 1.8f * rng.u();
        s.center.y = -0.9f + 1.8f * rng.u();
        s.center.z = -0.9f + 1.8f * rng.u();
        s.radius = 0.01f + 0.02f * rng.u();
        geom->spheres.push_back(s);
    }
    auto lighting = std::make_shared<CollectionLighting>();
    lighting->addSquareLight(box_light_corner(), vec3f{0.0f, 0.0f, -1.0f}, vec3f{0.0f, 0.2f, 0.0f}, 1.0f);
    return Scene{geom, lighting, box_camera()};
}

Scene make_scene_random_lights(int n, uint64_t seed) {
    auto lighting = std::make_shared<CollectionLighting>();
    SplitMix64 rng{seed};
    for (int i = 0; i < n; ++i) {
        vec3f c, x, y;
        c.x = -0.8f + 1.4f * rng.u();
        c.y = -0.8f + 1.4f * rng.u();
        c.z = -0.8f + 1.4f * rng.u();
        x.x = 0.6f * rng.u() - 0.3f;
        x.y = 0.6f * rng.u() - 0.3f;
        x.z = 0.6f * rng.u() - 0.3f;
        y.x = 0.6f * rng.u() - 0.3f;
        y.y = 0.6f * rng.u() - 0.3f;
        y.z = 0.6f * rng.u() - 0.3f;
        const float power = 0.2f + 0.8f * rng.u();
        lighting->lights.push_back(std::make_shared<const AreaLight>(
            c, x, y, power, i % 3 == 2 ? AreaLight::TYPE_TRIANLE : AreaLight::TYPE_DIAMOND));
    }
    return Scene{std::make_shared<GeometrySphereInBox>(), lighting, box_camera()};
}

Scene make_scene_square_lit_by_square() {
    auto lighting = std::make_shared<CollectionLighting>();
    lighting->addSquareLight(vec3f{-0.05f, -0.05f, -0.9f}, vec3f{0, 0, -1}, vec3f{0, 0.1f, 0});
    const vec3 camera_pos = v3(0, -5.0f, 0);
    const vec3 camera_dir = normalize(v3(0, 0, -1.0f) - camera_pos);
    auto camera = std::make_shared<SimpleCamera>(h(camera_pos), h(camera_dir * 2.0f), vec3f{0, 1, 0});
    return Scene{std::make_shared<GeometryFloor>(), lighting, camera};
}

Scene make_scene_lit_corner() {
    auto lighting = std::make_shared<CollectionLighting>();
    const vec3 out = v3(1, 1, 1);
    const vec3 cx = v3(-0.5f, -1.0f, -1.0f) + 0.5f * out;
    const vec3 cy = v3(-1.0f, -0.5f, -1.0f) + 0.5f * out;
    const vec3 cz = v3(-1.0f, -1.0f, -0.5f) + 0.5f * out;
    lighting->addTriangleLight(h(cx), h(cz - cx), h(cy - cx));
    const vec3 camera_pos = v3(4.0f, 1.0f, 1.0f);
    const vec3 camera_dir = normalize(v3(0, 0, 0.0f) - camera_pos);
    return Scene{std::make_shared<GeometryCorner>(), lighting,
                 std::make_shared<SimpleCamera>(h(camera_pos), h(camera_dir))};
}

Scene make_scene_fractal() {
    auto lighting = std::make_shared<CollectionLighting>();
    lighting->addSphereLight(vec3f{-5.5f, 0, 0}, 1);
    auto camera = std::make_shared<SimpleCamera>(vec3f{0.0f, -4.0f, 0.0f}, vec3f{0, 1, 0});
    return Scene{std::make_shared<FractalSpheres>(), lighting, camera};
}
// GeometrySmallPt.cpp:24-33 (glm::vec3 converts each double to float)
GeometrySmallPt::GeometrySmallPt() {
    spheres = {{1e3, vec3f{(float)(1e3 + 1), 40.8f, 81.6f}},  {1e3, vec3f{(float)(-1e3 + 99), 40.8f, 81.6f}},
               {1e3, vec3f{50, 40.8f, (float)1e3}},          {1e3, vec3f{50, (float)1e3, 81.6f}},
               {1e3, vec3f{50, (float)(-1e3 + 81.6), 81.6f}}, {16.5, vec3f{27, 16.5f, 47}},
               {16.5, vec3f{73, 16.5f, 78}}};
}

Scene make_scene_smallpt() {
    auto lighting = std::make_shared<CollectionLighting>();
    const vec3 lc = v3(50, (float)(81.6 - 16.5), 81.6f);
    lighting->addSquareLight(h(lc - v3(4.0f, 0, 4.0f)), vec3f{0, -1, 0}, vec3f{8.0f, 0, 0});
    const vec3 camera_pos = v3(50.0f, 52.0f, 295.6f);
    const vec3 camera_dir = normalize(v3(0.0f, -0.042612f, -1.0f));
    auto camera = std::make_shared<SimpleCamera>(h(camera_pos), h(camera_dir * 2.0f), vec3f{0, 1, 0});
    return Scene{std::make_shared<GeometrySmallPt>(), lighting, camera};
}

Scene make_scene_by_name(const std::string& spec) {
    std::vector<std::string> f;
    size_t s = 0;
    for (size_t i = 0; i <= spec.size(); ++i)
        if (i == spec.size() || spec[i] == ':') {
            f.push_back(spec.substr(s, i - s));
            s = i + 1;
        }
    auto num = [&](size_t i, long long dflt) { return i < f.size() ? std::stoll(f[i]) : dflt; };
    const std::string& n = f[0];
    if (n == "box") return make_scene_box();
    if (n == "box_lights") return make_scene_box_lights((int)num(1, 16));
    if (n == "spheres") return make_scene_spheres((int)num(1, 10000), (uint64_t)num(2, 1));
    if (n == "random_lights") return make_scene_random_lights((int)num(1, 64), (uint64_t)num(2, 7));
    if (n == "fractal") return make_scene_fractal();
    if (n == "square_lit_by_square" || n == "floor") return make_scene_square_lit_by_square();
    if (n == "lit_corner" || n == "corner") return make_scene_lit_corner();
    if (n == "smallpt") return make_scene_smallpt();
    throw IptError(IPT_E_INVALID, "unknown scene '" + spec + "'");
}

// ---------------------------------------------------------------- flatten
FlatScene flatten(const Scene& s) {
    FlatScene out;
    if (!s.geometry || !s.lighting || !s.camera) throw IptError(IPT_E_INVALID, "scene has a null member");
    if (dynamic_cast<const GeometrySphereInBox*>(s.geometry.get())) {
        out.scene.geometry_kind = IPT_GEOM_SPHERE_IN_BOX;
    } else if (dynamic_cast<const GeometryFloor*>(s.geometry.get())) {
        out.scene.geometry_kind = IPT_GEOM_FLOOR;
    } else if (dynamic_cast<const GeometryCorner*>(s.geometry.get())) {
        out.scene.geometry_kind = IPT_GEOM_CORNER;
    } else if (auto gs = dynamic_cast<const GeometrySmallPt*>(s.geometry.get())) {
        out.scene.geometry_kind = IPT_GEOM_SMALLPT;
        for (const auto& q : gs->spheres) {
            ipt_sphere t{};
            t.center[0] = q.p.x;
            t.center[1] = q.p.y;
            t.center[2] = q.p.z;
            t.radius = (float)q.rad;  // 1e3 and 16.5: exact in float
            out.spheres.push_back(t);
        }
    } else if (auto fs = dynamic_cast<const FractalSpheres*>(s.geometry.get())) {
        out.scene.geometry_kind = IPT_GEOM_SPHERES;
        for (size_t i = 0; i < fs->rs.size(); ++i) {
            ipt_sphere t{};
            t.center[0] = fs->cs[i].x;
            t.center[1] = fs->cs[i].y;
            t.center[2] = fs->cs[i].z;
            t.radius = fs->rs[i];
            out.spheres.push_back(t);
        }
    } else if (auto sp = dynamic_cast<const SpheresInBox*>(s.geometry.get())) {
        out.scene.geometry_kind = IPT_GEOM_SPHERES_IN_BOX;
        for (const auto& q : sp->spheres) {
            ipt_sphere t{};
            t.center[0] = q.center.x;
            t.center[1] = q.center.y;
            t.center[2] = q.center.z;
            t.radius = q.radius;
            out.spheres.push_back(t);
        }
    } else {
        unsupported("geometry type");
    }
    auto coll = dynamic_cast<const CollectionLighting*>(s.lighting.get());
    if (!coll) unsupported("lighting type");
    for (const auto& l : coll->lights) {
        ipt_area_light L{};
        L.power = l->power;
        if (auto sl = dynamic_cast<const SphereLight*>(l.get())) {
            L.position[0] = sl->position.x;
            L.position[1] = sl->position.y;
            L.position[2] = sl->position.z;
            L.x_axis[0] = sl->radius;
            L.type = dynamic_cast<const InvertedSphereLight*>(l.get()) ? IPT_LIGHT_OUTER_SPHERE : IPT_LIGHT_SPHERE;
            out.lights.push_back(L);
            continue;
        }
        if (auto pl = dynamic_cast<const PointLight*>(l.get())) {
            L.position[0] = pl->position.x;
            L.position[1] = pl->position.y;
            L.position[2] = pl->position.z;
            L.x_axis[0] = pl->virtual_radius;
            L.type = IPT_LIGHT_POINT;
            out.lights.push_back(L);
            continue;
        }
        auto a = dynamic_cast<const AreaLight*>(l.get());
        if (!a) unsupported("light type");
        const vec3f* src[3] = {&a->position, &a->x_axis, &a->y_axis};
        float* dst[3] = {L.position, L.x_axis, L.y_axis};
        for (int k = 0; k < 3; ++k) {
            dst[k][0] = src[k]->x;
            dst[k][1] = src[k]->y;
            dst[k][2] = src[k]->z;
        }
        L.power = a->power;
        L.type = a->type == AreaLight::TYPE_TRIANLE ? IPT_LIGHT_AREA_TRIANGLE : IPT_LIGHT_AREA_DIAMOND;
        out.lights.push_back(L);
    }
    auto cam = dynamic_cast<const SimpleCamera*>(s.camera.get());
    if (!cam) unsupported("camera type");
    const vec3f* cs[4] = {&cam->position, &cam->direction, &cam->right, &cam->up};
    float* cd[4] = {out.scene.camera.position, out.scene.camera.direction, out.scene.camera.right,
                    out.scene.camera.up};
    for (int k = 0; k < 4; ++k) {
        cd[k][0] = cs[k]->x;
        cd[k][1] = cs[k]->y;
        cd[k][2] = cs[k]->z;
    }
    out.scene.n_lights = (int)out.lights.size();
    out.scene.lights = out.lights.data();
    out.scene.n_spheres = (int)out.spheres.size();
    out.scene.spheres = out.spheres.empty() ? nullptr : out.spheres.data();
    return out;
}

// ---------------------------------------------------------------- render
GpuRenderer::GpuRenderer(int device) { check(nullptr, ipt_create(device, &ctx_)); }
GpuRenderer::~GpuRenderer() { ipt_destroy(ctx_); }

void GpuRenderer::upload(const Scene& s) {
    FlatScene f = flatten(s);
    check(ctx_, ipt_upload_scene(ctx_, &f.scene));
}

namespace {
ipt_params to_params(size_t W, size_t H, const RenderParams& p) {
    ipt_params q{};
    q.width = (int)W;
    q.height = (int)H;
    q.spp = p.spp;
    q.spp_offset = p.spp_offset;
    q.n_rays = p.n_rays;
    q.depth_max = p.depth_max;
    q.seed = p.seed;
    q.flags = p.counters ? IPT_FLAG_COUNTERS : 0;
    if (p.n_shards > 1) {
        q.tile_rows = p.tile_rows;
        q.n_shards = p.n_shards;
        q.shard_id = p.shard_id;
    }
    return q;
}
// The plane's size_t counters as the library's 32-bit ones, and a zeroed
// per-pixel running max (GridRenderPlane::addRay's max_value, per pixel)
struct PlaneIo {
    std::vector<uint32_t> cnt;
    std::vector<float> pmax;
    PlaneIo(const GridRenderPlane& plane, int spp) : cnt(plane.pixel_counters.size()), pmax(cnt.size(), 0.0f) {
        for (size_t i = 0; i < cnt.size(); ++i) {
            if (plane.pixel_counters[i] > 0xffffffffull - (size_t)std::max(spp, 0))
                throw IptError(IPT_E_INVALID, "pixel counter would overflow 32 bits");
            cnt[i] = (uint32_t)plane.pixel_counters[i];
        }
    }
    ipt_image image(GridRenderPlane& plane) {
        ipt_image img{};
        img.pixels = plane.pixels.data();
        img.counters = cnt.data();
        img.pixel_max = pmax.data();
        return img;
    }
    void finish(GridRenderPlane& plane) const {
        for (size_t i = 0; i < cnt.size(); ++i) plane.pixel_counters[i] = cnt[i];
        for (float m : pmax) plane.max_value = std::max(plane.max_value, m);
    }
};
void check_plane(const GridRenderPlane& plane) {
    const size_t n = plane.width * plane.height;
    if (plane.pixels.size() != n || plane.pixel_counters.size() != n)
        throw IptError(IPT_E_INVALID, "GridRenderPlane buffers do not match width*height");
}
}  // namespace

void GpuRenderer::render_image(ipt_image& img, size_t width, size_t height, const RenderParams& p) {
    ipt_params q = to_params(width, height, p);
    check(ctx_, ipt_render(ctx_, &q, &img));
}

void GpuRenderer::render(GridRenderPlane& plane, const RenderParams& p) {
    check_plane(plane);
    PlaneIo io(plane, p.spp);
    ipt_image img = io.image(plane);
    render_image(img, plane.width, plane.height, p);
    io.finish(plane);
}

void GpuRenderer::transfer_bytes(uint64_t* host_to_device, uint64_t* device_to_host) const {
    check(ctx_, ipt_transfer_bytes(ctx_, host_to_device, device_to_host));
}

ipt_counters GpuRenderer::counters() const {
    ipt_counters c{};
    check(ctx_, ipt_get_counters(ctx_, &c));
    return c;
}

void GpuRenderer::last_kernel_ms(float* path_ms, float* accumulate_ms) const {
    check(ctx_, ipt_last_kernel_ms(ctx_, path_ms, accumulate_ms));
}

void GpuRenderer::smooth(GridRenderPlane& plane, size_t side) {
    float mx = 0.0f;
    check(ctx_, ipt_smooth(ctx_, plane.pixels.data(), (int)plane.width, (int)plane.height, (int)side, 1, &mx));
    plane.max_value = mx;
}

void GpuRenderer::computeSmoothedMax(GridRenderPlane& plane, size_t side) {
    float mx = 0.0f;
    check(ctx_, ipt_smooth(ctx_, plane.pixels.data(), (int)plane.width, (int)plane.height, (int)side, 0, &mx));
    plane.max_value = mx;
}

std::vector<float> GpuRenderer::glare(const GridRenderPlane& plane, float cutoff) {
    std::vector<float> out(plane.pixels.size());
    check(ctx_, ipt_glare(ctx_, plane.pixels.data(), out.data(), (int)plane.width, (int)plane.height, cutoff));
    return out;
}

void render_samples_gpu(const Scene& scene, GridRenderPlane& plane, const RenderParams& p, int device) {
    GpuRenderer r(device);
    r.upload(scene);
    r.render(plane, p);
}

MultiGpuRenderer::MultiGpuRenderer(const std::vector<int>& devices, int tile_rows) : tile_rows_(tile_rows) {
    if (devices.empty()) throw IptError(IPT_E_INVALID, "MultiGpuRenderer: no devices");
    if (tile_rows <= 0) throw IptError(IPT_E_INVALID, "MultiGpuRenderer: tile_rows must be positive");
    for (int d : devices) r_.push_back(std::make_unique<GpuRenderer>(d));
}

void MultiGpuRenderer::upload(const Scene& s) {
    FlatScene f = flatten(s);
    for (auto& r : r_) check(r->handle(), ipt_upload_scene(r->handle(), &f.scene));
}

void MultiGpuRenderer::render(GridRenderPlane& plane, const RenderParams& p) {
    const int n = (int)r_.size();
    if (n == 1) {
        r_[0]->render(plane, p);
        return;
    }
    check_plane(plane);
    // every context renders into the caller's plane itself: ipt_render reads
    // and writes only the context's own rows (its device keeps them between
    // calls), so the shards share the host buffers without copies or merging
    PlaneIo io(plane, p.spp);
    ipt_image img = io.image(plane);
    std::vector<int> code(n, IPT_OK);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    for (int k = 0; k < n; ++k)
        th.emplace_back([&, k] {
            RenderParams q = p;
            q.tile_rows = tile_rows_;
            q.n_shards = n;
            q.shard_id = k;
            try {
                ipt_image im = img;
                r_[k]->render_image(im, plane.width, plane.height, q);
            } catch (const IptError& e) {
                code[k] = e.code;
                msg[k] = e.what();
            } catch (const std::exception& e) {
                code[k] = IPT_E_DEVICE;
                msg[k] = e.what();
            }
        });
    for (auto& t : th) t.join();
    for (int k = 0; k < n; ++k)
        if (code[k] != IPT_OK) throw IptError(code[k], "shard " + std::to_string(k) + ": " + msg[k]);
    io.finish(plane);
}

void MultiGpuRenderer::transfer_bytes(uint64_t* host_to_device, uint64_t* device_to_host) const {
    uint64_t a = 0, b = 0;
    for (const auto& r : r_) {
        uint64_t x = 0, y = 0;
        r->transfer_bytes(&x, &y);
        a += x;
        b += y;
    }
    *host_to_device = a;
    *device_to_host = b;
}

void MultiGpuRenderer::last_kernel_ms(float* path_ms, float* accumulate_ms) const {
    float pm = 0.0f, am = 0.0f;
    for (const auto& r : r_) {
        float a = 0.0f, b = 0.0f;
        r->last_kernel_ms(&a, &b);
        pm = std::max(pm, a);
        am = std::max(am, b);
    }
    *path_ms = pm;
    *accumulate_ms = am;
}

// ---------------------------------------------------------------- output
std::vector<float> tone_map(const GridRenderPlane& plane) {
    // CImg max() of the pixel values; (arg/max).pow(1.0f/inv_gamma).cut(0, 1)
    // with inv_gamma a float 2.2 (gui.cpp:11-16). CImg's pow(double p) on a
    // float image evaluates std::pow(float, float) = powf per pixel.
    float mx = plane.pixels.empty() ? 0.0f : plane.pixels[0];
    for (float v : plane.pixels) mx = std::max(mx, v);
    const float inv_gamma = 2.2f;
    const float p = (float)(double)(1.0f / inv_gamma);
    std::vector<float> out(plane.pixels.size());
    for (size_t i = 0; i < out.size(); ++i) {
        float v = plane.pixels[i] / mx;
        v = std::pow(v, p);
        out[i] = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    }
    return out;
}

std::vector<uint8_t> to_gray8(const GridRenderPlane& plane) {
    std::vector<float> t = tone_map(plane);
    std::vector<uint8_t> out(t.size(), 0);
    if (t.empty()) return out;
    float m = t[0], M = t[0];
    for (float v : t) {
        m = std::min(m, v);
        M = std::max(M, v);
    }
    // CImg normalize(0, 255): constant image -> 0; else (v - m)/(M - m)*(255 - 0) + 0
    if (m != M && (m != 0.0f || M != 255.0f))
        for (float& v : t) v = (v - m) / (M - m) * 255.0f + 0.0f;
    else if (m == M)
        std::fill(t.begin(), t.end(), 0.0f);
    for (size_t i = 0; i < t.size(); ++i) out[i] = (uint8_t)t[i];  // libpng path: (unsigned char) cast
    return out;
}

namespace {
uint32_t crc32_table(int i) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    return c;
}
uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0) {
    static std::array<uint32_t, 256> tab = [] {
        std::array<uint32_t, 256> t{};
        for (int i = 0; i < 256; ++i) t[i] = crc32_table(i);
        return t;
    }();
    c ^= 0xffffffffu;
    for (size_t i = 0; i < n; ++i) c = tab[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return c ^ 0xffffffffu;
}
void put32(std::vector<uint8_t>& b, uint32_t v) {
    b.push_back((uint8_t)(v >> 24));
    b.push_back((uint8_t)(v >> 16));
    b.push_back((uint8_t)(v >> 8));
    b.push_back((uint8_t)v);
}
void chunk(std::ofstream& f, const char* type, const std::vector<uint8_t>& data) {
    std::vector<uint8_t> b;
    put32(b, (uint32_t)data.size());
    b.insert(b.end(), type, type + 4);
    b.insert(b.end(), data.begin(), data.end());
    const uint32_t c = crc32(b.data() + 4, b.size() - 4);
    put32(b, c);
    f.write(reinterpret_cast<const char*>(b.data()), (std::streamsize)b.size());
}
}  // namespace

void write_png_gray8(const std::string& path, size_t w, size_t hgt, const std::vector<uint8_t>& v) {
    if (v.size() != w * hgt) throw IptError(IPT_E_INVALID, "write_png_gray8: size mismatch");
    std::ofstream f(path, std::ios::binary);
    if (!f) throw IptError(IPT_E_INVALID, "cannot open " + path);
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
    f.write(reinterpret_cast<const char*>(sig), 8);
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)w);
    put32(ihdr, (uint32_t)hgt);
    ihdr.insert(ihdr.end(), {8, 0, 0, 0, 0});  // 8-bit gray, deflate, no filter, no interlace
    chunk(f, "IHDR", ihdr);
    // zlib stream of stored (uncompressed) deflate blocks over filter-0 scanlines
    std::vector<uint8_t> raw;
    raw.reserve((w + 1) * hgt);
    for (size_t y = 0; y < hgt; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), v.begin() + (long)(y * w), v.begin() + (long)((y + 1) * w));
    }
    std::vector<uint8_t> z = {0x78, 0x01};
    size_t pos = 0;
    do {
        const size_t len = std::min<size_t>(65535, raw.size() - pos);
        const bool last = pos + len == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)len);
        z.push_back((uint8_t)(len >> 8));
        z.push_back((uint8_t)~len);
        z.push_back((uint8_t)(~len >> 8));
        z.insert(z.end(), raw.begin() + (long)pos, raw.begin() + (long)(pos + len));
        pos += len;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;
    for (uint8_t c : raw) {
        a = (a + c) % 65521u;
        b = (b + a) % 65521u;
    }
    put32(z, (b << 16) | a);
    chunk(f, "IDAT", z);
    chunk(f, "IEND", {});
    if (!f) throw IptError(IPT_E_INVALID, "write failed: " + path);
}

int n_val(float val, float max, float contrast, float gamma) {
    float adj = val * contrast / max;
    adj = std::min(adj, contrast);
    adj = std::max(adj, 1.0f);
    float fn = std::log(adj) / std::log(contrast);  // float overloads, as main.cpp's `using namespace std`
    fn = std::pow(fn, gamma);
    int n = 256 * fn;
    n = std::max(0, n);
    n = std::min(255, n);
    return n;
}

void write_pgm(const std::string& path, const GridRenderPlane& plane, float contrast, float gamma) {
    FILE* fp = std::fopen(path.c_str(), "wb");
    if (!fp) throw IptError(IPT_E_INVALID, "cannot open " + path);
    std::fprintf(fp, "P2\n%lu %lu\n%d\n", (unsigned long)plane.width, (unsigned long)plane.height, 255);
    for (size_t y = 0; y < plane.height; ++y) {
        for (size_t x = 0; x < plane.width; ++x)
            std::fprintf(fp, "%d ", n_val(plane.pixels[y * plane.width + x], plane.max_value, contrast, gamma));
        std::fprintf(fp, "\n");
    }
    std::fclose(fp);
}

void write_pfm(const std::string& path, const GridRenderPlane& plane) {
    std::ofstream f(path, std::ios::binary);
    if (!f) throw IptError(IPT_E_INVALID, "cannot open " + path);
    f << "Pf\n" << plane.width << " " << plane.height << "\n-1.0\n";  // little-endian grayscale
    // PFM stores rows bottom to top; the plane's row 0 is the image top
    for (size_t y = plane.height; y-- > 0;)
        f.write(reinterpret_cast<const char*>(plane.pixels.data() + y * plane.width),
                (std::streamsize)(plane.width * sizeof(float)));
    if (!f) throw IptError(IPT_E_INVALID, "write failed: " + path);
}

}  // namespace ipt
