// render_gpu.cpp — the reference-side adapter of INTEGRATION.md §1: what a
// maintainer adds to dimalit/ipt to render sample passes through
// libipt_hip.so instead of calling render_sample (src/main.cpp:186-223) per
// pass. It is compiled against the reference's own headers
// (oracle/build_ref.sh, tests/test_reference_adapter.py), with the accessors
// the reference needs for fields it keeps private, added by the maintainer
// in the public sections:
//   AreaLight (src/lighting/lighting.h:20-23)
//       glm::vec3 xAxis() const { return x_axis; }
//       glm::vec3 yAxis() const { return y_axis; }
//       type_t lightType() const { return type; }
//   FractalSpheres (src/geometry/FractalSpheres.h:13-14)
//       const std::vector<float>& radii() const { return rs; }
//       const std::vector<glm::vec3>& centers() const { return cs; }
// Every sample_scenes entry (src/sample_scenes.cpp:20-108) flattens: the
// geometries GeometrySphereInBox, GeometryFloor, GeometryCorner,
// FractalSpheres and GeometrySmallPt, and CollectionLighting's AreaLight
// (square and triangle), SphereLight, PointLight and InvertedSphereLight
// (addOuterLight). Anything else throws.
#include "ipt_capi.h"  // include/ipt_capi.h from this repo

#include <CollectionLighting.h>
#include <GridRenderPlane.h>
#include <SimpleCamera.h>
#include <geometry/FractalSpheres.h>
#include <geometry/GeometryCorner.h>
#include <geometry/GeometryFloor.h>
#include <geometry/GeometrySmallPt.h>
#include <geometry/GeometrySphereInBox.h>
#include <lighting/lighting.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

// The flattened scene and the arrays it points into.
struct Flat {
    ipt_scene sc{};
    std::vector<ipt_area_light> lights;
    std::vector<ipt_sphere> spheres;
    bool operator==(const Flat& o) const {
        auto same = [](const void* a, const void* b, size_t n) { return n == 0 || std::memcmp(a, b, n) == 0; };
        return sc.geometry_kind == o.sc.geometry_kind && lights.size() == o.lights.size() &&
               spheres.size() == o.spheres.size() &&
               same(&sc.camera, &o.sc.camera, sizeof(ipt_camera)) &&
               same(lights.data(), o.lights.data(), lights.size() * sizeof(ipt_area_light)) &&
               same(spheres.data(), o.spheres.data(), spheres.size() * sizeof(ipt_sphere));
    }
};

void put3(float* d, const glm::vec3& v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
}

// GeometrySmallPt's room: the `spheres[]` table is local to its translation
// unit (src/geometry/GeometrySmallPt.cpp:23-32), so the adapter restates its
// radii and positions (the vec3 constructor's float roundings); the library
// intersects them in double as Sphere::intersect does.
void smallpt_spheres(std::vector<ipt_sphere>& out) {
    const struct {
        double rad;
        glm::vec3 p;
    } room[] = {{1e3, glm::vec3(1e3 + 1, 40.8, 81.6)},  {1e3, glm::vec3(-1e3 + 99, 40.8, 81.6)},
                {1e3, glm::vec3(50, 40.8, 1e3)},         {1e3, glm::vec3(50, 1e3, 81.6)},
                {1e3, glm::vec3(50, -1e3 + 81.6, 81.6)}, {16.5, glm::vec3(27, 16.5, 47)},
                {16.5, glm::vec3(73, 16.5, 78)}};
    for (const auto& s : room) {
        ipt_sphere q{};
        put3(q.center, s.p);
        q.radius = (float)s.rad;  // 1e3 and 16.5 are exact in float
        out.push_back(q);
    }
}

// Scene (tracer_interfaces.h:45-49) -> ipt_scene
void flatten(const Scene& s, Flat& f) {
    f = Flat{};
    if (std::dynamic_pointer_cast<const GeometrySphereInBox>(s.geometry)) {
        f.sc.geometry_kind = IPT_GEOM_SPHERE_IN_BOX;
    } else if (std::dynamic_pointer_cast<const GeometryFloor>(s.geometry)) {
        f.sc.geometry_kind = IPT_GEOM_FLOOR;
    } else if (std::dynamic_pointer_cast<const GeometryCorner>(s.geometry)) {
        f.sc.geometry_kind = IPT_GEOM_CORNER;
    } else if (auto fr = std::dynamic_pointer_cast<const FractalSpheres>(s.geometry)) {
        f.sc.geometry_kind = IPT_GEOM_SPHERES;
        const auto& rs = fr->radii();
        const auto& cs = fr->centers();
        for (size_t i = 0; i < rs.size(); ++i) {
            ipt_sphere q{};
            put3(q.center, cs[i]);
            q.radius = rs[i];
            f.spheres.push_back(q);
        }
    } else if (std::dynamic_pointer_cast<const GeometrySmallPt>(s.geometry)) {
        f.sc.geometry_kind = IPT_GEOM_SMALLPT;
        smallpt_spheres(f.spheres);
    } else {
        throw std::runtime_error("geometry not supported by libipt_hip");
    }
    auto coll = std::dynamic_pointer_cast<const CollectionLighting>(s.lighting);
    if (!coll) throw std::runtime_error("lighting must be a CollectionLighting");
    for (auto& l : coll->lights) {
        ipt_area_light L{};
        L.power = l->power;
        put3(L.position, l->position);
        if (auto a = std::dynamic_pointer_cast<const AreaLight>(l)) {
            put3(L.x_axis, a->xAxis());
            put3(L.y_axis, a->yAxis());
            L.type = a->lightType() == AreaLight::TYPE_TRIANLE ? IPT_LIGHT_AREA_TRIANGLE : IPT_LIGHT_AREA_DIAMOND;
        } else if (auto o = std::dynamic_pointer_cast<const InvertedSphereLight>(l)) {  // before SphereLight
            L.x_axis[0] = o->radius;
            L.type = IPT_LIGHT_OUTER_SPHERE;
        } else if (auto sl = std::dynamic_pointer_cast<const SphereLight>(l)) {
            L.x_axis[0] = sl->radius;
            L.type = IPT_LIGHT_SPHERE;
        } else if (std::dynamic_pointer_cast<const PointLight>(l)) {
            L.type = IPT_LIGHT_POINT;  // its virtual radius is not stored (lighting.h:31-42)
        } else {
            throw std::runtime_error("light type not supported by libipt_hip");
        }
        f.lights.push_back(L);
    }
    auto cam = std::dynamic_pointer_cast<const SimpleCamera>(s.camera);
    if (!cam) throw std::runtime_error("camera must be a SimpleCamera");
    put3(f.sc.camera.position, cam->position);
    put3(f.sc.camera.direction, cam->direction);
    put3(f.sc.camera.right, cam->right);
    put3(f.sc.camera.up, cam->up);
    f.sc.n_lights = (int)f.lights.size();
    f.sc.lights = f.lights.data();
    f.sc.n_spheres = (int)f.spheres.size();
    f.sc.spheres = f.spheres.empty() ? nullptr : f.spheres.data();
}

}  // namespace

// One context on one device; the scene is uploaded again only when its
// flattened content changes (a progressive loop renders one scene many times).
class GpuRenderer {
public:
    explicit GpuRenderer(int device = 0) {
        if (ipt_create(device, &ctx_) != IPT_OK) throw std::runtime_error(ipt_last_error(nullptr));
    }
    ~GpuRenderer() { ipt_destroy(ctx_); }
    GpuRenderer(const GpuRenderer&) = delete;
    GpuRenderer& operator=(const GpuRenderer&) = delete;

    // spp passes of render_sample into the C-ABI image `img` (the plane's
    // pixels, 32-bit counters, per-pixel running max), continuing its running
    // means (GridRenderPlane::addRay semantics, bit-exact against the CPU
    // restatement); with n_shards > 1 only the destination rows of tile shard
    // `shard_id` (tile_rows-row tiles dealt round-robin, ipt_shard_plan) are
    // rendered, read and written. The context keeps its rows on its device
    // between calls (ipt_render), so a call moves only those rows.
    void render_image(const Scene& scene, ipt_image& img, int width, int height, int spp, int spp_offset,
                      int n_rays, int depth_max, uint64_t seed, int n_shards = 1, int shard_id = 0,
                      int tile_rows = 16) {
        Flat f;
        flatten(scene, f);
        if (!has_scene_ || !(f == last_)) {
            has_scene_ = false;
            if (ipt_upload_scene(ctx_, &f.sc) != IPT_OK) throw std::runtime_error(ipt_last_error(ctx_));
            last_ = std::move(f);
            last_.sc.lights = last_.lights.data();
            last_.sc.spheres = last_.spheres.empty() ? nullptr : last_.spheres.data();
            has_scene_ = true;
            ++uploads_;
        }
        ipt_params p{};
        p.width = width;
        p.height = height;
        p.spp = spp;
        p.spp_offset = spp_offset;
        p.n_rays = n_rays;
        p.depth_max = depth_max;
        p.seed = seed;
        if (n_shards > 1) {
            p.tile_rows = tile_rows;
            p.n_shards = n_shards;
            p.shard_id = shard_id;
        }
        if (ipt_render(ctx_, &p, &img) != IPT_OK) throw std::runtime_error(ipt_last_error(ctx_));
    }
    uint64_t transferred() const {  // host <-> device bytes of the last call
        uint64_t a = 0, b = 0;
        if (ipt_transfer_bytes(ctx_, &a, &b) != IPT_OK) throw std::runtime_error(ipt_last_error(ctx_));
        return a + b;
    }
    int uploads() const { return uploads_; }

private:
    ipt_ctx* ctx_ = nullptr;
    Flat last_;
    bool has_scene_ = false;
    int uploads_ = 0;
};

// GridRenderPlane (size_t counters, GridRenderPlane.h) <-> the C-ABI image:
// 32-bit counters and a zeroed per-pixel running max for this call
struct PlaneIo {
    std::vector<uint32_t> cnt;
    std::vector<float> pmax;
    explicit PlaneIo(const GridRenderPlane& plane)
        : cnt(plane.pixel_counters.begin(), plane.pixel_counters.end()), pmax(plane.pixels.size(), 0.0f) {}
    ipt_image image(GridRenderPlane& plane) { return ipt_image{plane.pixels.data(), cnt.data(), nullptr, pmax.data()}; }
    void finish(GridRenderPlane& plane) const {
        std::copy(cnt.begin(), cnt.end(), plane.pixel_counters.begin());
        for (float m : pmax) plane.max_value = std::max(plane.max_value, m);
    }
};

// The free-function form of INTEGRATION.md §1 on process-wide renderers, one
// per device, released by render_gpu_release() (call it before exit: the HIP
// runtime may be torn down before static destructors run).
static std::vector<std::pair<int, std::unique_ptr<GpuRenderer>>> g_single;
static uint64_t g_last_transfer = 0;

static GpuRenderer& single_renderer(int device) {
    for (auto& e : g_single)
        if (e.first == device) return *e.second;
    g_single.emplace_back(device, std::make_unique<GpuRenderer>(device));
    return *g_single.back().second;
}

static void render_on(int device, const Scene& scene, GridRenderPlane& plane, int spp, int spp_offset, int n_rays,
                      int depth_max, uint64_t seed) {
    GpuRenderer& r = single_renderer(device);
    PlaneIo io(plane);
    ipt_image img = io.image(plane);
    r.render_image(scene, img, (int)plane.width, (int)plane.height, spp, spp_offset, n_rays, depth_max, seed);
    io.finish(plane);
    g_last_transfer = r.transferred();
}

void render_samples_gpu(const Scene& scene, GridRenderPlane& plane, int spp, int spp_offset, int n_rays,
                        int depth_max, uint64_t seed) {
    render_on(0, scene, plane, spp, spp_offset, n_rays, depth_max, seed);
}


// The N-device form (the reference renders with several threads into one
// plane, src/main.cpp:256-285): one context per entry of `devices` (a device
// may repeat), destination rows cut into `tile_rows`-row tiles dealt
// round-robin to the contexts (ipt_params.n_shards / shard_id), each context
// driven by its own host thread straight into the caller's plane: ipt_render
// reads and writes only the context's own rows, which its device keeps
// between calls, so every pixel has exactly one owner and nothing is merged.
// Each shard traces only the samples that can land in its rows, with the same
// (seed, pass, pixel) streams, so the plane is bit-identical to the
// one-device render.
static std::vector<std::unique_ptr<GpuRenderer>> g_multi;
static std::vector<int> g_multi_devices;

void render_samples_multi_gpu(const Scene& scene, GridRenderPlane& plane, int spp, int spp_offset, int n_rays,
                              int depth_max, uint64_t seed, const std::vector<int>& devices, int tile_rows) {
    const int n = (int)devices.size();
    if (n == 0) throw std::runtime_error("render_samples_multi_gpu: no devices");
    if (n == 1) {  // the listed device, not device 0
        render_on(devices[0], scene, plane, spp, spp_offset, n_rays, depth_max, seed);
        return;
    }
    if (g_multi_devices != devices) {
        g_multi.clear();
        for (int d : devices) g_multi.push_back(std::make_unique<GpuRenderer>(d));
        g_multi_devices = devices;
    }
    PlaneIo io(plane);
    const ipt_image img = io.image(plane);
    std::vector<std::string> err(n);
    std::vector<std::thread> th;
    for (int k = 0; k < n; ++k)
        th.emplace_back([&, k] {
            try {
                ipt_image im = img;
                g_multi[k]->render_image(scene, im, (int)plane.width, (int)plane.height, spp, spp_offset, n_rays,
                                         depth_max, seed, n, k, tile_rows);
            } catch (const std::exception& e) {
                err[k] = e.what();
            }
        });
    for (auto& t : th) t.join();
    for (int k = 0; k < n; ++k)
        if (!err[k].empty()) throw std::runtime_error(err[k]);
    io.finish(plane);
    g_last_transfer = 0;
    for (const auto& r : g_multi) g_last_transfer += r->transferred();
}

// host <-> device bytes of the last render call (all its contexts)
uint64_t render_gpu_last_transfer() { return g_last_transfer; }

// scene uploads of the most-uploaded context (1 when an unchanged scene is
// rendered progressively)
int render_gpu_uploads() {
    int u = 0;
    for (const auto& e : g_single) u = std::max(u, e.second->uploads());
    for (const auto& r : g_multi) u = std::max(u, r->uploads());
    return u;
}

void render_gpu_release() {
    g_single.clear();
    g_multi.clear();
    g_multi_devices.clear();
}
