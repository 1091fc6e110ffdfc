// ipt_host.h — the C++ host side above the C-ABI (include/ipt_capi.h).
//
// It mirrors the reference's host surface for the hot path, with the same
// names, argument meanings and defaults, so that scene setup and output code
// written against the reference reads the same here:
//   Scene / Geometry / Lighting / Camera / RenderPlane  (tracer_interfaces.h:26-54)
//   GeometrySphereInBox                                 (geometry/GeometrySphereInBox.h)
//   CollectionLighting::addSquareLight/addTriangleLight (CollectionLighting.h:11-20)
//   AreaLight                                           (lighting/lighting.h:15-29)
//   SimpleCamera(position, direction, up_hint=(0,0,1))  (SimpleCamera.h:9-17)
//   GridRenderPlane{pixels, pixel_counters, width, height, max_value}
//                                                       (GridRenderPlane.h:8-18)
//   make_scene_box()                                    (sample_scenes.cpp:20-41)
// plus the synthetic BASELINE scenes (C3 sphere list, C5 light grid).
//
// Objects here are scene DESCRIPTIONS: nothing in this layer traces a ray on
// the CPU. Rendering is GpuRenderer / render_samples_gpu, i.e. ipt_render on
// a gfx950 GPU, and it throws IptError(IPT_E_DEVICE) when there is none.
// Every sample_scenes entry and light type of the reference is supported;
// geometry or light classes outside them throw IptError(IPT_E_UNSUPPORTED)
// when flattened.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ipt_capi.h"

namespace ipt {

// glm::vec3 stand-in: plain float data; arithmetic goes through ipt_math.h so
// that constructor arithmetic matches the reference's glm order bit for bit.
struct vec3f {
    float x = 0.0f, y = 0.0f, z = 0.0f;
};

struct IptError : std::runtime_error {
    int code;
    IptError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ------------------------------------------------------------- geometry
struct Geometry {
    virtual ~Geometry() = default;
};
// Box walls {+x,+y,+z,-x,-z} and the r=0.5 sphere at the origin.
struct GeometrySphereInBox : Geometry {};
// The same box walls plus a list of spheres with FractalSpheres::traceRay's
// acceptance rule (FractalSpheres.cpp:75-84): BASELINE configs[2].
struct SpheresInBox : Geometry {
    struct Sphere {
        vec3f center;
        float radius;
    };
    std::vector<Sphere> spheres;
};

// The z = -1 face (GeometryFloor.cpp:10-23), unrotated CosineDdf.
struct GeometryFloor : Geometry {};
// The x = -1, y = -1, z = -1 faces (GeometryCorner.cpp:10-42).
struct GeometryCorner : Geometry {};
// FractalSpheres (FractalSpheres.cpp:46-97): the generated sphere chain
// between two r=0.5 spheres at (-2,0,0) and (2,0,0), no walls.
// GeometrySmallPt (GeometrySmallPt.cpp:11-58): smallpt's room of 7 spheres,
// intersected in double precision.
struct GeometrySmallPt : Geometry {
    struct Sphere {
        double rad;
        vec3f p;
    };
    std::vector<Sphere> spheres;
    GeometrySmallPt();
};
struct FractalSpheres : Geometry {
    std::vector<float> rs;
    std::vector<vec3f> cs;
    FractalSpheres();
};

// ------------------------------------------------------------- lighting
struct Light {
    float power = 1.0f;
    virtual ~Light() = default;
};
// Light(corner, x_axis, y_axis, power, type) (lighting.cpp:79-90).
struct AreaLight : Light {
    enum type_t { TYPE_DIAMOND = 0, TYPE_TRIANLE = 1 };  // the reference's spelling (lighting.h:17)
    vec3f position, x_axis, y_axis;
    type_t type = TYPE_DIAMOND;
    AreaLight(vec3f corner, vec3f x_axis, vec3f y_axis, float power, type_t type = TYPE_DIAMOND);
};

// SphereLight(origin, radius, power=1) (lighting.h:44-54)
struct SphereLight : Light {
    vec3f position;
    float radius;
    SphereLight(vec3f origin, float radius, float power = 1.0f);
};
// PointLight(origin, virtual_radius, power=1) (lighting.h:31-42)
struct PointLight : Light {
    vec3f position;
    float virtual_radius;
    PointLight(vec3f origin, float virtual_radius, float power = 1.0f);
};
// InvertedSphereLight(origin, radius, power) (lighting.h:57-72)
struct InvertedSphereLight : SphereLight {
    InvertedSphereLight(vec3f origin, float radius, float power);
};

struct Lighting {
    virtual ~Lighting() = default;
};
struct CollectionLighting : Lighting {
    std::vector<std::shared_ptr<const Light>> lights;
    // y_side = cross(normal, x_side) (CollectionLighting.cpp:42-46)
    void addSquareLight(vec3f corner, vec3f normal, vec3f x_side, float power = 1.0f);
    void addTriangleLight(vec3f corner, vec3f x_side, vec3f y_side, float power = 1.0f);
    void addPointLight(vec3f position, float virtual_radius, float power = 1.0f);
    void addSphereLight(vec3f position, float radius, float power = 1.0f);
    void addOuterLight(float radius, float power = 1.0f);  // InvertedSphereLight at the origin
};

// --------------------------------------------------------------- camera
struct Camera {
    virtual ~Camera() = default;
};
struct SimpleCamera : Camera {
    vec3f position, direction, right, up;
    // right = normalize(cross(direction, up_hint)); up = normalize(cross(right, direction))
    SimpleCamera(vec3f position, vec3f direction, vec3f up_hint = vec3f{0.0f, 0.0f, 1.0f});
};

struct Scene {
    std::shared_ptr<const Geometry> geometry;
    std::shared_ptr<const Lighting> lighting;
    std::shared_ptr<const Camera> camera;
};

// ---------------------------------------------------------------- plane
struct RenderPlane {
    virtual ~RenderPlane() = default;
};
// Running mean per pixel as GridRenderPlane::addRay keeps it (including its
// row mapping, GridRenderPlane.cpp:61-75); filled by the GPU accumulate kernel.
struct GridRenderPlane : RenderPlane {
    std::vector<float> pixels;
    std::vector<size_t> pixel_counters;
    size_t width, height;
    float max_value = 0;
    GridRenderPlane(size_t width, size_t height);
};

// --------------------------------------------------------- sample scenes
Scene make_scene_box();                                   // sample_scenes[0]
Scene make_scene_box_lights(int k);                       // [0]'s light as k*k squares (C5: k=16)
Scene make_scene_spheres(int n, uint64_t seed = 1);       // box + n spheres (C3: n=10000)
Scene make_scene_random_lights(int n, uint64_t seed = 7);  // overlapping random emitters (tests)
Scene make_scene_square_lit_by_square();                  // sample_scenes.cpp:73-85
Scene make_scene_lit_corner();                            // sample_scenes.cpp:88-108
Scene make_scene_fractal();                               // sample_scenes.cpp:43-55
Scene make_scene_smallpt();                               // sample_scenes.cpp:57-71
// "box", "box_lights:K", "spheres:N[:SEED]", "random_lights:N[:SEED]", "fractal", ...
Scene make_scene_by_name(const std::string& name);

// --------------------------------------------------------------- render
struct RenderParams {
    int spp = 1;          // sample passes (render_sample calls) in this call
    int spp_offset = 0;   // index of the first pass (RNG stream), for progressive rendering
    int n_rays = 16;      // main.cpp:53 ray_power(..., n_rays)
    int depth_max = 8;    // main.cpp:94
    uint64_t seed = 20241223;
    bool counters = false;
    // destination-row tile shard of this call (ipt_params.tile_rows / n_shards /
    // shard_id): n_shards <= 1 renders the whole frame
    int tile_rows = 16;
    int n_shards = 1;
    int shard_id = 0;
};

// Scene -> POD (ipt_scene). Owns the arrays the POD points into.
struct FlatScene {
    ipt_scene scene{};
    std::vector<ipt_area_light> lights;
    std::vector<ipt_sphere> spheres;
};
FlatScene flatten(const Scene& s);  // throws IptError(IPT_E_UNSUPPORTED)

class GpuRenderer {
   public:
    explicit GpuRenderer(int device = 0);
    ~GpuRenderer();
    GpuRenderer(const GpuRenderer&) = delete;
    GpuRenderer& operator=(const GpuRenderer&) = delete;
    void upload(const Scene& s);
    // spp passes of render_sample accumulated into plane (bit-exact GridRenderPlane semantics)
    void render(GridRenderPlane& plane, const RenderParams& p);
    // the same into a C-ABI image (32-bit counters); with p.n_shards > 1 only
    // the shard's rows of it are read and written (ipt_render)
    void render_image(ipt_image& img, size_t width, size_t height, const RenderParams& p);
    // host <-> device bytes of the last render (ipt_transfer_bytes): the
    // context keeps its rows of the plane on its device between calls
    void transfer_bytes(uint64_t* host_to_device, uint64_t* device_to_host) const;
    ipt_counters counters() const;
    void last_kernel_ms(float* path_ms, float* accumulate_ms) const;
    // GridRenderPlane::smooth / computeSmoothedMax (GridRenderPlane.cpp:10-59) on the GPU
    void smooth(GridRenderPlane& plane, size_t side);
    void computeSmoothedMax(GridRenderPlane& plane, size_t side);
    // Gui's glare bloom (gui.cpp:28-52) of the plane's pixels
    std::vector<float> glare(const GridRenderPlane& plane, float cutoff);
    ipt_ctx* handle() const { return ctx_; }

   private:
    ipt_ctx* ctx_ = nullptr;
};

// One-shot convenience (the INTEGRATION.md adapter's shape).
void render_samples_gpu(const Scene& scene, GridRenderPlane& plane, const RenderParams& p, int device = 0);

// N contexts (one per entry of `devices`; a device may repeat), i.e. the
// node's GPUs in one process. The reference renders with several worker
// threads into one plane (main.cpp:256-285); here the destination rows are cut
// into tile_rows-row tiles dealt round-robin to the contexts (ipt_shard_plan),
// each context is driven by its own host thread and renders into the caller's
// plane directly: its device keeps the context's own rows between calls, a call
// moves only those rows (16 B per owned pixel, ipt_render) and no other row is
// touched (one owner per pixel, so nothing is summed or merged). Each shard traces
// only the samples that can land in its rows, with the same (seed, pass, pixel)
// streams: the plane is bit-identical to GpuRenderer::render's.
class MultiGpuRenderer {
   public:
    explicit MultiGpuRenderer(const std::vector<int>& devices, int tile_rows = 16);
    void upload(const Scene& s);
    void render(GridRenderPlane& plane, const RenderParams& p);
    // host <-> device bytes of the last render, summed over the contexts
    void transfer_bytes(uint64_t* host_to_device, uint64_t* device_to_host) const;
    size_t size() const { return r_.size(); }
    GpuRenderer& context(size_t k) { return *r_[k]; }
    // the slowest context's kernel time of the last render (path, accumulate ms)
    void last_kernel_ms(float* path_ms, float* accumulate_ms) const;

   private:
    std::vector<std::unique_ptr<GpuRenderer>> r_;
    int tile_rows_;
};

// --------------------------------------------------------------- output
// Gui's display normalisation (gui.cpp:11-16): (v / max)^(1/2.2), cut to [0, 1].
std::vector<float> tone_map(const GridRenderPlane& plane);
// Gui::save (gui.cpp:133-135): tone map, CImg normalize(0, 255) (CImg.h
// normalize(a,b): (v - min)/(max - min)*255), then the 8-bit PNG writer's
// (unsigned char) cast. Written as a grayscale 8-bit PNG.
std::vector<uint8_t> to_gray8(const GridRenderPlane& plane);
void write_png_gray8(const std::string& path, size_t width, size_t height, const std::vector<uint8_t>& v);
// Raw outputs: PFM (float pixels, bottom-to-top rows per the format) and a
// little binary dump of counters.
void write_pfm(const std::string& path, const GridRenderPlane& plane);
// main.cpp's PGM writer (main.cpp:225-235 n_val, 297-309): ASCII P2, each pixel
// mapped by log(clamp(v*contrast/max, 1, contrast))/log(contrast), ^gamma, *256.
int n_val(float val, float max, float contrast, float gamma);
void write_pgm(const std::string& path, const GridRenderPlane& plane, float contrast = 500.0f, float gamma = 0.6f);

}  // namespace ipt
