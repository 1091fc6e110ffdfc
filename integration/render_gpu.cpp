// render_gpu.cpp — the reference-side adapter of INTEGRATION.md §1: what a
// maintainer adds to dimalit/ipt to render sample passes through
// libipt_hip.so instead of calling render_sample (src/main.cpp:186-223) per
// pass. It is compiled against the reference's own headers
// (oracle/build_ref.sh, tests/test_reference_adapter.py), with the one
// change the reference needs: AreaLight keeps x_axis / y_axis / type private
// (src/lighting/lighting.h:20-23), so the maintainer adds, in its public
// section,
//     glm::vec3 xAxis() const { return x_axis; }
//     glm::vec3 yAxis() const { return y_axis; }
//     type_t lightType() const { return type; }
#include "ipt_capi.h"  // include/ipt_capi.h from this repo

#include <CollectionLighting.h>
#include <GridRenderPlane.h>
#include <SimpleCamera.h>
#include <geometry/GeometrySphereInBox.h>
#include <lighting/lighting.h>

#include <algorithm>
#include <memory>
#include <stdexcept>
#include <vector>

// Scene (tracer_interfaces.h:45-49) -> ipt_scene; sample_scenes[0]'s classes
// (GeometrySphereInBox, CollectionLighting of AreaLights, SimpleCamera).
static ipt_scene flatten(const Scene& s, std::vector<ipt_area_light>& lights) {
    ipt_scene out{};
    if (!std::dynamic_pointer_cast<const GeometrySphereInBox>(s.geometry))
        throw std::runtime_error("geometry not supported by libipt_hip");
    out.geometry_kind = IPT_GEOM_SPHERE_IN_BOX;
    auto coll = std::dynamic_pointer_cast<const CollectionLighting>(s.lighting);
    if (!coll) throw std::runtime_error("lighting must be a CollectionLighting");
    for (auto& l : coll->lights) {
        auto a = std::dynamic_pointer_cast<const AreaLight>(l);
        if (!a) throw std::runtime_error("only AreaLight is supported");
        ipt_area_light L{};
        const glm::vec3 x = a->xAxis(), y = a->yAxis();
        for (int k = 0; k < 3; ++k) {
            L.position[k] = a->position[k];
            L.x_axis[k] = x[k];
            L.y_axis[k] = y[k];
        }
        L.power = a->power;
        L.type = a->lightType() == AreaLight::TYPE_TRIANLE ? IPT_LIGHT_AREA_TRIANGLE : IPT_LIGHT_AREA_DIAMOND;
        lights.push_back(L);
    }
    out.n_lights = (int)lights.size();
    out.lights = lights.data();
    auto cam = std::dynamic_pointer_cast<const SimpleCamera>(s.camera);
    if (!cam) throw std::runtime_error("camera must be a SimpleCamera");
    for (int k = 0; k < 3; ++k) {
        out.camera.position[k] = cam->position[k];
        out.camera.direction[k] = cam->direction[k];
        out.camera.right[k] = cam->right[k];
        out.camera.up[k] = cam->up[k];
    }
    return out;
}

// spp passes of render_sample into `plane`, continuing its running means
// (GridRenderPlane::addRay semantics, bit-exact against the CPU restatement)
void render_samples_gpu(const Scene& scene, GridRenderPlane& plane, int spp, int spp_offset, int n_rays,
                        int depth_max, uint64_t seed) {
    static ipt_ctx* ctx = nullptr;
    if (!ctx && ipt_create(0, &ctx) != IPT_OK) throw std::runtime_error(ipt_last_error(nullptr));
    std::vector<ipt_area_light> lights;
    ipt_scene sc = flatten(scene, lights);
    if (ipt_upload_scene(ctx, &sc) != IPT_OK) throw std::runtime_error(ipt_last_error(ctx));
    ipt_params p{};
    p.width = (int)plane.width;
    p.height = (int)plane.height;
    p.spp = spp;
    p.spp_offset = spp_offset;
    p.n_rays = n_rays;
    p.depth_max = depth_max;
    p.seed = seed;
    std::vector<uint32_t> cnt(plane.pixel_counters.begin(), plane.pixel_counters.end());
    std::vector<float> pmax(plane.pixels.size(), 0.0f);
    ipt_image img{plane.pixels.data(), cnt.data(), nullptr, pmax.data()};
    if (ipt_render(ctx, &p, &img) != IPT_OK) throw std::runtime_error(ipt_last_error(ctx));
    std::copy(cnt.begin(), cnt.end(), plane.pixel_counters.begin());
    for (float m : pmax) plane.max_value = std::max(plane.max_value, m);
}
