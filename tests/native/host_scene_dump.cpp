// Test helper (tests/test_host_cpp.py): exercises the C++ host layer without a
// GPU. "scene NAME" prints the flattened ipt_scene as JSON (floats as bit
// patterns); "gray8 W H in.f32 out.png" writes the Gui-normalised PNG of a raw
// float plane; "scene-error NAME" prints the IptError code.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <vector>

#include "ipt_host.h"

static unsigned bits(float f) {
    unsigned u;
    std::memcpy(&u, &f, 4);
    return u;
}
static void vec(const float* v) { std::printf("[%u, %u, %u]", bits(v[0]), bits(v[1]), bits(v[2])); }

int main(int argc, char** argv) {
    if (argc >= 3 && std::strcmp(argv[1], "scene") == 0) {
        ipt::FlatScene f = ipt::flatten(ipt::make_scene_by_name(argv[2]));
        std::printf("{\"geometry_kind\": %d, \"camera\": [", f.scene.geometry_kind);
        vec(f.scene.camera.position); std::printf(", ");
        vec(f.scene.camera.direction); std::printf(", ");
        vec(f.scene.camera.right); std::printf(", ");
        vec(f.scene.camera.up);
        std::printf("], \"lights\": [");
        for (size_t i = 0; i < f.lights.size(); ++i) {
            const ipt_area_light& L = f.lights[i];
            std::printf("%s[", i ? ", " : "");
            vec(L.position); std::printf(", ");
            vec(L.x_axis); std::printf(", ");
            vec(L.y_axis);
            std::printf(", %u, %d]", bits(L.power), L.type);
        }
        std::printf("], \"spheres\": [");
        for (size_t i = 0; i < f.spheres.size(); ++i) {
            std::printf("%s[", i ? ", " : "");
            vec(f.spheres[i].center);
            std::printf(", %u]", bits(f.spheres[i].radius));
        }
        std::printf("]}\n");
        return 0;
    }
    if (argc >= 3 && std::strcmp(argv[1], "scene-error") == 0) {
        try {
            ipt::flatten(ipt::make_scene_by_name(argv[2]));
            std::printf("0\n");
        } catch (const ipt::IptError& e) {
            std::printf("%d\n", e.code);
        }
        return 0;
    }
    if (argc >= 6 && std::strcmp(argv[1], "gray8") == 0) {
        const size_t w = std::strtoul(argv[2], nullptr, 10), h = std::strtoul(argv[3], nullptr, 10);
        ipt::GridRenderPlane plane(w, h);
        std::ifstream in(argv[4], std::ios::binary);
        in.read(reinterpret_cast<char*>(plane.pixels.data()), (std::streamsize)(w * h * 4));
        ipt::write_png_gray8(argv[5], w, h, ipt::to_gray8(plane));
        return 0;
    }
    if (argc >= 7 && std::strcmp(argv[1], "pgm") == 0) {
        const size_t w = std::strtoul(argv[2], nullptr, 10), h = std::strtoul(argv[3], nullptr, 10);
        ipt::GridRenderPlane plane(w, h);
        std::ifstream in(argv[4], std::ios::binary);
        in.read(reinterpret_cast<char*>(plane.pixels.data()), (std::streamsize)(w * h * 4));
        plane.max_value = std::strtof(argv[5], nullptr);
        ipt::write_pgm(argv[6], plane);
        return 0;
    }
    std::fprintf(stderr, "usage: host_scene_dump scene NAME | scene-error NAME | gray8 W H in.f32 out.png | "
                         "pgm W H in.f32 MAX out.pgm\n");
    return 2;
}
