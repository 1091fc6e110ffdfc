// adapter_check.cpp — drives render_gpu.cpp the way the
// reference's main would: one of the reference's own sample scenes
// (sample_scenes.cpp:20-108) and its GridRenderPlane (GridRenderPlane.cpp),
// then render_samples_gpu once per batch of passes (a progressive loop, the
// scene uploaded once). Writes the plane's pixels (f32) and counters (u32)
// for tests/test_reference_adapter.py; exit 3 with the library's message
// when there is no gfx950 device.
#include <GridRenderPlane.h>
#include <sample_scenes.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

void render_samples_gpu(const Scene& scene, GridRenderPlane& plane, int spp, int spp_offset, int n_rays,
                        int depth_max, uint64_t seed);
int render_gpu_uploads();
uint64_t render_gpu_last_transfer();
void render_gpu_release();
void render_samples_multi_gpu(const Scene& scene, GridRenderPlane& plane, int spp, int spp_offset, int n_rays,
                              int depth_max, uint64_t seed, const std::vector<int>& devices, int tile_rows);

int main(int argc, char** argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: adapter_check SCENE W H SPP_PER_CALL CALLS OUT_PREFIX [N_RAYS DEPTH [DEVICES [TILE]]]\n"
                             "  SCENE: box | fractal | smallpt | square_lit_by_square | lit_corner\n"
                             "  DEVICES: comma-separated HIP devices, one context each (may repeat: 0,0,0)\n");
        return 2;
    }
    const std::string name = argv[1];
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), spp = std::atoi(argv[4]), calls = std::atoi(argv[5]);
    const int n_rays = argc > 7 ? std::atoi(argv[7]) : 16, depth = argc > 8 ? std::atoi(argv[8]) : 8;
    std::vector<int> devices;
    if (argc > 9)
        for (const char* c = argv[9]; *c;) {
            devices.push_back(std::atoi(c));
            while (*c && *c != ',') ++c;
            if (*c == ',') ++c;
        }
    const int tile = argc > 10 ? std::atoi(argv[10]) : 16;
    Scene scene;
    if (name == "box") scene = make_scene_box();
    else if (name == "fractal") scene = make_scene_fractal();
    else if (name == "smallpt") scene = make_scene_smallpt();
    else if (name == "square_lit_by_square") scene = make_scene_square_lit_by_square();
    else if (name == "lit_corner") scene = make_scene_lit_corner();
    else {
        std::fprintf(stderr, "adapter_check: unknown scene %s\n", name.c_str());
        return 2;
    }
    GridRenderPlane plane(W, H);
    try {
        for (int c = 0; c < calls; ++c) {
            if (devices.empty())
                render_samples_gpu(scene, plane, spp, c * spp, n_rays, depth, 20241223);
            else
                render_samples_multi_gpu(scene, plane, spp, c * spp, n_rays, depth, 20241223, devices, tile);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "adapter_check: %s\n", e.what());
        render_gpu_release();
        return 3;
    }
    const int uploads = render_gpu_uploads();
    const unsigned long long transfer = render_gpu_last_transfer();
    render_gpu_release();
    std::vector<unsigned> cnt(plane.pixel_counters.begin(), plane.pixel_counters.end());
    const std::string pre = argv[6];
    FILE* f = std::fopen((pre + ".f32").c_str(), "wb");
    std::fwrite(plane.pixels.data(), 4, plane.pixels.size(), f);
    std::fclose(f);
    f = std::fopen((pre + ".u32").c_str(), "wb");
    std::fwrite(cnt.data(), 4, cnt.size(), f);
    std::fclose(f);
    std::printf("max_value %.9g uploads %d last_call_transfer_bytes %llu\n", plane.max_value, uploads, transfer);
    return 0;
}
