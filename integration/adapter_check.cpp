// adapter_check.cpp — drives render_gpu.cpp the way the
// reference's main would: the reference's own make_scene_box()
// (sample_scenes.cpp:20-41) and GridRenderPlane (GridRenderPlane.cpp), then
// render_samples_gpu. Writes the plane's pixels (f32) and counters (u32)
// for tests/test_reference_adapter.py; exit 3 with the library's message
// when there is no gfx950 device.
#include <GridRenderPlane.h>
#include <sample_scenes.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>

void render_samples_gpu(const Scene& scene, GridRenderPlane& plane, int spp, int spp_offset, int n_rays,
                        int depth_max, uint64_t seed);

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: adapter_check W H SPP_PER_CALL CALLS OUT_PREFIX\n");
        return 2;
    }
    const int W = std::atoi(argv[1]), H = std::atoi(argv[2]), spp = std::atoi(argv[3]), calls = std::atoi(argv[4]);
    Scene scene = make_scene_box();
    GridRenderPlane plane(W, H);
    try {
        for (int c = 0; c < calls; ++c) render_samples_gpu(scene, plane, spp, c * spp, 16, 8, 20241223);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "adapter_check: %s\n", e.what());
        return 3;
    }
    std::vector<unsigned> cnt(plane.pixel_counters.begin(), plane.pixel_counters.end());
    const std::string pre = argv[5];
    FILE* f = std::fopen((pre + ".f32").c_str(), "wb");
    std::fwrite(plane.pixels.data(), 4, plane.pixels.size(), f);
    std::fclose(f);
    f = std::fopen((pre + ".u32").c_str(), "wb");
    std::fwrite(cnt.data(), 4, cnt.size(), f);
    std::fclose(f);
    std::printf("max_value %.9g\n", plane.max_value);
    return 0;
}
