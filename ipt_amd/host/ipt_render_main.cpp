// ipt_render — headless C++ front end of the GPU path (the reference's main.cpp
// render loop, main.cpp:237-312, without the X11 Gui): builds a sample scene,
// renders `passes` batches of `spp` render_sample passes into a
// GridRenderPlane on one MI355X through GpuRenderer (C-ABI), and writes the
// Gui-normalised 8-bit PNG (Gui::save, gui.cpp:133-135) plus optional raw
// float pixels (PFM) and counters.
//
//   ipt_render [--scene box|box_lights:K|spheres:N[:SEED]|random_lights:N[:SEED]]
//              [--width 640] [--height 640] [--spp 16] [--passes 1]
//              [--n-rays 16] [--depth 8] [--seed 20241223] [--device 0]
//              [--devices 0,1,...,7 [--tile-rows 16]]
//              [--out result.png] [--pfm pixels.pfm] [--counts counts.u32]
//              [--pgm result.pgm] [--smooth SIDE] [--glare CUTOFF --glare-out glare.pfm]
//
// --smooth applies GridRenderPlane::smooth(SIDE) on the GPU before output;
// --glare writes Gui's glare bloom of the plane (gui.cpp:28-52, GPU) as PFM;
// --pgm writes main.cpp's contrast/gamma PGM (main.cpp:297-309).
// --devices renders with one context per listed device (MultiGpuRenderer: the
// rows cut into --tile-rows tiles dealt round-robin, owned rows assembled at
// the end of each batch; a device may repeat); the image is the same bits.
//
// Prints one JSON line: scene, size, passes, Mpaths/s (whole call and kernel).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "ipt_host.h"

namespace {
[[noreturn]] void usage(const char* msg) {
    std::fprintf(stderr, "ipt_render: %s\n", msg);
    std::fprintf(stderr,
                 "usage: ipt_render [--scene NAME] [--width W] [--height H] [--spp S] [--passes P]\n"
                 "                  [--n-rays N] [--depth D] [--seed X] [--device I]\n"
                 "                  [--devices I,J,... [--tile-rows 16]]\n"
                 "                  [--out result.png] [--pfm pixels.pfm] [--counts counts.u32]\n"
                 "                  [--pgm result.pgm] [--smooth SIDE] [--glare CUTOFF --glare-out F.pfm]\n");
    std::exit(2);
}
}  // namespace

int main(int argc, char** argv) {
    std::string scene_name = "box", out = "result.png", pfm, counts, pgm, glare_out;
    long smooth = 0;
    double glare = -1.0;
    long width = 640, height = 640, spp = 16, passes = 1, n_rays = 16, depth = 8, device = 0, tile_rows = 16;
    std::vector<int> devices;
    unsigned long long seed = 20241223ull;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) usage(("missing value for " + a).c_str());
            return argv[++i];
        };
        if (a == "--scene") scene_name = val();
        else if (a == "--width") width = std::atol(val());
        else if (a == "--height") height = std::atol(val());
        else if (a == "--spp") spp = std::atol(val());
        else if (a == "--passes") passes = std::atol(val());
        else if (a == "--n-rays") n_rays = std::atol(val());
        else if (a == "--depth") depth = std::atol(val());
        else if (a == "--seed") seed = std::strtoull(val(), nullptr, 0);
        else if (a == "--device") device = std::atol(val());
        else if (a == "--devices") {
            devices.clear();
            for (const char* c = val(); *c;) {
                devices.push_back(std::atoi(c));
                while (*c && *c != ',') ++c;
                if (*c == ',') ++c;
            }
        } else if (a == "--tile-rows") tile_rows = std::atol(val());
        else if (a == "--out") out = val();
        else if (a == "--pfm") pfm = val();
        else if (a == "--counts") counts = val();
        else if (a == "--pgm") pgm = val();
        else if (a == "--smooth") smooth = std::atol(val());
        else if (a == "--glare") glare = std::atof(val());
        else if (a == "--glare-out") glare_out = val();
        else usage(("unknown option " + a).c_str());
    }
    if (width <= 0 || height <= 0 || spp <= 0 || passes <= 0 || n_rays < 0 || depth < 0) usage("bad sizes");
    try {
        const ipt::Scene scene = ipt::make_scene_by_name(scene_name);
        if (devices.empty()) devices.push_back((int)device);
        if (tile_rows <= 0) usage("bad --tile-rows");
        ipt::MultiGpuRenderer gpus(devices, (int)tile_rows);
        ipt::GpuRenderer& gpu = gpus.context(0);  // post-process runs on the first context
        gpus.upload(scene);
        ipt::GridRenderPlane plane((size_t)width, (size_t)height);
        ipt::RenderParams p;
        p.spp = (int)spp;
        p.n_rays = (int)n_rays;
        p.depth_max = (int)depth;
        p.seed = seed;
        double kernel_ms = 0.0;
        const auto t0 = std::chrono::steady_clock::now();
        for (long pass = 0; pass < passes; ++pass) {  // progressive: each batch continues the RNG stream
            p.spp_offset = (int)(pass * spp);
            gpus.render(plane, p);
            float pm = 0.0f, am = 0.0f;
            gpus.last_kernel_ms(&pm, &am);
            kernel_ms += pm + am;
        }
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        uint64_t h2d = 0, d2h = 0;  // the last batch's plane transfers (all contexts)
        gpus.transfer_bytes(&h2d, &d2h);
        if (smooth > 0) gpu.smooth(plane, (size_t)smooth);
        if (glare >= 0.0 && !glare_out.empty()) {
            ipt::GridRenderPlane g(plane.width, plane.height);
            g.pixels = gpu.glare(plane, (float)glare);
            ipt::write_pfm(glare_out, g);
        }
        if (!pgm.empty()) ipt::write_pgm(pgm, plane);
        if (!out.empty()) ipt::write_png_gray8(out, plane.width, plane.height, ipt::to_gray8(plane));
        if (!pfm.empty()) ipt::write_pfm(pfm, plane);
        if (!counts.empty()) {
            std::ofstream f(counts, std::ios::binary);
            for (size_t c : plane.pixel_counters) {
                const uint32_t v = (uint32_t)c;
                f.write(reinterpret_cast<const char*>(&v), 4);
            }
        }
        const double paths = (double)width * height * spp * passes;
        std::printf(
            "{\"scene\": \"%s\", \"width\": %ld, \"height\": %ld, \"spp\": %ld, \"passes\": %ld, "
            "\"n_rays\": %ld, \"depth_max\": %ld, \"devices\": %zu, \"max_value\": %.9g, \"seconds\": %.4f, "
            "\"Mpaths_per_s\": %.3f, \"kernel_Mpaths_per_s\": %.3f, \"last_batch_h2d_bytes\": %llu, "
            "\"last_batch_d2h_bytes\": %llu}\n",
            scene_name.c_str(), width, height, spp, passes, n_rays, depth, gpus.size(), (double)plane.max_value, secs,
            paths / secs / 1e6, kernel_ms > 0 ? paths / (kernel_ms * 1e-3) / 1e6 : 0.0, (unsigned long long)h2d,
            (unsigned long long)d2h);
    } catch (const ipt::IptError& e) {
        std::fprintf(stderr, "ipt_render: error %d: %s\n", e.code, e.what());
        return 1;
    }
    return 0;
}
