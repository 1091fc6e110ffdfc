// Analysis tool (not product code): replays C2 paths through the oracle and
// classifies the iterations whose light pick is a certain skip (the node lies
// behind the light's plane), to price skip-merging policies of the path
// kernel's step loop before writing them (it links the C-ABI library only for
// the host layer's scene builder; no GPU is used). Build and run:
//   g++ -O2 -std=c++17 -Iinclude -Iipt_amd/host scripts/skip_stats.cpp ipt_amd/host/ipt_host.cpp \
//       -o /tmp/skip_stats -lpthread -L ipt_amd/lib -lipt_hip -Wl,-rpath,$PWD/ipt_amd/lib
//   /tmp/skip_stats 128 4      # 128x128 pixels, 4 passes of sample_scenes[0]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

struct Ev {
    int depth, i, n;
    uint32_t k;
    bool skip, back;
};
static thread_local std::vector<Ev>* g_evs = nullptr;
static float g_pz = 0.0f, g_nz = 0.0f;
#define IPT_ORACLE_ITER_HOOK(depth, i, n, k, skip, pos) \
    do {                                                 \
        if (g_evs) g_evs->push_back(Ev{depth, i, n, k, skip, ((pos).z - g_pz) * g_nz < 0.0f}); \
    } while (0)
#include "../oracle/ipt_oracle.cpp"
#include "ipt_host.h"

struct Pol {
    const char* name;
    uint32_t jmerge, omax, jmax;
    bool pre, post;
};
static const Pol kPols[] = {
    {"prologue merge j<=1 (product)", 1, 0, 3, false, false},
    {"prologue merge j<=2", 2, 0, 3, false, false},
    {"merge j<=1 + pre-pop pre-skip, o<=4 (window as now)", 1, 4, 3, true, false},
    {"merge j<=1 + pre-pop pre-skip, o<=6 (j up to 5)", 1, 6, 5, true, false},
    {"no merge + pre-pop pre-skip, o<=6", 0xffffffffu, 6, 5, true, false},
    {"merge j<=1 + post-pop pre-skip (non-last), o<=6", 1, 6, 5, false, true},
    {"merge j<=1 + pre-pop and post-pop pre-skips, o<=6", 1, 6, 5, true, true},
    {"12-word window: merge j<=1 + pre-pop pre-skip, o<=7 (j up to 6)", 1, 7, 6, true, false},
    {"12-word window: merge j<=2 + pre-pop pre-skip, o<=7 (j up to 6)", 2, 7, 6, true, false},
    {"12-word window: merge j<=1 + pre-pop pre-skip, o<=9 (j up to 8)", 1, 9, 8, true, false},
};
constexpr int kPol = sizeof(kPols) / sizeof(kPols[0]);

int main(int argc, char** argv) {
    const int W = argc > 1 ? std::atoi(argv[1]) : 256;
    const int spp = argc > 2 ? std::atoi(argv[2]) : 4;
    ipt::FlatScene f = ipt::flatten(ipt::make_scene_by_name("box"));
    const ipt_area_light& L = f.lights[0];
    const float nx = L.x_axis[1] * L.y_axis[2] - L.x_axis[2] * L.y_axis[1];
    const float ny = L.x_axis[2] * L.y_axis[0] - L.x_axis[0] * L.y_axis[2];
    const float nz = L.x_axis[0] * L.y_axis[1] - L.x_axis[1] * L.y_axis[0];
    g_pz = L.position[2];
    g_nz = nz / std::sqrt(nx * nx + ny * ny + nz * nz);
    ipt_params p{};
    p.width = W;
    p.height = W;
    p.spp = 1;
    p.n_rays = 16;
    p.depth_max = 8;
    p.seed = 0x1234abcdULL;
    SceneO sc = make_scene(&f.scene);
    Mixture mix = build_mixture(sc);
    Ctx cx{&sc, &mix, p.depth_max};
    // policies: steps per path when certain skips merge into the next iteration's step
    uint64_t paths = 0, iters = 0, skips = 0, cert = 0, cert_last = 0, cert_j[4] = {}, cert_chain = 0,
             n1_cert = 0, merged_cur = 0, merged_any1 = 0, merged_chain = 0, sim_steps[kPol] = {}, sim_bad[kPol] = {}, rem[4] = {}, rem_j[6] = {};
    std::vector<Ev> evs;
    g_evs = &evs;
    for (int s = 0; s < spp; ++s)
        for (int iy = 0; iy < W; ++iy)
            for (int ix = 0; ix < W; ++ix) {
                evs.clear();
                p.spp_offset = s;
                int xo, yo;
                oracle_pixel(cx, &p, ix, iy, 0, &xo, &yo);
                ++paths;
                iters += evs.size();
                // Step simulation (8-word window, one shift per step: at the step's
                // start the window holds blocks blk, blk + 1 with blk advanced once
                // when k >= 4 blk + 4, so j = k - 4 blk may reach 5). A step takes one
                // event; the prologue merges a certain skip that is not its node's last
                // iteration with the next one when j <= jmerge; after the step, the
                // next event is consumed as well when it is a certain skip of the same
                // node (i + 1) or of the pushed child (i = 0) and its pick word offset
                // o <= omax (so that the next step's j stays <= 5).
                for (int pol = 0; pol < kPol; ++pol) {
                    const Pol& q = kPols[pol];
                    uint32_t blk = 0;
                    for (size_t e = 0; e < evs.size();) {
                        const Ev& v = evs[e];
                        ++sim_steps[pol];
                        if (v.k >= 4u * blk + 4u) ++blk;
                        const uint32_t j = v.k - 4u * blk;
                        if (j > q.jmax) ++sim_bad[pol];
                        size_t r = e;  // the step's real event
                        if (v.skip && v.back && v.i != v.n - 1 && j <= q.jmerge) r = e + 1;
                        size_t nx = r + 1;
                        // pre-skip before the step's pop: the next event of the same node or of the pushed child
                        if (q.pre && nx < evs.size()) {
                            const Ev& a = evs[r];
                            const Ev& b = evs[nx];
                            const bool same = b.depth == a.depth && b.i == a.i + 1;
                            const bool child = b.depth == a.depth + 1 && b.i == 0;
                            if ((same || child) && b.skip && b.back && b.k - 4u * blk <= q.omax) ++nx;
                        }
                        // pre-skip after the pop: the next event whatever it is, if not its node's last
                        if (q.post && nx < evs.size()) {
                            const Ev& b = evs[nx];
                            if (b.skip && b.back && b.i != b.n - 1 && b.k - 4u * blk <= q.omax) ++nx;
                        }
                        if (pol == 3) {
                            // the step's own event when it is still a certain skip (a lane-step spent on it)
                            const Ev& a = evs[r];
                            if (a.skip && a.back) {
                                const bool after_pop = r > 0 && evs[r - 1].depth > a.depth;
                                const bool last = a.i == a.n - 1;
                                ++rem[(after_pop ? 2 : 0) + (last ? 1 : 0)];
                                if (!after_pop && !last) ++rem_j[j > 5u ? 5u : j];
                            }
                        }
                        e = nx;
                    }
                }
                // events arrive in DFS order; within a node consecutive i
                bool prev_merged_skip = false;  // previous event (same node, i-1) was a skip merged into this step
                for (size_t e = 0; e < evs.size(); ++e) {
                    const Ev& v = evs[e];
                    if (v.skip) ++skips;
                    const bool c = v.skip && v.back;
                    if (!c) { prev_merged_skip = false; continue; }
                    ++cert;
                    const bool last = v.i == v.n - 1;
                    if (last) ++cert_last;
                    if (v.n == 1) ++n1_cert;
                    ++cert_j[v.k & 3u];
                    if (!last) {
                        // the product rule: j <= 1, one skip per step
                        if ((v.k & 3u) <= 1u && !prev_merged_skip) ++merged_cur;
                        if (!prev_merged_skip) ++merged_any1;
                        ++merged_chain;
                        if (prev_merged_skip) ++cert_chain;
                        prev_merged_skip = true;
                    } else {
                        prev_merged_skip = false;
                    }
                }
            }
    const double P = (double)paths;
    for (int pol = 0; pol < kPol; ++pol)
        std::printf("%-55s lane-steps per path %.3f (j beyond the window: %llu)\n", kPols[pol].name,
                    sim_steps[pol] / P, (unsigned long long)sim_bad[pol]);
    std::printf("product policy: certain-skip lane-steps left: not after a pop: non-last %.3f last %.3f | after a pop: non-last %.3f last %.3f\n",
                rem[0] / P, rem[1] / P, rem[2] / P, rem[3] / P);
    std::printf("  (not after a pop, non-last, by j: %.3f %.3f %.3f %.3f %.3f %.3f)\n", rem_j[0] / P, rem_j[1] / P,
                rem_j[2] / P, rem_j[3] / P, rem_j[4] / P, rem_j[5] / P);
    std::printf("paths %llu iterations/path %.3f skipped %.3f certain %.3f (last-iteration %.3f, n=1 nodes %.3f)\n",
                (unsigned long long)paths, iters / P, skips / P, cert / P, cert_last / P, n1_cert / P);
    std::printf("certain by window offset j: %.3f %.3f %.3f %.3f; second-in-a-row %.3f\n", cert_j[0] / P,
                cert_j[1] / P, cert_j[2] / P, cert_j[3] / P, cert_chain / P);
    std::printf("merged per path: j<=1 one per step %.3f | any j one per step %.3f | chains %.3f\n",
                merged_cur / P, merged_any1 / P, merged_chain / P);
    std::printf("lane-steps per path: none %.3f | current %.3f | any-j %.3f | chains %.3f | chains + n=1 push elision %.3f\n",
                iters / P, (iters - merged_cur) / P, (iters - merged_any1) / P, (iters - merged_chain) / P,
                (iters - merged_chain - n1_cert) / P);
    return 0;
}
