// Host check of the light lattice (ipt_path.h light_grid_build + the path
// kernel's candidate lookup, restated here with the same float operations).
// stdin: n, then n lines "px py pz xx xy xz yx yy yz power type"; argv[1] =
// number of random rays. Prints the lattice verdict and, for an accepted
// lattice, checks that every light the exact axis-aligned test hits lies in
// one of the <= 4 candidate cells, for random rays and for rays aimed at
// cell edges and corners. Exit status 0 = no light missed.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../ipt_amd/csrc/ipt_path.h"

using namespace ipt;

int main(int argc, char** argv) {
    const long nrays = argc > 1 ? std::atol(argv[1]) : 100000;
    int n = 0;
    if (std::scanf("%d", &n) != 1 || n <= 0) return 2;
    std::vector<LightDev> L(n);
    for (int i = 0; i < n; ++i) {
        float v[11];
        for (float& f : v)
            if (std::scanf("%f", &f) != 1) return 2;
        L[i] = make_light(v3(v[0], v[1], v[2]), v3(v[3], v[4], v[5]), v3(v[6], v[7], v[8]), v[9], (int)v[10]);
    }
    LightGrid g;
    const bool ok = light_grid_build(L.data(), n, g);
    std::printf("lattice %d pattern %d nu %d nv %d e_log2 %d\n", ok ? 1 : 0, g.pattern, g.nu, g.nv,
                ok ? (int)std::lround(std::log2(g.e)) : 0);
    if (!ok) return 0;
    const int XA = g.pattern == 1 ? 1 : 0, YA = 1 - XA;
    auto comp = [](vec3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); };
    std::mt19937_64 rng(5);
    std::uniform_real_distribution<float> U(-1.0f, 1.0f);
    long missed = 0, hits = 0, multi = 0;
    const float cw = 1.0f / g.icw, ch = 1.0f / g.ich;
    for (long r = 0; r < nrays; ++r) {
        // origins inside the box below the light plane; targets on the plane,
        // every other ray aimed at a cell edge or corner of the lattice
        const vec3 o = v3(U(rng), U(rng), U(rng) * 0.5f - 0.5f);
        float tu = g.u0 + (U(rng) * 0.6f + 0.5f) * g.nu * cw, tv = g.v0 + (U(rng) * 0.6f + 0.5f) * g.nv * ch;
        if (r & 1) {
            tu = g.u0 + (float)(rng() % (g.nu + 1)) * cw;
            if (r & 2) tv = g.v0 + (float)(rng() % (g.nv + 1)) * ch;
        }
        vec3 t = v3(0, 0, g.pn);
        (XA == 0 ? t.x : t.y) = tu;
        (YA == 0 ? t.x : t.y) = tv;
        const vec3 d = normalize(t - o);
        // the kernel's lookup
        const float n_dir = g.nn * d.z;
        const float tt = g.nn * (g.pn - o.z) / n_dir;
        const float u = (comp(o, XA) + comp(d, XA) * tt - g.u0) * g.icw;
        const float v = (comp(o, YA) + comp(d, YA) * tt - g.v0) * g.ich;
        std::vector<int> cand;
        if (u > -1.0f && u < (float)g.nu + 1.0f && v > -1.0f && v < (float)g.nv + 1.0f) {
            const float e = g.e;
            const int is[2] = {(int)std::floor(u - e), (int)std::floor(u + e)};
            const int js[2] = {(int)std::floor(v - e), (int)std::floor(v + e)};
            for (int a = 0; a < 2; ++a)
                for (int b = 0; b < 2; ++b) {
                    const int i = is[a], j = js[b];
                    if (i >= 0 && i < g.nu && j >= 0 && j < g.nv && g.cells[i + g.nu * j] >= 0)
                        cand.push_back(g.cells[i + g.nu * j]);
                }
        }
        int nh = 0;
        for (int l = 0; l < n; ++l) {
            vec3 hp, hn;
            const bool h = XA == 1 ? light_trace_ax<1, 0, false>(L[l], o, d, &hp, &hn)
                                   : light_trace_ax<0, 1, false>(L[l], o, d, &hp, &hn);
            if (!h) continue;
            ++nh;
            bool found = false;
            for (int c : cand) found |= c == l;
            if (!found) ++missed;
        }
        hits += nh;
        multi += nh > 1;
    }
    std::printf("rays %ld hits %ld multi %ld missed %ld\n", nrays, hits, multi, missed);
    return missed != 0;
}
