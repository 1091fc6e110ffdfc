// Golden vectors for Gui's glare, produced by the
// reference's OWN static glare() (gui.cpp:38-52, with draw_halo gui.cpp:28-36
// and CImg::cut CImg.h:33334). glare() has internal linkage, so this harness
// compiles the reference's gui.cpp translation unit where it lies under
// /root/reference (included by path, nothing copied) and calls it directly;
// no Gui / CImgDisplay object is ever constructed (no X display is opened).
// Built by oracle/build_ref.sh into oracle/_ref/ref_glare; the output file
// tests/golden/ref_glare.bin is data (inputs + the reference's outputs):
//   float32 n_cases, then per case: W, H, cutoff, input[W*H], output[W*H].
// Test infrastructure only (tests/test_post.py), never the product path.
#include "gui.cpp"

#include <cmath>
#include <cstdio>
#include <cstdint>
#include <limits>
#include <vector>

namespace {
struct Case {
    int W, H;
    float cutoff;
    std::vector<float> in;
};

uint32_t g_state = 0x9e3779b9u;
float unit() {  // xorshift32 -> [0,1)
    g_state ^= g_state << 13;
    g_state ^= g_state >> 17;
    g_state ^= g_state << 5;
    return (g_state >> 8) * (1.0f / 16777216.0f);
}

Case random_case(int W, int H, float cutoff, float hot_frac, float hot_scale) {
    Case c{W, H, cutoff, std::vector<float>((size_t)W * H)};
    for (auto& v : c.in) {
        v = unit() * 0.5f * cutoff;
        if (unit() < hot_frac) v = cutoff + unit() * hot_scale;
    }
    return c;
}
}  // namespace

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : ".";
    std::vector<Case> cases;
    {  // one bright pixel, GUI cutoff as in gui.h:25
        Case c{9, 7, 1.01f, std::vector<float>(63, 0.0f)};
        c.in[3 * 9 + 4] = 10.0f;
        cases.push_back(c);
    }
    cases.push_back(random_case(64, 48, 1.0f, 0.03f, 40.0f));
    cases.push_back(random_case(97, 33, 1.01f, 0.2f, 40.0f));
    {  // non-default cutoff; negative pixels, a pixel exactly at the cutoff,
       // one just above it and one +inf (its halo saturates every pixel)
        Case c = random_case(40, 40, 0.37f, 0.05f, 3.0f);
        c.in[0] = -2.0f;
        c.in[41] = 0.37f;
        c.in[82] = std::nextafter(0.37f, 1.0f);
        cases.push_back(c);
        Case d = random_case(23, 17, 0.37f, 0.02f, 3.0f);
        d.in[100] = std::numeric_limits<float>::infinity();
        cases.push_back(d);
    }
    {  // a NaN above nothing: !(NaN <= cutoff) draws a NaN halo everywhere
        Case c = random_case(11, 5, 1.0f, 0.0f, 0.0f);
        c.in[7] = std::numeric_limits<float>::quiet_NaN();
        cases.push_back(c);
    }
    cases.push_back(random_case(1, 1, 1.0f, 1.0f, 5.0f));
    cases.push_back(random_case(1, 37, 2.5f, 0.3f, 10.0f));
    cases.push_back(random_case(200, 3, 1.0f, 0.1f, 1e4f));

    std::string path = std::string(dir) + "/ref_glare.bin";
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return 1;
    const float n = (float)cases.size();
    std::fwrite(&n, 4, 1, f);
    for (const Case& c : cases) {
        CImg<float> img(c.W, c.H);
        for (int y = 0; y < c.H; ++y)
            for (int x = 0; x < c.W; ++x) img(x, y) = c.in[(size_t)y * c.W + x];
        CImg<float> out = glare(img, c.cutoff);
        const float hdr[3] = {(float)c.W, (float)c.H, c.cutoff};
        std::fwrite(hdr, 4, 3, f);
        std::fwrite(c.in.data(), 4, c.in.size(), f);
        for (int y = 0; y < c.H; ++y)
            for (int x = 0; x < c.W; ++x) {
                const float v = out(x, y);
                std::fwrite(&v, 4, 1, f);
            }
    }
    std::fclose(f);
    std::printf("%zu glare cases -> %s\n", cases.size(), path.c_str());
    return 0;
}
