// ipt_bvh.h — exact-result acceleration for the sphere-list geometry
// (IPT_GEOM_SPHERES_IN_BOX, BASELINE configs[2]).
//
// The reference scans every sphere (FractalSpheres.cpp:75-84) and keeps the
// first sphere whose t is the strict minimum. A BVH returns the same sphere
// iff (1) no sphere that the scan would accept is pruned and (2) ties on t are
// broken by the lowest original index. (1) holds because every node box is
// the union of its spheres' boxes padded by a relative margin far above the
// rounding error of sphere_t's hit point, and a subtree is skipped on its
// entry distance only with a margin; (2) is enforced explicitly. The exact
// per-sphere test is the same sphere_t() the brute-force path uses, so the
// result is bit-identical (tests/test_gpu_parity.py::test_spheres_in_box_*).
//
// Layout: nodes in depth-first order with skip links (stackless traversal):
// an inner node's first child is the next node; `skip` is the node after its
// subtree. Leaves reference a contiguous range of the reordered sphere array.
#pragma once

#include <algorithm>
#include <cmath>
#include <functional>
#include <vector>

#include "ipt_math.h"

namespace ipt {

struct BvhNode {
    float bmin[3];
    int skip;   // next node index when this subtree is done or missed
    float bmax[3];
    int leaf;   // -1: inner; else first sphere index (reordered) | count << 24
};

struct BvhSphere {
    float c[3];
    float r;
    int index;  // original index (FractalSpheres' scan order)
    int pad[3];
};

// Host builder: median split on the widest axis, leaves of <= 4 spheres.
// The tree is emitted as kBvhOrders = 8 depth-first linearisations, one per
// ray-direction octant (bit a set = direction negative along axis a): at every
// inner node the child on the near side of the split axis comes first, so the
// stackless walk meets near hits early and prunes the rest on `best`. The
// order only changes how much is visited, never the result (tie-break above).
constexpr int kBvhOrders = 8;
inline void bvh_build(const float* cr /* [n][4] c.xyz r */, int n, std::vector<BvhNode>& nodes,
                      std::vector<BvhSphere>& prims, int* nodes_per_order) {
    nodes.clear();
    prims.clear();
    *nodes_per_order = 0;
    if (n <= 0) return;
    struct TreeNode {
        float lo[3], hi[3];
        int axis, leaf, child[2];
    };
    std::vector<TreeNode> tree;
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    auto sphere_box = [&](int i, float* lo, float* hi) {
        const float r = cr[4 * i + 3];
        for (int a = 0; a < 3; ++a) {
            const float c = cr[4 * i + a];
            // relative + absolute padding: >> the float error of o + d*t
            const float pad = 1e-4f * (std::fabs(c) + r + 1.0f);
            lo[a] = c - r - pad;
            hi[a] = c + r + pad;
        }
    };
    std::function<int(int, int)> rec = [&](int lo, int hi) -> int {
        TreeNode tn{};
        for (int a = 0; a < 3; ++a) {
            tn.lo[a] = INFINITY;
            tn.hi[a] = -INFINITY;
        }
        for (int k = lo; k < hi; ++k) {
            float l[3], h[3];
            sphere_box(idx[k], l, h);
            for (int a = 0; a < 3; ++a) {
                tn.lo[a] = std::min(tn.lo[a], l[a]);
                tn.hi[a] = std::max(tn.hi[a], h[a]);
            }
        }
        const int me = (int)tree.size();
        tree.push_back(tn);
        if (hi - lo <= 4) {
            tree[me].leaf = (int)prims.size() | ((hi - lo) << 24);
            for (int k = lo; k < hi; ++k) {
                BvhSphere s{};
                for (int a = 0; a < 3; ++a) s.c[a] = cr[4 * idx[k] + a];
                s.r = cr[4 * idx[k] + 3];
                s.index = idx[k];
                prims.push_back(s);
            }
            return me;
        }
        int axis = 0;
        float ext = tn.hi[0] - tn.lo[0];
        for (int a = 1; a < 3; ++a)
            if (tn.hi[a] - tn.lo[a] > ext) {
                ext = tn.hi[a] - tn.lo[a];
                axis = a;
            }
        const int mid = (lo + hi) / 2;
        std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi,
                         [&](int x, int y) { return cr[4 * x + axis] < cr[4 * y + axis]; });
        const int c0 = rec(lo, mid);  // lower half along axis
        const int c1 = rec(mid, hi);
        tree[me].leaf = -1;
        tree[me].axis = axis;
        tree[me].child[0] = c0;
        tree[me].child[1] = c1;
        return me;
    };
    rec(0, n);
    const int per = (int)tree.size();
    *nodes_per_order = per;
    nodes.resize((size_t)per * kBvhOrders);
    for (int oct = 0; oct < kBvhOrders; ++oct) {
        BvhNode* out = nodes.data() + (size_t)per * oct;
        int next = 0;
        std::function<void(int)> emit = [&](int k) {
            const int me = next++;
            const TreeNode& tn = tree[k];
            for (int a = 0; a < 3; ++a) {
                out[me].bmin[a] = tn.lo[a];
                out[me].bmax[a] = tn.hi[a];
            }
            out[me].leaf = tn.leaf;
            if (tn.leaf < 0) {
                const int neg = (oct >> tn.axis) & 1;  // negative direction: upper half first
                emit(tn.child[neg]);
                emit(tn.child[1 - neg]);
            }
            out[me].skip = next;
        };
        emit(0);
    }
}

}  // namespace ipt
