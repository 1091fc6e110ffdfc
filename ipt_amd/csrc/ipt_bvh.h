// ipt_bvh.h — exact-result acceleration structures for the two O(N) scans on
// the path: the sphere list (IPT_GEOM_SPHERES_IN_BOX, BASELINE configs[2],
// FractalSpheres.cpp:75-84) and the light list (CollectionLighting.cpp:23-34
// and UnionDdf::value over its lights, ddf.cpp:157-162; configs with L=256).
//
// A BVH returns the scan's result iff no item that the scan would accept is
// skipped, and ties are resolved as the scan resolves them.
//
// * Conservativeness. Every item box is padded so that any ray the exact
//   per-item test (sphere_t / light_trace, the same functions the scans use)
//   accepts passes through the padded box, rounding included. The padding is
//   derived from a bound D on |origin - item| (ray origins are the camera or
//   surface points of the scene, both known at upload):
//     sphere: the float discriminant 4b^2 - 4(|oc|^2 - r^2) carries an
//       absolute error below ~1e-6 D^2 (dot products, squares, |d| != 1), so a
//       ray whose distance to the centre is up to sqrt(r^2 + 4e-6 D^2) may be
//       accepted: pad = (sqrt(r^2 + 4e-6 D^2) - r) + 1e-4 (|c| + r + 1).
//       Near tangency the computed t moves by up to sqrt(4e-6) D / 2 = 1e-3 D
//       along the ray, so an accepted t may lie up to 1e-3 D before the padded
//       box's entry: the walk's pruning compare (entry <= best) carries that
//       as an additive margin, tmargin = max over spheres of 1e-3 D (rather
//       than padding every box by it, which made boxes ~2x the volume).
//     light: the hit point o + d t and coord = inv * rel carry errors of a few
//       ulps of D plus cond(M) ulps of the light extent. pad = 1e-5 D
//       + 1e-4 (|P| + |x| + |y| + 1) + 1e-5 cond (|x| + |y|); ill-conditioned
//       (cond > 1e4) or non-finite lights disable the light BVH.
//   The slab test itself uses approximate reciprocals with a relative margin.
// * Ties. Spheres: the walk can meet them in any order, so equal t is broken
//   by the lowest original index (the scan's first-strict-minimum). Lights:
//   the tree is built over contiguous INDEX ranges, so its depth-first walk
//   meets lights in increasing index order and the scan's running compare and
//   running sum are reproduced operation for operation; a light the walk skips
//   would have contributed exactly +0 to the sum and nothing to the nearest
//   hit.
//
// Layout: nodes in depth-first order with skip links (stackless traversal):
// an inner node's first child is the next node; `skip` is the node after its
// subtree. Leaves reference a contiguous range of items.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "ipt_knobs.h"
#include "ipt_math.h"

namespace ipt {

struct BvhNode {
    float bmin[3];
    int skip;   // next node index when this subtree is done or missed
    float bmax[3];
    int leaf;   // -1: inner; else first item | count << 24
};

struct BvhSphere {
    float c[3];
    float r;
    int index;  // original index (FractalSpheres' scan order)
    int pad[3];
};

struct BvhBox {
    float lo[3], hi[3];
};

// Binary tree over items [0, n) with item boxes `box`. spatial: median split
// of box centres on the widest axis (items permuted, `perm` = original index
// per slot); otherwise split the index range in half (perm = identity, leaves
// in index order). Emits `orders` depth-first linearisations of
// nodes_per_order nodes each: with orders == 8, linearisation `oct` (bit a set
// = ray direction negative on axis a) puts the near child first at every node.
inline void bvh_build_boxes(const std::vector<BvhBox>& box, int leaf_size, bool spatial, int orders,
                            std::vector<BvhNode>& nodes, std::vector<int>& perm, int* nodes_per_order) {
    const int n = (int)box.size();
    nodes.clear();
    perm.clear();
    *nodes_per_order = 0;
    if (n <= 0) return;
    struct TreeNode {
        float lo[3], hi[3];
        int axis, leaf, child[2];
    };
    std::vector<TreeNode> tree;
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    std::function<int(int, int)> rec = [&](int lo, int hi) -> int {
        TreeNode tn{};
        for (int a = 0; a < 3; ++a) {
            tn.lo[a] = INFINITY;
            tn.hi[a] = -INFINITY;
        }
        for (int k = lo; k < hi; ++k)
            for (int a = 0; a < 3; ++a) {
                tn.lo[a] = std::min(tn.lo[a], box[idx[k]].lo[a]);
                tn.hi[a] = std::max(tn.hi[a], box[idx[k]].hi[a]);
            }
        const int me = (int)tree.size();
        tree.push_back(tn);
        if (hi - lo <= leaf_size) {
            tree[me].leaf = (int)perm.size() | ((hi - lo) << 24);
            for (int k = lo; k < hi; ++k) perm.push_back(idx[k]);
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
        if (spatial)
            std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi, [&](int x, int y) {
                return box[x].lo[axis] + box[x].hi[axis] < box[y].lo[axis] + box[y].hi[axis];
            });
        const int c0 = rec(lo, mid);  // lower half (along axis, or of the index range)
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
    nodes.resize((size_t)per * orders);
    for (int oct = 0; oct < orders; ++oct) {
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
                // negative direction along the split axis: upper half first
                const int neg = (spatial && orders == 8) ? (oct >> tn.axis) & 1 : 0;
                emit(tn.child[neg]);
                emit(tn.child[1 - neg]);
            }
            out[me].skip = next;
        };
        emit(0);
    }
}

// Bound on |origin - p| for every ray origin of the scene and every point p
// of an item box [lo, hi]: origins are the camera or surface points in [-B, B]^3.
inline double origin_bound(const float cam[3], float B, const float lo[3], const float hi[3]) {
    double dc = 0.0, db = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double e1 = std::max(std::fabs((double)cam[a] - lo[a]), std::fabs((double)cam[a] - hi[a]));
        const double e2 = (double)B + std::max(std::fabs((double)lo[a]), std::fabs((double)hi[a]));
        dc += e1 * e1;
        db += e2 * e2;
    }
    return std::sqrt(std::max(dc, db));
}

constexpr int kBvhOrders = 8;

// Sphere BVH (8 octant orders, leaves of <= IPT_BVH_LEAF spheres; measured on
// C3: 16 beats 2/4/8/32/64). cr: [n][4] c.xyz r. *tmargin: the pruning margin.
inline void bvh_build_spheres(const float* cr, int n, const float cam[3], float B, std::vector<BvhNode>& nodes,
                              std::vector<BvhSphere>& prims, int* nodes_per_order, float* tmargin) {
    std::vector<BvhBox> box(n);
    double tm = 0.0;
    for (int i = 0; i < n; ++i) {
        const float r = cr[4 * i + 3];
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = cr[4 * i + a] - r;
            hi[a] = cr[4 * i + a] + r;
        }
        const double D = origin_bound(cam, B, lo, hi);
        const double cn = std::fabs((double)cr[4 * i]) + std::fabs((double)cr[4 * i + 1]) +
                          std::fabs((double)cr[4 * i + 2]);
        const double pad = (std::sqrt((double)r * r + 4e-6 * D * D) - r) + 1e-4 * (cn + r + 1.0);
        tm = std::max(tm, 1e-3 * D);
        for (int a = 0; a < 3; ++a) {
            box[i].lo[a] = (float)((double)lo[a] - pad);
            box[i].hi[a] = (float)((double)hi[a] + pad);
        }
    }
    *tmargin = (float)(tm * (1.0 + 1e-6)) + 1e-7f;  // rounded up
    std::vector<int> perm;
    bvh_build_boxes(box, IPT_BVH_LEAF, true, kBvhOrders, nodes, perm, nodes_per_order);
    prims.resize(perm.size());
    for (size_t k = 0; k < perm.size(); ++k) {
        const int i = perm[k];
        BvhSphere s{};
        for (int a = 0; a < 3; ++a) s.c[a] = cr[4 * i + a];
        s.r = cr[4 * i + 3];
        s.index = i;
        prims[k] = s;
    }
}

// Uniform grid over the sphere list (IPT_GEOM_SPHERES_IN_BOX, many small
// spheres — BASELINE configs[2]): a ray walks the cells it crosses in order
// (3D DDA) and stops once the next cell starts beyond the best hit, so a walk
// costs the cells along the (short) ray instead of a root-to-leaf descent per
// candidate. Exactness, with the BVH's padded sphere boxes and margin:
// * registration: a sphere's padded box (ipt_bvh.h header) is the bound of
//   its padded ball (centre c, radius R = r + pad: the box's half-width), and
//   any ray the exact sphere_t accepts passes within R of c. With
//   IPT_GRID_SPHERE_REG (default) the sphere is registered in every cell of
//   its box range (inflated by m, computed in double, rounded outward) whose
//   distance to the box centre is at most R + m + 1e-6 (1 + |c|_1) (the last
//   term covers the box centre's offset from the float centre, i.e. the
//   roundings of c -+ r), times (1 + 1e-9); without it, in every cell of the
//   box range;
// * walk: the DDA's float rounding (approximate reciprocals, cell-boundary
//   t's) can only make it visit a cell adjacent to the exact ray's where the
//   ray passes within ~1e-6 |t| of a cell edge. Let q be the exact ray's
//   point nearest c, inside the ball, and Q the cell holding q: Q is within
//   R of c, hence registered; where the DDA strays it visits instead a
//   neighbour of Q whose distance to q is < 1e-6 |t|, far inside m = 1e-4
//   (1 + max |coord|), so that neighbour is within R + m of c and registered
//   too. Every accepted sphere is therefore in a cell the walk visits at
//   some t <= (ball entry t) + m, and the ball's entry t is >= the padded
//   box's entry t;
// * it stops after a cell whose exit t exceeds (best*1.0001 + 1e-5 + tmargin
//   + m) * (1 + 1e-5) + 1e-5: a sphere registered only in later cells has its
//   ball entry (>= its box entry) beyond best + tmargin, and (tmargin:
//   tangency t-error) cannot produce a computed t below or equal to best;
// * order: each cell's items are in ascending original index (the fill loop
//   runs over i in order; checked after the fill), which the wave walk's
//   (t bits, item position) slot key relies on for the lowest-index tie rule;
// * ties: equal t is broken by the lowest original index, as in the BVH
//   (spheres registered in several cells are tested again, harmlessly).
struct SphereGrid {
    float g0[3], h[3], inv_h[3];
    int n[3];
    float m, tmargin;
    std::vector<int> start;         // [cells + 1]
    std::vector<BvhSphere> items;   // per-cell sphere records
};

// A grid cell with its first three items inline (64 bytes, one cache line):
// the walk's next cell is known from the DDA alone, so its record -- item
// range and first items -- is fetched one cell ahead in a single round trip
// instead of the range, then the items. Items beyond the third are read from
// SphereGrid::items[s0 + 3, s1) as before; it[q] copies items[s0 + q].c / r.
struct GridCell {
    int s0, s1, pad0, pad1;
    float it[3][4];
};
static_assert(sizeof(GridCell) == 64, "GridCell is one 64-byte line");
inline void grid_cells_build(const SphereGrid& g, std::vector<GridCell>& cells) {
    const size_t nc = g.start.size() - 1;
    cells.assign(nc, GridCell{});
    for (size_t c = 0; c < nc; ++c) {
        GridCell& r = cells[c];
        r.s0 = g.start[c];
        r.s1 = g.start[c + 1];
        for (int q = 0; q < 3 && r.s0 + q < r.s1; ++q) {
            const BvhSphere& b = g.items[(size_t)r.s0 + q];
            r.it[q][0] = b.c[0];
            r.it[q][1] = b.c[1];
            r.it[q][2] = b.c[2];
            r.it[q][3] = b.r;
        }
    }
}

inline bool grid_build_spheres(const float* cr, int n, const float cam[3], float B, SphereGrid& g) {
    if (n <= 0) return false;
    std::vector<double> lo(3 * (size_t)n), hi(3 * (size_t)n);
    double glo[3] = {INFINITY, INFINITY, INFINITY}, ghi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double tm = 0.0, maxabs = std::max(std::fabs((double)cam[0]), std::max(std::fabs((double)cam[1]), std::fabs((double)cam[2])));
    for (int i = 0; i < n; ++i) {
        const float r = cr[4 * i + 3];
        float blo[3], bhi[3];
        for (int a = 0; a < 3; ++a) {
            blo[a] = cr[4 * i + a] - r;
            bhi[a] = cr[4 * i + a] + r;
        }
        const double D = origin_bound(cam, B, blo, bhi);
        const double cn = std::fabs((double)cr[4 * i]) + std::fabs((double)cr[4 * i + 1]) +
                          std::fabs((double)cr[4 * i + 2]);
        const double pad = (std::sqrt((double)r * r + 4e-6 * D * D) - r) + 1e-4 * (cn + r + 1.0);
        if (!std::isfinite(pad) || !std::isfinite(cn) || !(r >= 0.0f)) return false;
        tm = std::max(tm, 1e-3 * D);
        for (int a = 0; a < 3; ++a) {
            lo[3 * (size_t)i + a] = (double)blo[a] - pad;
            hi[3 * (size_t)i + a] = (double)bhi[a] + pad;
            glo[a] = std::min(glo[a], lo[3 * (size_t)i + a]);
            ghi[a] = std::max(ghi[a], hi[3 * (size_t)i + a]);
            maxabs = std::max(maxabs, std::max(std::fabs(glo[a]), std::fabs(ghi[a])));
        }
    }
    const double m = 1e-4 * (1.0 + maxabs);
    double ext[3], vol = 1.0;
    for (int a = 0; a < 3; ++a) {
        glo[a] -= 2.0 * m;
        ghi[a] += 2.0 * m;
        ext[a] = ghi[a] - glo[a];
        vol *= ext[a];
    }
    const double hc = std::cbrt(vol / (IPT_GRID_CELLS_PER_SPHERE * n));
    size_t cells = 1;
    for (int a = 0; a < 3; ++a) {
        g.n[a] = (int)std::min(256.0, std::max(1.0, std::round(ext[a] / hc)));
        g.h[a] = (float)(ext[a] / g.n[a]);
        g.g0[a] = (float)glo[a];
        g.inv_h[a] = 1.0f / g.h[a];
        cells *= (size_t)g.n[a];
    }
    g.m = (float)m;
    g.tmargin = (float)(tm * (1.0 + 1e-6)) + 1e-7f;
    // cell range of an inflated box, rounded outward, in double
    auto range = [&](int a, double l, double h2, int* i0, int* i1) {
        const double f0 = (l - m - (double)g.g0[a]) / (double)g.h[a], f1 = (h2 + m - (double)g.g0[a]) / (double)g.h[a];
        *i0 = (int)std::max(0.0, std::floor(f0 - 1e-9));
        *i1 = (int)std::min((double)g.n[a] - 1, std::floor(f1 + 1e-9));
    };
    g.start.assign(cells + 1, 0);
    for (int pass = 0; pass < 2; ++pass) {
        std::vector<int> fill;
        if (pass == 1) {
            for (size_t c = 0; c < cells; ++c) g.start[c + 1] += g.start[c];
            g.items.resize(g.start[cells]);
            fill.assign(g.start.begin(), g.start.end() - 1);
        }
        for (int i = 0; i < n; ++i) {
            int r0[3], r1[3];
            for (int a = 0; a < 3; ++a) range(a, lo[3 * (size_t)i + a], hi[3 * (size_t)i + a], &r0[a], &r1[a]);
            // IPT_GRID_SPHERE_REG: of the padded box's cells, only those within
            // the padded sphere's reach (the box is that sphere's bound: its
            // half-width pad + r enlarges the radius), inflated by m plus a
            // rounding allowance, in double
            double cc[3], reach2 = 0.0;
            if (IPT_GRID_SPHERE_REG) {
                double rr = 0.0;
                for (int a = 0; a < 3; ++a) {
                    cc[a] = 0.5 * (lo[3 * (size_t)i + a] + hi[3 * (size_t)i + a]);
                    rr = std::max(rr, 0.5 * (hi[3 * (size_t)i + a] - lo[3 * (size_t)i + a]));
                }
                // + the box centre's offset from the float centre (fl(c -+ r) roundings)
                const double reach = (rr + m + 1e-6 * (1.0 + std::fabs(cc[0]) + std::fabs(cc[1]) + std::fabs(cc[2]))) *
                                     (1.0 + 1e-9);
                reach2 = reach * reach;
            }
            for (int z = r0[2]; z <= r1[2]; ++z)
                for (int y = r0[1]; y <= r1[1]; ++y)
                    for (int x = r0[0]; x <= r1[0]; ++x) {
                        if (IPT_GRID_SPHERE_REG) {
                            const int xyz[3] = {x, y, z};
                            double d2 = 0.0;
                            for (int a = 0; a < 3; ++a) {
                                const double c0 = (double)g.g0[a] + (double)xyz[a] * (double)g.h[a];
                                const double c1 = (double)g.g0[a] + (double)(xyz[a] + 1) * (double)g.h[a];
                                const double dd = cc[a] < c0 ? c0 - cc[a] : (cc[a] > c1 ? cc[a] - c1 : 0.0);
                                d2 += dd * dd;
                            }
                            if (d2 > reach2) continue;
                        }
                        const size_t c = (size_t)x + (size_t)g.n[0] * ((size_t)y + (size_t)g.n[1] * z);
                        if (pass == 0) {
                            ++g.start[c + 1];
                        } else {
                            BvhSphere sp{};
                            for (int a = 0; a < 3; ++a) sp.c[a] = cr[4 * i + a];
                            sp.r = cr[4 * i + 3];
                            sp.index = i;
                            g.items[fill[c]++] = sp;
                        }
                    }
        }
    }
    // the wave walk's tie rule needs every cell in ascending index order: an
    // internal invariant, so a violation (a changed fill order) aborts loudly
    for (size_t c = 0; c < cells; ++c)
        for (int k = g.start[c] + 1; k < g.start[c + 1]; ++k)
            if (!(g.items[k - 1].index < g.items[k].index)) {
                std::fprintf(stderr, "ipt: sphere grid cell %zu not in ascending index order\n", c);
                std::abort();
            }
    return true;
}

// Light BVH over index ranges (one order, leaves of <= 2 lights, items in
// index order). P, x, y: corner and axes; inv: inverse(mat3(x, y, cross)) as
// the trace uses it (9 floats). Returns false (no BVH) when a light is
// non-finite or ill-conditioned.
inline bool bvh_build_lights(int n, const float (*P)[3], const float (*x)[3], const float (*y)[3],
                             const float (*inv)[9], const float cam[3], float B, std::vector<BvhNode>& nodes,
                             int* nodes_per_order) {
    std::vector<BvhBox> box(n);
    for (int i = 0; i < n; ++i) {
        double mn = 0.0, in = 0.0, ext = 0.0, pn = 0.0;
        const double cx = (double)x[i][1] * y[i][2] - (double)x[i][2] * y[i][1];
        const double cy = (double)x[i][2] * y[i][0] - (double)x[i][0] * y[i][2];
        const double cz = (double)x[i][0] * y[i][1] - (double)x[i][1] * y[i][0];
        for (int a = 0; a < 3; ++a) {
            mn += (double)x[i][a] * x[i][a] + (double)y[i][a] * y[i][a];
            pn += std::fabs((double)P[i][a]);
            ext += std::fabs((double)x[i][a]) + std::fabs((double)y[i][a]);
        }
        mn += cx * cx + cy * cy + cz * cz;
        for (int k = 0; k < 9; ++k) in += (double)inv[i][k] * inv[i][k];
        const double cond = std::sqrt(mn) * std::sqrt(in);
        if (!std::isfinite(cond) || !std::isfinite(pn + ext) || cond > 1e4) return false;
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            const float c0 = P[i][a], c1 = P[i][a] + x[i][a], c2 = P[i][a] + y[i][a],
                        c3 = P[i][a] + x[i][a] + y[i][a];
            lo[a] = std::min(std::min(c0, c1), std::min(c2, c3));
            hi[a] = std::max(std::max(c0, c1), std::max(c2, c3));
        }
        const double D = origin_bound(cam, B, lo, hi);
        const double pad = 1e-5 * D + 1e-4 * (pn + ext + 1.0) + 1e-5 * cond * ext;
        for (int a = 0; a < 3; ++a) {
            box[i].lo[a] = (float)((double)lo[a] - pad);
            box[i].hi[a] = (float)((double)hi[a] + pad);
        }
    }
    std::vector<int> perm;
    bvh_build_boxes(box, IPT_LBVH_LEAF, false, 1, nodes, perm, nodes_per_order);
    return true;
}

}  // namespace ipt
