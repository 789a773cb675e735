// rt_bvh.h — host-side BVH construction for commit_scene (rt_api.cpp): SAH build over the world-level
// spheres, moving spheres and curves, the BVH2 traversal layout and the BVH4 collapse for the curve walk.
// Host code only (no device code, no HIP): tests/csrc/bvh_check.cpp compiles it with g++ to check the
// threaded build against the serial one.
#pragma once
#include <algorithm>
#include <atomic>
#include <cmath>
#include <limits>
#include <thread>
#include <utility>
#include <vector>

#include <sched.h>

#include "rt_device.h"

namespace rtamd {

// ------------------------------------------------------------------ BVH
// Binned-SAH BVH over the world-level spheres / moving spheres / curves,
// traversed per lane by k_extend (rt_kernels.hip bvh_closest_lane).  Boxes are
// padded outward (relative 1e-8) so culling is conservative and the closest
// hit is exactly the flat list's (geometry.scm:33-50), ties aside.  Moving
// spheres are bounded over every time a ray can carry: camera rays in
// [time0, time1], scattered rays at 0 (Q4, Q13); curves by their control
// points +- width/2 (bezier.scm:88-98).
struct PrimRef { double lo[3], hi[3], c[3]; int leaf; int type; };
// build-time node: inner c = -1, a/b = children, d = split axis; leaf c = -2, refs [a, b)
struct BvhNode { double lo[3], hi[3]; int32_t a, b, c, d; };

// Host threads a scene commit's BVH build may use: the process's CPUs (its affinity mask, which a
// container's cpuset narrows), at most 16 (the GPU box's share per GPU).
inline int build_threads() {
    const unsigned hw = std::thread::hardware_concurrency();
    int n = hw ? (int)hw : 1;
#ifdef CPU_COUNT
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = std::max(1, (int)CPU_COUNT(&set));
#endif
    return std::min(n, 16);
}

// f(b, e) over [0, n) cut into `threads` contiguous ranges, one host thread each (small n: inline)
template <class F>
inline void parallel_for(const size_t n, const int threads, F f) {
    if (threads <= 1 || n < 65536) { f((size_t)0, n); return; }
    const size_t chunk = (n + (size_t)threads - 1) / (size_t)threads;
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) {
        const size_t b = (size_t)t * chunk, e = std::min(n, b + chunk);
        if (b < e) th.emplace_back(f, b, e);
    }
    f((size_t)0, std::min(n, chunk));
    for (std::thread& x : th) x.join();
}

// The builder.  build() appends nodes in depth-first preorder (a node, its left subtree, its right
// subtree); a subtree's shape depends only on its own primitives, which it reorders within its own range
// [b, e) of refs.  So subtrees of at least kGrain primitives can be built by other threads into vectors of
// their own and appended afterwards, with their inner child indices moved by the append offset: the node
// array is the serial build's bit for bit (tests/csrc/bvh_check.cpp compares them).  C5's 2^20 curves:
// 2.8 s on one thread (round 5), the host's threads now (rt_scene_commit).
struct BvhBuild {
    std::vector<PrimRef>& refs;
    std::vector<BvhNode> nodes;
    int leaf_max = 2;                 // RTAMD_BVH_LEAF
    bool singles = false;             // split down to one primitive per leaf even where SAH would stop
    double trav_cost = 0.5;           // node visit cost relative to one primitive test
    int sweep_max = 0;                // RTAMD_BVH_SWEEP: nodes of at most this many primitives use the exact SAH sweep
    int threads = 1;                  // host threads the build may use (build_all)
    static constexpr int kBins = 16;
    static constexpr int kGrain = 2048;   // smallest subtree handed to another thread
    std::atomic<int> live{1};

    static double area(const double* lo, const double* hi) {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (dx < 0 || dy < 0 || dz < 0) return 0.0;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
    // centroid order with NaN last (a degenerate shutter can give NaN boxes): a strict
    // weak ordering, which std::stable_sort / nth_element require
    static bool c_less(const double x, const double y) {
        if (std::isnan(x)) return false;
        return std::isnan(y) || x < y;
    }
    static void grow(double* lo, double* hi, const double* plo, const double* phi) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], plo[k]); hi[k] = std::max(hi[k], phi[k]); }
    }
    // One node over refs [b, e): its box, and either a leaf (returns -1; N.c = -2, N.a / N.b = the range) or a
    // split (returns mid, refs [b, mid) / [mid, e) reordered for the children; N.c = -1, N.d = the axis).
    int decide(int b, int e, int depth, BvhNode& N) {
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        double clo[3] = {1e300, 1e300, 1e300}, chi[3] = {-1e300, -1e300, -1e300};
        for (int i = b; i < e; ++i) { grow(lo, hi, refs[i].lo, refs[i].hi); grow(clo, chi, refs[i].c, refs[i].c); }
        for (int k = 0; k < 3; ++k) { N.lo[k] = lo[k]; N.hi[k] = hi[k]; }
        auto leaf = [&]() { N.a = b; N.b = e; N.c = -2; N.d = 0; return -1; };   // ranges fixed up after the build
        const int n = e - b;
        if (n <= leaf_max || depth >= kLaneStack - 2) return leaf();
        if (n <= sweep_max) {                        // exact SAH: every split position on all three axes
            // each axis's centroid order as the stable sort of [b, e) by c_less gives it: (key, position)
            // pairs sorted by key, then position (the same permutation, without the indirect comparisons)
            int best_axis = -1, best_i = -1;
            double best = 1e300;
            std::vector<std::pair<double, int>> key(n);
            std::vector<int> ord(n), best_ord;
            std::vector<double> right(n + 1);
            for (int ax = 0; ax < 3; ++ax) {
                for (int i = 0; i < n; ++i) key[i] = {refs[b + i].c[ax], b + i};
                std::sort(key.begin(), key.end(), [](const std::pair<double, int>& x, const std::pair<double, int>& y) {
                    return c_less(x.first, y.first) || (!c_less(y.first, x.first) && x.second < y.second);
                });
                for (int i = 0; i < n; ++i) ord[i] = key[i].second;
                double rlo[3] = {1e300, 1e300, 1e300}, rhi[3] = {-1e300, -1e300, -1e300};
                for (int i = n - 1; i >= 1; --i) { grow(rlo, rhi, refs[ord[i]].lo, refs[ord[i]].hi); right[i] = area(rlo, rhi); }
                double llo[3] = {1e300, 1e300, 1e300}, lhi[3] = {-1e300, -1e300, -1e300};
                const int before = best_axis;
                for (int i = 1; i < n; ++i) {        // left = ord[0, i), right = ord[i, n)
                    grow(llo, lhi, refs[ord[i - 1]].lo, refs[ord[i - 1]].hi);
                    const double c = area(llo, lhi) * i + right[i] * (n - i);
                    if (c < best) { best = c; best_axis = ax; best_i = i; }
                }
                if (best_axis != before) best_ord = ord;
            }
            // no finite cost (unbounded / NaN boxes, e.g. a degenerate shutter): the binned path's median split
            if (best_axis >= 0) {
                const double parent = area(lo, hi);
                const bool worth = parent <= 0 || trav_cost + best / parent < (double)n;
                if (!worth && n <= 2 * leaf_max && !singles) return leaf();
                // refs [b, e) in the best axis's order: the stable sort by its centroids
                std::vector<PrimRef> tmp(n);
                for (int i = 0; i < n; ++i) tmp[i] = refs[best_ord[i]];
                std::copy(tmp.begin(), tmp.end(), refs.begin() + b);
                N.c = -1; N.d = best_axis;
                return b + best_i;
            }
        }
        int axis = 0;
        for (int k = 1; k < 3; ++k) if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
        const double ext = chi[axis] - clo[axis];
        int mid = -1;
        if (ext > 0) {
            int cnt[kBins] = {0};
            double blo[kBins][3], bhi[kBins][3];
            for (int k = 0; k < kBins; ++k) for (int j = 0; j < 3; ++j) { blo[k][j] = 1e300; bhi[k][j] = -1e300; }
            auto bin_of = [&](const PrimRef& r) {
                const double f = (r.c[axis] - clo[axis]) / ext * kBins;
                if (!(f >= 0.0)) return 0;                      // NaN centroids go to the first bin
                return f >= (double)kBins ? kBins - 1 : (int)f;
            };
            for (int i = b; i < e; ++i) { const int k = bin_of(refs[i]); cnt[k]++; grow(blo[k], bhi[k], refs[i].lo, refs[i].hi); }
            double best = 1e300;
            int best_k = -1;
            for (int k = 1; k < kBins; ++k) {
                double llo[3] = {1e300, 1e300, 1e300}, lhi[3] = {-1e300, -1e300, -1e300};
                double rlo[3] = {1e300, 1e300, 1e300}, rhi[3] = {-1e300, -1e300, -1e300};
                int nl = 0, nr = 0;
                for (int j = 0; j < k; ++j) if (cnt[j]) { grow(llo, lhi, blo[j], bhi[j]); nl += cnt[j]; }
                for (int j = k; j < kBins; ++j) if (cnt[j]) { grow(rlo, rhi, blo[j], bhi[j]); nr += cnt[j]; }
                if (!nl || !nr) continue;
                const double c = area(llo, lhi) * nl + area(rlo, rhi) * nr;
                if (c < best) { best = c; best_k = k; }
            }
            const double parent = area(lo, hi);
            const bool worth = best_k > 0 && (parent <= 0 || trav_cost + best / parent < (double)n);
            if (!worth && n <= 2 * leaf_max && !singles) return leaf();
            if (best_k > 0) {
                auto it = std::partition(refs.begin() + b, refs.begin() + e,
                                         [&](const PrimRef& r) { return bin_of(r) < best_k; });
                mid = (int)(it - refs.begin());
            }
        }
        if (mid <= b || mid >= e) {                  // degenerate: median split on the axis
            mid = b + n / 2;
            std::nth_element(refs.begin() + b, refs.begin() + mid, refs.begin() + e,
                             [&](const PrimRef& x, const PrimRef& y) { return c_less(x.c[axis], y.c[axis]); });
        }
        N.c = -1; N.d = axis;
        return mid;
    }
    // a thread for a subtree, if the budget allows (live counts the threads building)
    bool take_thread() {
        int v = live.load();
        while (v < threads)
            if (live.compare_exchange_weak(v, v + 1)) return true;
        return false;
    }
    // the subtree over refs [b, e) appended to out in preorder; returns its root's index in out
    int build_into(std::vector<BvhNode>& out, int b, int e, int depth) {
        const int node = (int)out.size();
        out.push_back(BvhNode{});
        BvhNode N{};
        const int mid = decide(b, e, depth, N);
        if (mid >= 0) {
            std::vector<BvhNode> rnodes;
            std::thread th;
            const bool par = threads > 1 && e - mid >= kGrain && take_thread();
            if (par) th = std::thread([&, mid, e, depth]() { build_into(rnodes, mid, e, depth + 1); live.fetch_sub(1); });
            N.a = build_into(out, b, mid, depth + 1);
            if (par) {
                th.join();
                const int off = (int)out.size();         // the right subtree after the left one, as the serial build
                for (BvhNode R : rnodes) {
                    if (R.c == -1) { R.a += off; R.b += off; }
                    out.push_back(R);
                }
                N.b = off;
            } else {
                N.b = build_into(out, mid, e, depth + 1);
            }
        }
        out[node] = N;
        return node;
    }
    // the whole tree over refs [b, e) (root = node 0 of `nodes` for an empty builder)
    int build(int b, int e, int depth) { return build_into(nodes, b, e, depth); }
};

// f64 -> f32 rounded toward -inf / +inf (BVH boxes stay conservative)
inline float f32_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
}
inline float f32_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
}

inline void pad_box(double* lo, double* hi) {
    double m = 1.0;
    for (int k = 0; k < 3; ++k) m = std::max(m, std::max(std::fabs(lo[k]), std::fabs(hi[k])));
    const double pad = 1e-8 * m;
    for (int k = 0; k < 3; ++k) { lo[k] -= pad; hi[k] += pad; }
}

// Nodes of at most this many primitives take the exact SAH split (every
// position on all three axes) instead of 16 bins on the widest axis: sphere
// trees (hundreds of primitives) throughout — C2 extend -2 %, +1.1 % frame
// (profiles/r02/ab/ab_sweep*.log); curve trees (2^20 primitives) keep the
// binned build, whose cost stays linear per level.  RTAMD_BVH_SWEEP overrides.
// Build-time tree -> traversal layout (BvhNode2: both child boxes in the
// parent, f32 rounded outward and widened by `margin`; child refs >= 0 inner,
// < 0 ~leaf).  leaf_of(b, e) gives the BvhLeaf of a build leaf over refs
// [b, e).  lane_stack = deepest BVH2 level (stack entries a traversal needs).
template <class LeafFn>
inline void flatten_bvh2(const std::vector<BvhNode>& nodes, double margin, LeafFn leaf_of, std::vector<BvhNode2>& bvh2,
                  std::vector<BvhLeaf>& bleaf, int32_t& root, int32_t& lane_stack, const int threads = 1) {
    std::vector<int> inner_idx(nodes.size(), -1), leaf_idx(nodes.size(), -1);
    bvh2.reserve(bvh2.size() + nodes.size() / 2 + 1);
    bleaf.reserve(bleaf.size() + nodes.size() / 2 + 1);
    for (size_t i = 0; i < nodes.size(); ++i) {
        const BvhNode& N = nodes[i];
        if (N.c == -1) { inner_idx[i] = (int)bvh2.size(); bvh2.push_back(BvhNode2{}); continue; }
        leaf_idx[i] = (int)bleaf.size();
        bleaf.push_back(leaf_of(N.a, N.b));
    }
    auto ref_of = [&](int i) { return inner_idx[i] >= 0 ? inner_idx[i] : ~leaf_idx[i]; };
    parallel_for(nodes.size(), threads, [&](const size_t b, const size_t e) {    // each node on its own
        for (size_t i = b; i < e; ++i) {
            if (inner_idx[i] < 0) continue;
            BvhNode2& M = bvh2[inner_idx[i]];
            const BvhNode& L = nodes[nodes[i].a];
            const BvhNode& R = nodes[nodes[i].b];
            for (int k = 0; k < 3; ++k) {
                M.b[2 * k] = f32_down(L.lo[k] - margin); M.b[6 + 2 * k] = f32_up(L.hi[k] + margin);
                M.b[2 * k + 1] = f32_down(R.lo[k] - margin); M.b[7 + 2 * k] = f32_up(R.hi[k] + margin);
            }
            M.l = ref_of(nodes[i].a); M.r = ref_of(nodes[i].b);
        }
    });
    root = ref_of(0);
    std::vector<int> depth(nodes.size(), 0);
    for (size_t i = 0; i < nodes.size(); ++i)
        if (nodes[i].c == -1) { depth[nodes[i].a] = depth[i] + 1; depth[nodes[i].b] = depth[i] + 1; }
    for (int dd : depth) lane_stack = std::max(lane_stack, dd);
}

// The BVH4 of a BVH2 (BvhNode4): node p's children, an inner child replaced
// by its own two children with their boxes as the BVH2 stores them.  Returns
// the root ref; stack4 = the most stack entries its walk can hold (a node
// pushes all but the child it enters: the sum of (children - 1) along a path).
inline int32_t collapse_bvh4(const std::vector<BvhNode2>& bvh2, int32_t root, std::vector<BvhNode4>& bvh4, int32_t& stack4) {
    stack4 = 0;
    if (root < 0) return root;
    struct Slot { int32_t ref; float lo[3], hi[3]; };
    auto child = [&](const BvhNode2& M, const int side, Slot& o) {          // side 0 = l, 1 = r
        o.ref = side ? M.r : M.l;
        for (int k = 0; k < 3; ++k) { o.lo[k] = M.b[2 * k + side]; o.hi[k] = M.b[6 + 2 * k + side]; }
    };
    // iterative: (bvh2 node, bvh4 index) pairs still to fill
    std::vector<std::pair<int32_t, int32_t>> todo{{root, 0}};
    std::vector<int32_t> need;                     // per bvh4 node: children - 1
    std::vector<int32_t> parent;                   // per bvh4 node: its parent (-1: the root)
    bvh4.assign(1, BvhNode4{});
    need.assign(1, 0);
    parent.assign(1, -1);
    bvh4.reserve(bvh2.size());
    need.reserve(bvh2.size());
    parent.reserve(bvh2.size());
    while (!todo.empty()) {
        const auto [p, q] = todo.back();
        todo.pop_back();
        Slot sl[4];
        int n = 0;
        for (int side = 0; side < 2; ++side) {
            Slot c;
            child(bvh2[p], side, c);
            if (c.ref >= 0) { child(bvh2[c.ref], 0, sl[n++]); child(bvh2[c.ref], 1, sl[n++]); }
            else sl[n++] = c;
        }
        BvhNode4 N{};
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 3; ++k) { N.lo[k][j] = 0.0f; N.hi[k][j] = -1.0f; }   // empty: never read (j >= n)
        N.n = n;
        for (int j = 0; j < n; ++j) {
            for (int k = 0; k < 3; ++k) { N.lo[k][j] = sl[j].lo[k]; N.hi[k][j] = sl[j].hi[k]; }
            if (sl[j].ref >= 0) {
                const int32_t q2 = (int32_t)bvh4.size();
                bvh4.push_back(BvhNode4{});
                need.push_back(0);
                parent.push_back(q);
                todo.push_back({sl[j].ref, q2});
                N.ref[j] = q2;
            } else {
                N.ref[j] = sl[j].ref;
            }
        }
        for (int j = n; j < 4; ++j) N.ref[j] = sl[0].ref;
        bvh4[q] = N;
        need[q] = n - 1;
    }
    // children were appended after their parents: fold the stack bound bottom-up (deepest child into the parent)
    std::vector<int32_t> deep(bvh4.size(), 0), below(bvh4.size(), 0);
    for (size_t q = bvh4.size(); q-- > 0;) {
        deep[q] = need[q] + below[q];
        if (parent[q] >= 0) below[parent[q]] = std::max(below[parent[q]], deep[q]);
    }
    stack4 = deep[0];
    return 0;
}


}  // namespace rtamd
