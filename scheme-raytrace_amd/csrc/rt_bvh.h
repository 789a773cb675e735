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

// Host record arrays that threads fill after a resize(): an allocator whose value-less construct leaves
// the element uninitialised, so resize() costs no serial zeroing and the pages are first touched by the
// filling threads (C5's curve and leaf records: ~230 MB, 46 ms of zeroing on one thread).
template <class T>
struct NoInit : std::allocator<T> {
    template <class U> struct rebind { using other = NoInit<U>; };
    NoInit() = default;
    template <class U> NoInit(const NoInit<U>&) {}
    template <class U> void construct(U* p) noexcept { ::new ((void*)p) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
template <class T> using HostVec = std::vector<T, NoInit<T>>;

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
    // Sweep nodes keep their centroid orders (round 6): ord[ax][b, e) = the positions of refs [b, e) sorted
    // on axis ax by (centroid, position) — the stable sort's permutation.  A sweep split passes them down:
    // the split axis's order is the children's identity, the other axes' orders split by side in one pass
    // (a filtered sorted list stays sorted), ties re-ordered by their new positions.  So only a sweep node
    // under a binned one sorts; the round-5 build sorted three times at every node (2.8 s of C5's commit).
    std::vector<int32_t> ord[3];

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
    static bool c_same(const double x, const double y) { return !c_less(x, y) && !c_less(y, x); }
    // One node over refs [b, e): its box, and either a leaf (returns -1; N.c = -2, N.a / N.b = the range) or a
    // split (returns mid, refs [b, mid) / [mid, e) reordered for the children; N.c = -1, N.d = the axis).
    // sorted: in, ord[*][b, e) holds the node's orders; out, the children's.
    int decide(int b, int e, int depth, BvhNode& N, bool& sorted) {
        const bool have = sorted;
        sorted = false;
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        double clo[3] = {1e300, 1e300, 1e300}, chi[3] = {-1e300, -1e300, -1e300};
        for (int i = b; i < e; ++i) { grow(lo, hi, refs[i].lo, refs[i].hi); grow(clo, chi, refs[i].c, refs[i].c); }
        for (int k = 0; k < 3; ++k) { N.lo[k] = lo[k]; N.hi[k] = hi[k]; }
        auto leaf = [&]() { N.a = b; N.b = e; N.c = -2; N.d = 0; return -1; };   // ranges fixed up after the build
        const int n = e - b;
        if (n <= leaf_max || depth >= kLaneStack - 2) return leaf();
        if (n <= sweep_max) {                        // exact SAH: every split position on all three axes
            int32_t* o[3] = {ord[0].data() + b, ord[1].data() + b, ord[2].data() + b};
            if (!have) {
                // each axis's centroid order as the stable sort of [b, e) by c_less gives it: (key, position)
                // pairs sorted by key, then position (the same permutation, without the indirect comparisons)
                std::vector<std::pair<double, int>> key(n);
                for (int ax = 0; ax < 3; ++ax) {
                    for (int i = 0; i < n; ++i) key[i] = {refs[b + i].c[ax], b + i};
                    std::sort(key.begin(), key.end(), [](const std::pair<double, int>& x, const std::pair<double, int>& y) {
                        return c_less(x.first, y.first) || (!c_less(y.first, x.first) && x.second < y.second);
                    });
                    for (int i = 0; i < n; ++i) o[ax][i] = key[i].second;
                }
            }
            int best_axis = -1, best_i = -1;
            double best = 1e300;
            thread_local std::vector<double> right;
            right.resize((size_t)n + 1);
            for (int ax = 0; ax < 3; ++ax) {
                const int32_t* od = o[ax];
                double rlo[3] = {1e300, 1e300, 1e300}, rhi[3] = {-1e300, -1e300, -1e300};
                for (int i = n - 1; i >= 1; --i) { grow(rlo, rhi, refs[od[i]].lo, refs[od[i]].hi); right[i] = area(rlo, rhi); }
                double llo[3] = {1e300, 1e300, 1e300}, lhi[3] = {-1e300, -1e300, -1e300};
                for (int i = 1; i < n; ++i) {        // left = od[0, i), right = od[i, n)
                    grow(llo, lhi, refs[od[i - 1]].lo, refs[od[i - 1]].hi);
                    const double c = area(llo, lhi) * i + right[i] * (n - i);
                    if (c < best) { best = c; best_axis = ax; best_i = i; }
                }
            }
            // no finite cost (unbounded / NaN boxes, e.g. a degenerate shutter): the binned path's median split
            if (best_axis >= 0) {
                const double parent = area(lo, hi);
                const bool worth = parent <= 0 || trav_cost + best / parent < (double)n;
                if (!worth && n <= 2 * leaf_max && !singles) return leaf();
                split_orders(b, e, best_axis, b + best_i, o);
                sorted = true;
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
    // refs [b, e) into the split axis's order (the stable sort by its centroids), and the children's orders
    void split_orders(const int b, const int e, const int axis, const int mid, int32_t* const* o) {
        const int n = e - b;
        thread_local std::vector<PrimRef> tmp;
        thread_local std::vector<int32_t> pos, rest;
        tmp.resize((size_t)n); pos.resize((size_t)n); rest.resize((size_t)n);
        const int32_t* os = o[axis];
        for (int i = 0; i < n; ++i) { tmp[i] = refs[os[i]]; pos[os[i] - b] = b + i; }
        std::copy(tmp.begin(), tmp.end(), refs.begin() + b);
        for (int ax = 0; ax < 3; ++ax) {
            if (ax == axis) continue;
            int32_t* oa = o[ax];
            int nl = 0, nr = 0;
            for (int j = 0; j < n; ++j) {            // stable split by side (nl <= j: in place for the left)
                const int32_t p = pos[oa[j] - b];
                if (p < mid) oa[nl++] = p; else rest[nr++] = p;
            }
            std::copy(rest.begin(), rest.begin() + nr, oa + nl);
            for (const auto& [s0, s1] : {std::pair<int, int>{0, nl}, std::pair<int, int>{nl, n}})
                for (int j = s0; j < s1;) {          // runs of equal centroids: by position, as the stable sort
                    int k = j + 1;
                    while (k < s1 && c_same(refs[oa[k]].c[ax], refs[oa[j]].c[ax])) ++k;
                    if (k - j > 1) std::sort(oa + j, oa + k);
                    j = k;
                }
        }
        int32_t* ow = o[axis];
        for (int i = 0; i < n; ++i) ow[i] = b + i;
    }
    // a thread for a subtree, if the budget allows (live counts the threads building)
    bool take_thread() {
        int v = live.load();
        while (v < threads)
            if (live.compare_exchange_weak(v, v + 1)) return true;
        return false;
    }
    // the subtree over refs [b, e) appended to out in preorder; returns its root's index in out
    int build_into(std::vector<BvhNode>& out, int b, int e, int depth, bool sorted) {
        const int node = (int)out.size();
        out.push_back(BvhNode{});
        BvhNode N{};
        const int mid = decide(b, e, depth, N, sorted);
        if (mid >= 0) {
            std::vector<BvhNode> rnodes;
            std::thread th;
            const bool par = threads > 1 && e - mid >= kGrain && take_thread();
            if (par) {
                rnodes.reserve(2 * (size_t)(e - mid));
                th = std::thread([&, mid, e, depth, sorted]() { build_into(rnodes, mid, e, depth + 1, sorted); live.fetch_sub(1); });
            }
            N.a = build_into(out, b, mid, depth + 1, sorted);
            if (par) {
                th.join();
                const int off = (int)out.size();         // the right subtree after the left one, as the serial build
                for (BvhNode R : rnodes) {
                    if (R.c == -1) { R.a += off; R.b += off; }
                    out.push_back(R);
                }
                N.b = off;
            } else {
                N.b = build_into(out, mid, e, depth + 1, sorted);
            }
        }
        out[node] = N;
        return node;
    }
    // the whole tree over refs [b, e) (root = node 0 of `nodes` for an empty builder)
    int build(int b, int e, int depth) {
        if (sweep_max > 0)
            for (auto& v : ord) v.resize(refs.size());
        nodes.reserve(nodes.size() + 2 * (size_t)(e - b));
        return build_into(nodes, b, e, depth, false);
    }
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
template <class LeafFn, class V2, class VL>
inline void flatten_bvh2(const std::vector<BvhNode>& nodes, double margin, LeafFn leaf_of, V2& bvh2, VL& bleaf,
                         int32_t& root, int32_t& lane_stack, const int threads = 1) {
    // inner node i -> bvh2 index = inner nodes before i; leaf i -> bleaf index = leaves before i (counted per
    // thread range, then offset)
    const size_t nn = nodes.size();
    std::vector<int> idx(nn);
    const int nt = (threads > 1 && nn >= 65536) ? threads : 1;
    const size_t chunk = std::max<size_t>(1, (nn + (size_t)nt - 1) / (size_t)nt);
    std::vector<size_t> n_in((size_t)nt + 1, 0), n_lf((size_t)nt + 1, 0);
    // (parallel_for cuts [0, nn) into the same nt ranges of `chunk` nodes: range t starts at t * chunk)
    parallel_for(nn, nt, [&](const size_t b, const size_t e) {
        size_t ni = 0;                                 // (counted locally: the shared counts sit on one line)
        for (size_t i = b; i < e; ++i) ni += nodes[i].c == -1;
        n_in[b / chunk + 1] = ni;
        n_lf[b / chunk + 1] = (e - b) - ni;
    });
    for (int t = 0; t < nt; ++t) { n_in[t + 1] += n_in[t]; n_lf[t + 1] += n_lf[t]; }
    const size_t in0 = bvh2.size(), lf0 = bleaf.size();
    bvh2.resize(in0 + n_in[nt]);
    bleaf.resize(lf0 + n_lf[nt]);
    parallel_for(nn, nt, [&](const size_t b, const size_t e) {
        const size_t t = b / chunk;
        size_t a = in0 + n_in[t], l = lf0 + n_lf[t];
        for (size_t i = b; i < e; ++i) {
            if (nodes[i].c == -1) { idx[i] = (int)a; bvh2[a++] = BvhNode2{}; }
            else { idx[i] = ~(int)l; bleaf[l++] = leaf_of(nodes[i].a, nodes[i].b); }
        }
    });
    parallel_for(nn, threads, [&](const size_t b, const size_t e) {    // each node on its own
        for (size_t i = b; i < e; ++i) {
            if (nodes[i].c != -1) continue;
            BvhNode2& M = bvh2[idx[i]];
            const BvhNode& L = nodes[nodes[i].a];
            const BvhNode& R = nodes[nodes[i].b];
            for (int k = 0; k < 3; ++k) {
                M.b[2 * k] = f32_down(L.lo[k] - margin); M.b[6 + 2 * k] = f32_up(L.hi[k] + margin);
                M.b[2 * k + 1] = f32_down(R.lo[k] - margin); M.b[7 + 2 * k] = f32_up(R.hi[k] + margin);
            }
            M.l = idx[nodes[i].a]; M.r = idx[nodes[i].b];
        }
    });
    root = idx[0];
    std::vector<int> depth(nn, 0);
    for (size_t i = 0; i < nn; ++i)
        if (nodes[i].c == -1) { depth[nodes[i].a] = depth[i] + 1; depth[nodes[i].b] = depth[i] + 1; }
    for (int dd : depth) lane_stack = std::max(lane_stack, dd);
}

// The BVH4 of a BVH2 (BvhNode4): node p's children, an inner child replaced
// by its own two children with their boxes as the BVH2 stores them.  Returns
// the root ref; stack4 = the most stack entries its walk can hold (a node
// pushes all but the child it enters: the sum of (children - 1) along a path).
// Numbering (the round-5 collapse's, which filled the array from a stack): a node's inner children take
// consecutive indices when it is filled, then its subtrees are filled last child first.  With every
// subtree's node count known (pass 1, bottom-up) each subtree's first index follows from its parent's, so
// the subtrees below level kTop are measured and filled on the host threads (round 6: C5's 2^20 curves,
// ~70 ms on one thread).  tests/csrc/bvh_check.cpp compares the array with the stack-order collapse.
template <class V2, class V4>
inline int32_t collapse_bvh4(const V2& bvh2, int32_t root, V4& bvh4, int32_t& stack4, const int threads = 1) {
    stack4 = 0;
    if (root < 0) return root;
    struct Slot { int32_t ref; float lo[3], hi[3]; };
    auto child = [&](const BvhNode2& M, const int side, Slot& o) {          // side 0 = l, 1 = r
        o.ref = side ? M.r : M.l;
        for (int k = 0; k < 3; ++k) { o.lo[k] = M.b[2 * k + side]; o.hi[k] = M.b[6 + 2 * k + side]; }
    };
    auto slots = [&](const int32_t p, Slot* sl) {
        int n = 0;
        for (int side = 0; side < 2; ++side) {
            Slot c;
            child(bvh2[p], side, c);
            if (c.ref >= 0) { child(bvh2[c.ref], 0, sl[n++]); child(bvh2[c.ref], 1, sl[n++]); }
            else sl[n++] = c;
        }
        return n;
    };
    constexpr int kTop = 3;                          // levels above the subtrees the threads take (<= 64 subtrees)
    const bool par = threads > 1 && bvh2.size() >= 65536;
    std::vector<int32_t> size4(bvh2.size()), deep(bvh2.size());    // per BVH2 node heading a BVH4 node
    struct Task { int32_t p, q, start; };
    std::vector<Task> todo;
    // pass 1: subtree node counts and stack bounds; `cut`: stop at level kTop, listing those heads
    auto measure = [&](auto&& self, const int32_t p, const int level, const bool cut) -> void {
        if (cut && level == kTop) { todo.push_back({p, 0, 0}); return; }
        Slot sl[4];
        const int n = slots(p, sl);
        int32_t sz = 1, below = 0;
        for (int j = 0; j < n; ++j)
            if (sl[j].ref >= 0) {
                self(self, sl[j].ref, level + 1, cut);
                sz += size4[sl[j].ref];
                below = std::max(below, deep[sl[j].ref]);
            }
        size4[p] = sz;
        deep[p] = n - 1 + below;
    };
    auto run_tasks = [&](auto&& fn) {
        std::atomic<size_t> next{0};
        auto worker = [&]() { for (size_t t; (t = next.fetch_add(1)) < todo.size();) fn(todo[t]); };
        std::vector<std::thread> th;
        for (int t = 1; t < threads; ++t) th.emplace_back(worker);
        worker();
        for (std::thread& x : th) x.join();
    };
    if (par) {
        measure(measure, root, 0, true);             // lists the level-kTop heads
        run_tasks([&](const Task& t) { measure(measure, t.p, kTop, false); });
        todo.clear();
    }
    measure(measure, root, 0, par);                  // (the listed heads are measured: cut there again)
    todo.clear();
    // pass 2: node q from BVH2 head p; its inner children take start, start + 1, ...; the subtree of inner
    // child t starts at start + k + the node counts (less their heads) of inner children t + 1 .. k - 1
    bvh4.resize((size_t)size4[root]);
    auto fill = [&](auto&& self, const int32_t p, const int32_t q, const int32_t start, const int level, const bool cut) -> void {
        if (cut && level == kTop) { todo.push_back({p, q, start}); return; }
        Slot sl[4];
        const int n = slots(p, sl);
        BvhNode4 N{};
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 3; ++k) { N.lo[k][j] = 0.0f; N.hi[k][j] = -1.0f; }   // empty: never read (j >= n)
        N.n = n;
        int32_t inner[4], kin = 0;
        for (int j = 0; j < n; ++j) {
            for (int k = 0; k < 3; ++k) { N.lo[k][j] = sl[j].lo[k]; N.hi[k][j] = sl[j].hi[k]; }
            if (sl[j].ref >= 0) { inner[kin] = sl[j].ref; N.ref[j] = start + kin; ++kin; }
            else N.ref[j] = sl[j].ref;
        }
        for (int j = n; j < 4; ++j) N.ref[j] = sl[0].ref;
        bvh4[(size_t)q] = N;
        int32_t cs = start + kin;
        for (int t = kin - 1; t >= 0; --t) {
            self(self, inner[t], start + t, cs, level + 1, cut);
            cs += size4[inner[t]] - 1;
        }
    };
    fill(fill, root, 0, 1, 0, par);
    if (par) run_tasks([&](const Task& t) { fill(fill, t.p, t.q, t.start, kTop, false); });
    stack4 = deep[root];
    return 0;
}

}  // namespace rtamd
