// bvh_check.cpp — the threaded scene-commit BVH build (scheme-raytrace_amd/csrc/rt_bvh.h, round 6: key-pair
// sorts in the SAH sweep, centroid orders passed down the sweep, subtrees on host threads, the BVH4 collapse
// numbered from subtree sizes) against the round-5 serial builder (RefBuild below, std::stable_sort sweeps)
// and its stack-order collapse (ref_collapse_bvh4), on the host (no GPU): the same node array bit for bit,
// the same primitive order, the same BVH2 layout and BVH4 array.  Input: a file of n primitives, 7 doubles each (lo[3], hi[3] of the
// unpadded box, type), as commit_scene forms them (curves: control points +- width/2).  Prints one JSON
// line with both build times.  usage: bvh_check FILE THREADS [SWEEP_MAX]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "../../scheme-raytrace_amd/csrc/rt_bvh.h"

using namespace rtamd;

struct RefBuild {     // the round-5 builder: serial, std::stable_sort sweeps (the reference the threaded build must equal)
    std::vector<PrimRef>& refs;
    std::vector<BvhNode> nodes;
    int leaf_max = 2;                 // RTAMD_BVH_LEAF
    bool singles = false;             // split down to one primitive per leaf even where SAH would stop
    double trav_cost = 0.5;           // node visit cost relative to one primitive test
    int sweep_max = 0;                // RTAMD_BVH_SWEEP: nodes of at most this many primitives use the exact SAH sweep
    static constexpr int kBins = 16;

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
    int make_leaf(int node, int b, int e, const double* lo, const double* hi) {
        BvhNode& N = nodes[node];
        for (int k = 0; k < 3; ++k) { N.lo[k] = lo[k]; N.hi[k] = hi[k]; }
        N.a = b; N.b = e; N.c = -2; N.d = 0;        // ranges fixed up after the build
        return node;
    }
    int build(int b, int e, int depth) {
        const int node = (int)nodes.size();
        nodes.push_back(BvhNode{});
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        double clo[3] = {1e300, 1e300, 1e300}, chi[3] = {-1e300, -1e300, -1e300};
        for (int i = b; i < e; ++i) { grow(lo, hi, refs[i].lo, refs[i].hi); grow(clo, chi, refs[i].c, refs[i].c); }
        const int n = e - b;
        if (n <= leaf_max || depth >= kLaneStack - 2) return make_leaf(node, b, e, lo, hi);
        if (n <= sweep_max) {                        // exact SAH: every split position on all three axes
            int best_axis = -1, best_i = -1;
            double best = 1e300;
            std::vector<int> ord(n);
            std::vector<double> right(n + 1);
            for (int ax = 0; ax < 3; ++ax) {
                for (int i = 0; i < n; ++i) ord[i] = b + i;
                std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return c_less(refs[x].c[ax], refs[y].c[ax]); });
                double rlo[3] = {1e300, 1e300, 1e300}, rhi[3] = {-1e300, -1e300, -1e300};
                for (int i = n - 1; i >= 1; --i) { grow(rlo, rhi, refs[ord[i]].lo, refs[ord[i]].hi); right[i] = area(rlo, rhi); }
                double llo[3] = {1e300, 1e300, 1e300}, lhi[3] = {-1e300, -1e300, -1e300};
                for (int i = 1; i < n; ++i) {        // left = ord[0, i), right = ord[i, n)
                    grow(llo, lhi, refs[ord[i - 1]].lo, refs[ord[i - 1]].hi);
                    const double c = area(llo, lhi) * i + right[i] * (n - i);
                    if (c < best) { best = c; best_axis = ax; best_i = i; }
                }
            }
            // no finite cost (unbounded / NaN boxes, e.g. a degenerate shutter): the binned path's median split
            if (best_axis >= 0) {
                const double parent = area(lo, hi);
                const bool worth = parent <= 0 || trav_cost + best / parent < (double)n;
                if (!worth && n <= 2 * leaf_max && !singles) return make_leaf(node, b, e, lo, hi);
                std::stable_sort(refs.begin() + b, refs.begin() + e,
                                 [&](const PrimRef& x, const PrimRef& y) { return c_less(x.c[best_axis], y.c[best_axis]); });
                const int l = build(b, b + best_i, depth + 1);
                const int r = build(b + best_i, e, depth + 1);
                BvhNode& N = nodes[node];
                for (int k = 0; k < 3; ++k) { N.lo[k] = lo[k]; N.hi[k] = hi[k]; }
                N.a = l; N.b = r; N.c = -1; N.d = best_axis;
                return node;
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
            if (!worth && n <= 2 * leaf_max && !singles) return make_leaf(node, b, e, lo, hi);
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
        const int l = build(b, mid, depth + 1);
        const int r = build(mid, e, depth + 1);
        BvhNode& N = nodes[node];
        for (int k = 0; k < 3; ++k) { N.lo[k] = lo[k]; N.hi[k] = hi[k]; }
        N.a = l; N.b = r; N.c = -1; N.d = axis;
        return node;
    }
};

// the round-5 collapse: BVH4 nodes numbered in the order a stack of (BVH2 node, BVH4 index) pairs fills them
static int32_t ref_collapse_bvh4(const std::vector<BvhNode2>& bvh2, int32_t root, std::vector<BvhNode4>& bvh4, int32_t& stack4) {
    stack4 = 0;
    if (root < 0) return root;
    struct Slot { int32_t ref; float lo[3], hi[3]; };
    auto child = [&](const BvhNode2& M, const int side, Slot& o) {
        o.ref = side ? M.r : M.l;
        for (int k = 0; k < 3; ++k) { o.lo[k] = M.b[2 * k + side]; o.hi[k] = M.b[6 + 2 * k + side]; }
    };
    std::vector<std::pair<int32_t, int32_t>> todo{{root, 0}};
    std::vector<int32_t> need(1, 0), parent(1, -1);
    bvh4.assign(1, BvhNode4{});
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
            for (int k = 0; k < 3; ++k) { N.lo[k][j] = 0.0f; N.hi[k][j] = -1.0f; }
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
    std::vector<int32_t> deep(bvh4.size(), 0), below(bvh4.size(), 0);
    for (size_t q = bvh4.size(); q-- > 0;) {
        deep[q] = need[q] + below[q];
        if (parent[q] >= 0) below[parent[q]] = std::max(below[parent[q]], deep[q]);
    }
    stack4 = deep[0];
    return 0;
}

static std::vector<PrimRef> load(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    std::vector<double> v;
    double buf[7];
    while (std::fread(buf, sizeof(double), 7, f) == 7) v.insert(v.end(), buf, buf + 7);
    std::fclose(f);
    std::vector<PrimRef> refs(v.size() / 7);
    for (size_t i = 0; i < refs.size(); ++i) {
        PrimRef& r = refs[i];
        for (int k = 0; k < 3; ++k) { r.lo[k] = v[7 * i + k]; r.hi[k] = v[7 * i + 3 + k]; }
        r.type = (int)v[7 * i + 6];
        r.leaf = (int)i;
        pad_box(r.lo, r.hi);
        for (int k = 0; k < 3; ++k) r.c[k] = 0.5 * (r.lo[k] + r.hi[k]);
    }
    return refs;
}

struct Built { std::vector<BvhNode> nodes; std::vector<int> order; std::vector<BvhNode2> bvh2; std::vector<BvhNode4> bvh4;
               int32_t root = 0, stack = 0, stack4 = 0; double ms = 0; };

template <class B>
static Built run(std::vector<PrimRef> refs, int threads, int sweep) {
    Built o;
    const auto t0 = std::chrono::steady_clock::now();
    B bb{refs, {}};
    bb.leaf_max = 1;
    bb.sweep_max = sweep;
    if constexpr (std::is_same<B, BvhBuild>::value) bb.threads = threads;
    bb.build(0, (int)refs.size(), 0);
    o.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    o.nodes = std::move(bb.nodes);
    for (const PrimRef& r : refs) o.order.push_back(r.leaf);
    std::vector<BvhLeaf> bleaf;
    flatten_bvh2(o.nodes, 1e-6, [&](int b, int e) { return BvhLeaf{b, e - b, 0, 0, 0, 0, 0, 0}; }, o.bvh2, bleaf,
                 o.root, o.stack, std::is_same<B, BvhBuild>::value ? threads : 1);
    if constexpr (std::is_same<B, BvhBuild>::value) collapse_bvh4(o.bvh2, o.root, o.bvh4, o.stack4, threads);
    else ref_collapse_bvh4(o.bvh2, o.root, o.bvh4, o.stack4);
    return o;
}

int main(int argc, char** argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: bvh_check FILE THREADS [SWEEP_MAX]\n"); return 2; }
    const std::vector<PrimRef> refs = load(argv[1]);
    const int threads = std::atoi(argv[2]);
    const int sweep = argc > 3 ? std::atoi(argv[3]) : 1 << 16;
    const Built a = run<RefBuild>(refs, 1, sweep), b = run<BvhBuild>(refs, threads, sweep);
    const bool nodes = a.nodes.size() == b.nodes.size() &&
                       std::memcmp(a.nodes.data(), b.nodes.data(), a.nodes.size() * sizeof(BvhNode)) == 0;
    const bool order = a.order == b.order;
    const bool bvh2 = a.bvh2.size() == b.bvh2.size() &&
                      std::memcmp(a.bvh2.data(), b.bvh2.data(), a.bvh2.size() * sizeof(BvhNode2)) == 0;
    const bool bvh4 = a.bvh4.size() == b.bvh4.size() && a.stack4 == b.stack4 &&
                      std::memcmp(a.bvh4.data(), b.bvh4.data(), a.bvh4.size() * sizeof(BvhNode4)) == 0;
    std::printf("{\"prims\": %zu, \"nodes\": %zu, \"threads\": %d, \"round5_serial_ms\": %.1f, \"threaded_ms\": %.1f, "
                "\"same_nodes\": %d, \"same_order\": %d, \"same_bvh2\": %d, \"same_bvh4\": %d}\n",
                refs.size(), a.nodes.size(), threads, a.ms, b.ms, nodes, order, bvh2, bvh4);
    return nodes && order && bvh2 && bvh4 ? 0 : 1;
}
