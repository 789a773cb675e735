// rt_api.cpp — C ABI (include/rt.h) of librtamd: scene builder, flattening
// of the reference's object tree into grouped leaves, device upload and the
// wavefront driver loop (raygen → [extend → shade/compact]* → accumulate).
#include <hip/hip_runtime.h>
#include <unistd.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/rt.h"
#include "rt_device.h"
#include "rt_bvh.h"

namespace rtamd {
hipError_t launch_raygen(const DevScene&, const RenderParams&, const PathState&, hipStream_t);
hipError_t launch_extend(const DevScene&, const DevScene*, const RenderParams&, const PathState&, const QView&, uint32_t,
                         const HitBuf&, uint32_t, uint32_t*, bool, unsigned int*, const CurveFuse*, hipStream_t);
hipError_t launch_shade(int, const DevScene&, const DevScene*, const RenderParams&, const PathState&, const HitBuf&,
                        const QView&, uint32_t, const PathState&, uint32_t*, uint32_t, uint32_t, hipStream_t);
hipError_t launch_finish(const DevScene&, const DevScene*, const RenderParams&, const PathState&, const QView&, uint32_t,
                         unsigned long long*, size_t, uint32_t, hipStream_t);
hipError_t launch_accumulate(const RenderParams&, uint32_t, double*, hipStream_t);
size_t extend_lds_bytes(const DevScene&);
hipError_t extend_lds_prepare(const DevScene&, size_t, uint32_t*);
size_t camera_lds_bytes(const DevScene&);
hipError_t camera_prepare(const DevScene&, size_t, uint32_t*);
hipError_t launch_camera(const DevScene&, const RenderParams&, const PathState&, uint32_t, const HitBuf&,
                         uint32_t, uint32_t*, size_t, uint32_t, unsigned long long*, hipStream_t);
hipError_t launch_extend_lds(const DevScene&, const RenderParams&, const PathState&, const QView&, uint32_t,
                             const HitBuf&, uint32_t, uint32_t*, uint32_t, unsigned long long*, hipStream_t);
hipError_t launch_resolve_u8(const double*, uint32_t, int, uint8_t*, hipStream_t);
hipError_t launch_scatter_pixels(const double*, const uint32_t*, uint32_t, double*, hipStream_t);
bool curve_persistent();
hipError_t launch_curve_depth(const double*, const double*, uint32_t, int32_t*, hipStream_t);
hipError_t take_fault(uint32_t*);
hipError_t take_curve_stats(unsigned long long out[2]);
hipError_t launch_hit_rays(const DevScene&, const double*, uint32_t, double*, int32_t*, hipStream_t);
hipError_t set_test_caps(int, uint32_t);
}  // namespace rtamd

using namespace rtamd;

namespace {
thread_local std::string g_err;
int fail(const std::string& msg) { g_err = msg; return 1; }

#define HIPCHK(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(std::string(#expr) + ": " + hipGetErrorString(e_));            \
    } while (0)

// ------------------------------------------------------------- objects
enum ObjType { O_SPHERE, O_MSPHERE, O_RECT, O_FLIP, O_BOX, O_TRANSLATE, O_ROTATE_Y, O_LIST, O_BVH, O_BEZIER, O_MEDIUM, O_KLEIN };

struct Obj {
    ObjType type;
    int mat = -1, child = -1, axis = 0;
    std::vector<int> kids;
    double c0[3] = {0, 0, 0}, c1[3] = {0, 0, 0};
    double r = 0, t0 = 0, t1 = 0;
    double a0 = 0, a1 = 0, b0 = 0, b1 = 0, k = 0;
    double sin_t = 0, cos_t = 1;
    double cp[12] = {0};       // O_BEZIER control points a, b, c, d
    double width = 0;
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};


// A lane = one path pool + stream.  render_impl deals the sample chunks of a
// render to the lanes round-robin and keeps them in flight together, so the
// long, narrow tail of one chunk (its last few paths bouncing to depth 100)
// overlaps the wide first iterations of the next one instead of leaving the
// chip mostly idle.  Accumulation stays in chunk (= sample) order.
constexpr int kLanes = 4;                  // most lanes a render may use (RT_OPT_LANES)
constexpr int kCurveLdsStack = RT_CURVE_LDS_STACK;   // k_extend_curves' BVH4 stack entries in LDS per lane
struct Lane {
    DevBuf st_a, st_b, hit, sb, counts, seg_tail;
    uint32_t* h_counts = nullptr;              // pinned survivor counts, one row per iteration
    hipStream_t stream = nullptr;
    hipEvent_t ev_cnt = nullptr;               // the last iteration's survivor counts are on the host
    hipEvent_t ev_acc = nullptr;               // this lane's last accumulate
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};             // profiling: extend / shade brackets
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_fin;      // profiling: tail kernel brackets
    size_t n_fin = 0;
    // the chunk in flight
    enum State { IDLE, RUNNING, DONE } state = IDLE;
    int chunk = -1, depth = 0;
    int index = 0;                             // the lane's position in Context::lanes
    bool fused_camera = false;                 // depth 0 runs k_camera (no raygen pass)
    uint32_t n = 0, S = 0;
    uint64_t seq = 0;                          // enqueue order of the pending iteration
    RenderParams rp{};
    PathState A{}, B{}, *cur = nullptr, *nxt = nullptr;
    QView view{nullptr, 0};
    ~Lane() {
        if (h_counts) (void)hipHostFree(h_counts);
        for (hipEvent_t e : {ev_cnt, ev_acc, ev[0], ev[1], ev[2]}) if (e) (void)hipEventDestroy(e);
        for (auto& pr : ev_fin) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// The frame-end gather's layout for one frame size and world (rt_gather_layout): per rank its shard's
// pixel count and the offset of its pixels in the ranks' concatenated pixel lists (rt_shard_pixels order,
// ranks in order).  The root (rank 0) also keeps that concatenated list on the device and a receive
// buffer for the other ranks' compact accumulators: rank r's lands at doubles recv_at(r).  Both gathers —
// over RCCL (rt_gather_shards) and within one process (rt_gather_shards_local) — fill it the same way and
// place it with the same kernel (gather_place).
struct GatherPlan {
    int nx = -1, ny = -1, world = 0;
    bool root = false;
    std::vector<int64_t> count, off;
    DevBuf pix, recv;
    size_t recv_at(int r) const { return 3 * (size_t)(off[r] - count[0]); }
    int64_t others() const { return off[world - 1] + count[world - 1] - count[0]; }
};

// A context owns the render lanes' path pools: every scene rendered on it
// shares them (the C ABI renders one scene at a time per context), so a
// second scene does not take a second 65 % of device memory.
// The render schedule's knobs are options of the context (rt_context_set_option,
// include/rt.h RT_OPT_*), 0 = the library's automatic choice.
struct Context {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf accum_tmp, img_tmp;
    size_t pool_cap = 0;                       // paths per chunk (max_paths), fixed at the first render
    int pool_lanes = 0;                        // the lanes pool_cap was sized for
    std::unique_ptr<Lane> lanes[kLanes];       // rt_context_release_pools frees them
    int64_t opt_lanes = 0;                     // RT_OPT_LANES (0: 2, or 1 for curve-kernel scenes)
    int64_t opt_max_paths = 0;                 // RT_OPT_MAX_PATHS (0: sized from free memory)
    int64_t opt_tail_paths = 0;                // RT_OPT_TAIL_PATHS (0: 32768)
    int64_t opt_tail_div = 0;                  // RT_OPT_TAIL_DIV (0: 256)
    bool wavefront_only = false;               // RT_OPT_TAIL_OFF: no tail kernel (tests, A/B)
    GatherPlan gplan;                          // rt_gather_shards_local's plan (the frame size last gathered)
    int64_t opt_exact_libm = RT_LIBM_AUTO;     // RT_OPT_EXACT_LIBM: the bounce directions' sin / cos
};

struct Scene {
    int ctx = -1;
    std::vector<DevTexture> texs;
    std::vector<DevMaterial> mats;
    std::vector<Obj> objs;
    double cam[RT_CAMERA_DOUBLES] = {0};
    bool have_cam = false;
    int sky = RT_SKY_GRADIENT;
    int light = -1;                   // rt_set_light_sampling target (-1: off)
    std::vector<double> ranvec;
    std::vector<int32_t> perm;
    bool have_perlin = false;
    bool committed = false;

    // flattened + uploaded
    DevScene dev{};
    DevBuf d_sph, d_msph, d_rect, d_bez, d_klein, d_med, d_bgroups, d_groups, d_chains, d_leaves, d_mats, d_texs, d_ranvec, d_perm, d_bvh2, d_bleaf;
    DevBuf d_fbvh2, d_fbleaf, d_fsph, d_fid;      // time-0 BVH (commit_scene)
    DevBuf d_bvh4, d_stk_ovf, d_bez_ring, d_fuse_ring;         // curve trees: BVH4, the walk's stack overflow, rings
    DevBuf d_dev;                                  // a device copy of `dev` (kernels that take the scene by pointer)
    DevBuf d_leaf_cls;
    size_t ext_lds = 0;                            // k_extend_lds: LDS bytes (0 = not used) and grid cap
    uint32_t ext_lds_blocks = 0;
    size_t cam_lds = 0;                            // k_camera (fused raygen + depth-0 extend), same
    uint32_t cam_blocks = 0;
    // render buffers (the lanes' path pools belong to the context)
    DevBuf pixlist;
    int pix_nx = -1, pix_ny = -1, pix_y0 = -1, pix_y1 = -1, pix_shard = -1, pix_nshard = -1;
    uint32_t pix_n = 0;
    bool profiling = false;
    rt_stats stats{};
    double commit_ms = 0.0, commit_upload_ms = 0.0;   // rt_scene_commit: wall time, of it device allocation + copies
    double commit_sah_ms = 0.0;                        // ... and the SAH builds (commit_threads host threads)
    int commit_threads = 1;
};

// A multi-GPU frame's communicator (rt_comm_create): one RCCL rank per process, bound to a context's
// device.  The gather's plan is kept for the frame size last gathered.
struct Comm {
    int ctx = -1, rank = 0, world = 1;
    int device = 0;
    ncclComm_t nc = nullptr;
    GatherPlan plan;
    ~Comm() { if (nc) (void)ncclCommDestroy(nc); }
};

std::mutex g_mu;
std::map<int, std::unique_ptr<Context>> g_ctx;
std::map<int, std::unique_ptr<Scene>> g_scene;
// shared: rt_gather_shards keeps its communicator alive outside the lock (it waits for the other ranks)
std::map<int, std::shared_ptr<Comm>> g_comm;
int g_next_ctx = 1, g_next_scene = 1, g_next_comm = 1;

Context* get_ctx(int h) {
    auto it = g_ctx.find(h);
    return it == g_ctx.end() ? nullptr : it->second.get();
}
Scene* get_scene(int h) {
    auto it = g_scene.find(h);
    return it == g_scene.end() ? nullptr : it->second.get();
}

#define SCENE_OR_FAIL(s, h)                                                     \
    std::lock_guard<std::mutex> lk_(g_mu);                                      \
    Scene* s = get_scene(h);                                                    \
    if (!s) return fail("invalid scene handle " + std::to_string(h));            \
    if (s->committed) return fail("scene " + std::to_string(h) + " already committed");

int check_tex(Scene* s, int t) {
    if (t < 0 || t >= (int)s->texs.size()) return fail("invalid texture id " + std::to_string(t));
    return 0;
}
int check_mat(Scene* s, int m) {
    if (m < 0 || m >= (int)s->mats.size()) return fail("invalid material id " + std::to_string(m));
    return 0;
}
int check_obj(Scene* s, int o) {
    if (o < 0 || o >= (int)s->objs.size()) return fail("invalid object id " + std::to_string(o));
    return 0;
}

// --------------------------------------------------------- flattening
struct LeafTmp {
    int type;          // LeafType
    int chain;         // -1 = world
    int flip;
    int obj;           // source object
    int aux = -1;      // LEAF_MEDIUM: index into Flattener::bounds
};

struct Flattener {
    Scene* s;
    std::vector<std::vector<ChainOpRec>> chains;   // unique chains
    std::vector<LeafTmp> leaves;                   // DFS order
    std::vector<std::vector<LeafTmp>> bounds;      // per constant medium: its boundary's leaves
    std::vector<ChainOpRec> cur;
    int depth_guard = 0;
    bool in_boundary = false;

    int chain_id() {
        if (cur.empty()) return -1;
        for (size_t i = 0; i < chains.size(); ++i) {
            if (chains[i].size() == cur.size() &&
                std::memcmp(chains[i].data(), cur.data(), cur.size() * sizeof(ChainOpRec)) == 0)
                return (int)i;
        }
        chains.push_back(cur);
        return (int)chains.size() - 1;
    }
    int walk(int id, int flip) {
        if (++depth_guard > 10000) return fail("object graph too deep (cycle?)");
        const Obj& o = s->objs[id];
        int rc = 0;
        switch (o.type) {
        case O_SPHERE: leaves.push_back({LEAF_SPHERE, chain_id(), flip, id}); break;
        case O_MSPHERE: leaves.push_back({LEAF_MSPHERE, chain_id(), flip, id}); break;
        case O_RECT: leaves.push_back({LEAF_RECT_XY + o.axis, chain_id(), flip, id}); break;
        case O_BEZIER:
            if (in_boundary) return fail("a constant medium's boundary may hold spheres, rects, boxes and instances only");
            leaves.push_back({LEAF_BEZIER, chain_id(), flip, id});
            break;
        case O_KLEIN:
            if (in_boundary) return fail("a constant medium's boundary may hold spheres, rects, boxes and instances only");
            leaves.push_back({LEAF_KLEIN, chain_id(), flip, id});
            break;
        case O_MEDIUM: {
            if (in_boundary) return fail("constant media cannot be nested");
            std::vector<LeafTmp> saved;
            saved.swap(leaves);
            in_boundary = true;
            rc = walk(o.child, 0);
            in_boundary = false;
            std::vector<LeafTmp> b;
            b.swap(leaves);
            leaves.swap(saved);
            if (rc) break;
            bounds.push_back(std::move(b));
            LeafTmp L{LEAF_MEDIUM, chain_id(), flip, id};
            L.aux = (int)bounds.size() - 1;
            leaves.push_back(L);
            break;
        }
        case O_FLIP: rc = walk(o.child, flip ^ 1); break;
        case O_BOX:
        case O_LIST:
        case O_BVH:
            for (int k : o.kids) { if ((rc = walk(k, flip))) break; }
            break;
        case O_TRANSLATE:
        case O_ROTATE_Y: {
            if ((int)cur.size() >= kMaxChain) return fail("instance nesting deeper than 4 transforms");
            ChainOpRec op{};
            if (o.type == O_TRANSLATE) { op.op = OP_TRANSLATE; op.x = o.c0[0]; op.y = o.c0[1]; op.z = o.c0[2]; }
            else { op.op = OP_ROTATE_Y; op.x = o.sin_t; op.y = o.cos_t; op.z = 0; }
            cur.push_back(op);
            rc = walk(o.child, flip);
            cur.pop_back();
            break;
        }
        }
        --depth_guard;
        return rc;
    }
};

int bvh_sweep_max(const bool curves) {
    const char* e = std::getenv("RTAMD_BVH_SWEEP");
    return e ? std::atoi(e) : (curves ? 0 : 1 << 16);
}

size_t bvh_min_prims() {
    const char* e = std::getenv("RTAMD_BVH_MIN");
    return e ? (size_t)std::strtoull(e, nullptr, 10) : 16;
}

// device time commit_scene spends in upload() (allocation + copy), for rt_scene_info's split of the
// commit into host build and device upload
thread_local double tl_upload_ms = 0.0;
template <class T, class A>
int upload(DevBuf& b, const std::vector<T, A>& v, const T** out) {
    const auto t0 = std::chrono::steady_clock::now();
    size_t n = std::max<size_t>(1, v.size()) * sizeof(T);
    HIPCHK(b.ensure(n));
    if (!v.empty()) HIPCHK(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = b.as<const T>();
    tl_upload_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

// An L2 bound on the world-space distance from the origin of every point a
// ray can start from: all leaves (instance chains applied: rotations keep the
// norm, translations add theirs), medium boundaries, the camera; x4 for the
// off-surface points curves report (Q10) and motion extrapolation.
double scene_radius(const Scene* s, const Flattener& f) {
    auto n3 = [](const double* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); };
    auto chain_len = [&](int ch) {
        double t = 0;
        if (ch >= 0)
            for (const ChainOpRec& op : f.chains[ch])
                if (op.op == OP_TRANSLATE) t += std::sqrt(op.x * op.x + op.y * op.y + op.z * op.z);
        return t;
    };
    auto leaf_r = [&](const LeafTmp& L) {
        const Obj& o = s->objs[L.obj];
        double r = 0;
        switch (L.type) {
        case LEAF_SPHERE: r = n3(o.c0) + std::fabs(o.r); break;
        case LEAF_MSPHERE: r = 2 * std::max(n3(o.c0), n3(o.c1)) + std::fabs(o.r); break;
        case LEAF_BEZIER:
            for (int i = 0; i < 4; ++i) r = std::max(r, n3(o.cp + 3 * i));
            r += std::fabs(o.width);
            break;
        case LEAF_KLEIN: r = n3(o.c0) + 1200; break;
        case LEAF_MEDIUM: r = 0; break;
        default:
            r = std::sqrt(3.0) * std::max({std::fabs(o.a0), std::fabs(o.a1), std::fabs(o.b0), std::fabs(o.b1),
                                           std::fabs(o.k)});
        }
        return r + chain_len(L.chain);
    };
    double R = n3(s->cam + 9) + std::fabs(s->cam[21]);
    const int nt = build_threads();
    std::vector<double> part((size_t)nt, R);        // (max is order-free: a NaN radius never enters)
    parallel_for(f.leaves.size(), nt, [&](const size_t b, const size_t e) {
        double r = R;
        for (size_t i = b; i < e; ++i) r = std::max(r, leaf_r(f.leaves[i]));
        part[b / std::max<size_t>(1, (f.leaves.size() + (size_t)nt - 1) / (size_t)nt)] = r;
    });
    for (const double r : part) R = std::max(R, r);
    for (const auto& b : f.bounds) for (const LeafTmp& L : b) R = std::max(R, leaf_r(L));
    return 4 * R + 1;
}

size_t extend_lds_budget() { return (size_t)64 << 10; }   // largest LDS footprint k_extend_lds may take

// A commit's host scratch (C5: ~0.7 GB of build arrays) takes ~65 ms to unmap on one thread; the commit
// hands it to this worker instead and returns as soon as the device scene is ready.  The worker drains its
// queue before the library unloads.  A forked child inherits the object but not the thread: it starts its
// own and leaves the parent's alone (joining a thread of another process would hang).
class Reaper {
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<std::shared_ptr<void>> q_;
    bool stop_ = false;
    std::thread* th_ = nullptr;
    pid_t pid_ = 0;
    void run() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
            std::vector<std::shared_ptr<void>> batch;
            batch.swap(q_);
            lk.unlock();
            batch.clear();                              // the frees, outside the lock
            lk.lock();
            if (stop_ && q_.empty()) return;
        }
    }
public:
    template <class... V>
    void reap(V&&... v) {
        auto bundle = std::make_shared<std::tuple<std::decay_t<V>...>>(std::move(v)...);
        std::lock_guard<std::mutex> lk(mu_);
        if (!th_ || pid_ != getpid()) {
            th_ = new std::thread([this] { run(); });   // (a parent's thread object stays with the parent)
            pid_ = getpid();
        }
        q_.push_back(std::move(bundle));
        cv_.notify_one();
    }
    ~Reaper() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_one();
        if (th_ && pid_ == getpid()) {
            th_->join();
            delete th_;
        }
    }
};
Reaper g_reaper;

#ifdef RT_COMMIT_PROFILE
#define COMMIT_MARK(tag) std::fprintf(stderr, "commit %-12s %9.1f ms\n", tag, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - cp0).count())
#else
#define COMMIT_MARK(tag) ((void)0)
#endif
int commit_scene(Scene* s, int world) {
#ifdef RT_COMMIT_PROFILE
    const auto cp0 = std::chrono::steady_clock::now();
#endif
    Context* c = get_ctx(s->ctx);
    if (!c) return fail("scene's context was destroyed");
    HIPCHK(hipSetDevice(c->device));
    if (!s->have_cam) return fail("rt_scene_commit: no camera set (rt_set_camera)");
    for (const auto& t : s->texs)
        if ((t.type == TEX_NOISE || t.type == TEX_MARBLE) && !s->have_perlin)
            return fail("rt_scene_commit: noise/marble texture needs rt_set_perlin_tables");
    Flattener f{s};
    f.leaves.reserve(s->objs.size());                // (a hint: an object listed twice is two leaves)
    if (int rc = f.walk(world, 0)) return rc;

    // group leaves by (chain, type) in first-appearance order of chains
    std::vector<int> chain_order;   // -1 first
    chain_order.push_back(-1);
    for (size_t i = 0; i < f.chains.size(); ++i) chain_order.push_back((int)i);
    HostVec<SphereRec> sph;                          // (filled by threads after a resize: rt_bvh.h, NoInit)
    HostVec<MSphereRec> msph;
    std::vector<RectRec> rect;
    std::vector<Group> groups;
    HostVec<LeafInfo> lsph, lmsph;
    std::vector<LeafInfo> lrect[3];

    HostVec<BezierRec> bez;
    HostVec<LeafInfo> lbez;
    std::vector<KleinRec> klein;
    std::vector<LeafInfo> lklein;
    auto bezier_rec = [](const Obj& o) {
        BezierRec b{};
        for (int k = 0; k < 12; ++k) b.cp[k] = o.cp[k];
        b.w1 = o.width / 2;                 // bezier.scm:63-65
        b.w2 = b.w1 * b.w1;
        b.eps8 = 8 * (o.width / 20);
        return b;
    };

    // A constant medium draws a random number inside its hit test, so its
    // position in the object list matters (the draw happens only if the
    // closest hit so far leaves part of its span): the leaves are cut into
    // segments at each medium and evaluated segment by segment, each medium
    // right after the objects that precede it.  Within a segment the order of
    // the other primitives does not change the closest hit.
    std::vector<int> seg(f.leaves.size(), 0);
    int nseg = 1;
    for (size_t i = 0; i < f.leaves.size(); ++i) {
        seg[i] = nseg - 1;
        if (f.leaves[i].type == LEAF_MEDIUM) ++nseg;
    }

    // BVH over the world-level (chain -1) spheres, moving spheres and curves of segment 0
    COMMIT_MARK("flatten");
    const int threads = build_threads();
    std::vector<int> in_bvh;                         // the leaves the BVH takes, in list order
    for (size_t i = 0; i < f.leaves.size(); ++i) {
        const LeafTmp& L = f.leaves[i];
        if (seg[i] == 0 && L.chain == -1 && (L.type == LEAF_SPHERE || L.type == LEAF_MSPHERE || L.type == LEAF_BEZIER))
            in_bvh.push_back((int)i);
    }
    std::vector<PrimRef> refs(in_bvh.size());
    parallel_for(in_bvh.size(), threads, [&](const size_t jb, const size_t je) {
      for (size_t j = jb; j < je; ++j) {
        const size_t i = (size_t)in_bvh[j];
        const LeafTmp& L = f.leaves[i];
        const Obj& o = s->objs[L.obj];
        PrimRef r{};
        r.leaf = (int)i;
        r.type = L.type;
        const double rad = std::fabs(o.r);
        if (L.type == LEAF_SPHERE) {
            for (int k = 0; k < 3; ++k) { r.lo[k] = o.c0[k] - rad; r.hi[k] = o.c0[k] + rad; }
        } else if (L.type == LEAF_BEZIER) {
            const double w1 = std::fabs(o.width / 2);
            for (int k = 0; k < 3; ++k) {
                r.lo[k] = std::min(std::min(o.cp[k], o.cp[3 + k]), std::min(o.cp[6 + k], o.cp[9 + k])) - w1;
                r.hi[k] = std::max(std::max(o.cp[k], o.cp[3 + k]), std::max(o.cp[6 + k], o.cp[9 + k])) + w1;
            }
        } else {
            const double den = o.t1 - o.t0;
            const double ct0 = s->cam[22], ct1 = s->cam[23];
            const double tlo = std::min(std::min(ct0, ct1), 0.0), thi = std::max(std::max(ct0, ct1), 0.0);
            if (!(den != 0.0) || !std::isfinite(den)) {
                for (int k = 0; k < 3; ++k) { r.lo[k] = -1e300; r.hi[k] = 1e300; }
            } else {
                const double f0 = (tlo - o.t0) / den, f1 = (thi - o.t0) / den;
                for (int k = 0; k < 3; ++k) {
                    const double dc = o.c1[k] - o.c0[k];
                    const double a = o.c0[k] + dc * f0, b = o.c0[k] + dc * f1;
                    r.lo[k] = std::min(a, b) - rad; r.hi[k] = std::max(a, b) + rad;
                }
            }
        }
        pad_box(r.lo, r.hi);
        for (int k = 0; k < 3; ++k) r.c[k] = 0.5 * (r.lo[k] + r.hi[k]);
        refs[j] = r;
      }
    });
    COMMIT_MARK("refs");
    const bool use_bvh = !refs.empty() && refs.size() >= bvh_min_prims();
    std::vector<BvhNode> bvh_nodes;
    HostVec<BvhNode2> bvh2;
    HostVec<BvhLeaf> bleaf;
    int32_t bvh2_root = 0;
    int32_t lane_stack = 0;
    HostVec<BvhNode4> bvh4;                          // curve trees (k_extend_curves)
    int32_t bvh4_root = 0, stack4 = 0;
    bool bvh_has_bez = false;
    float bvh_pad = 0.0f;
    double margin = 0.0;
    HostVec<BvhNode2> fbvh2;                         // time-0 tree (see below)
    HostVec<BvhLeaf> fbleaf;
    std::vector<SphereRec> fsph;
    std::vector<std::pair<int, int>> fsrc;           // (LEAF_SPHERE | LEAF_MSPHERE, local)
    int32_t fbvh2_root = 0;
    bool tree0_any_time = false;
    bool tree0_direct = false;
    if (use_bvh) {
        BvhBuild bb{refs, {}};
        // one primitive per leaf (measured fastest for sphere trees; for C5's curve tree, with the exact
        // SAH sweep below 65 536 primitives, +1.5 % / +0.6 % over two per leaf: profiles/r02/ab_c5,
        // profiles/r03/c5walk/ab_leaf1.log)
        bb.leaf_max = 1;
        bb.sweep_max = bvh_sweep_max(bb.leaf_max > 1 &&
                                     std::any_of(refs.begin(), refs.end(), [](const PrimRef& r) { return r.type == LEAF_BEZIER; }));
        bb.threads = threads;
        s->commit_threads = bb.threads;
        const auto ts = std::chrono::steady_clock::now();
        bb.build(0, (int)refs.size(), 0);
        s->commit_sah_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
        COMMIT_MARK("sah");
        // leaf ranges: refs order -> sphere / moving-sphere / curve array indices
        std::vector<int> ns(refs.size() + 1, 0), nm(refs.size() + 1, 0), nb(refs.size() + 1, 0);
        for (size_t i = 0; i < refs.size(); ++i) {
            ns[i + 1] = ns[i] + (refs[i].type == LEAF_SPHERE);
            nm[i + 1] = nm[i] + (refs[i].type == LEAF_MSPHERE);
            nb[i + 1] = nb[i] + (refs[i].type == LEAF_BEZIER);
        }
        bvh_has_bez = nb[refs.size()] > 0;
        bvh_nodes = std::move(bb.nodes);
        COMMIT_MARK("prefix");
        // f32 box margin: 2^-21 x a radius bound R on everything a ray can start
        // from (x4 included, see scene_radius).  The slab ends carry at most
        // ~4 ulps x (|box| + |o|) <= 2^-22 x 1.25 R of rounding; the margin is
        // 1.6x that.
        margin = std::ldexp(scene_radius(s, f), -21);
        bvh_pad = (float)margin;
        COMMIT_MARK("radius");
        flatten_bvh2(bvh_nodes, margin, [&](int b, int e) {
            return BvhLeaf{ns[b], ns[e] - ns[b], nm[b], nm[e] - nm[b], nb[b], nb[e] - nb[b], 0, 0};
        }, bvh2, bleaf, bvh2_root, lane_stack, threads);
        COMMIT_MARK("flatten2");
        if (bvh_has_bez) {                               // single-curve leaves: direct refs (kDirectCurve)
            auto direct = [&](int32_t& ref) {
                if (ref >= 0) return;
                const BvhLeaf& L = bleaf[~ref];
                if (L.sn == 0 && L.mn == 0 && L.bn == 1 && L.bb < kDirectCurve) ref = ~(kDirectCurve + L.bb);
            };
            for (BvhNode2& M : bvh2) { direct(M.l); direct(M.r); }
            direct(bvh2_root);
            COMMIT_MARK("bvh2");
            bvh4_root = collapse_bvh4(bvh2, bvh2_root, bvh4, stack4, threads);
            COMMIT_MARK("bvh4");
        }
        groups.push_back(Group{GROUP_BVH, -1, 0, (int)bvh_nodes.size()});
        // records in refs order: ref i is sphere ns[i] / moving sphere nm[i] / curve nb[i] of its type's
        // arrays (the prefix counts above), so the refs fill them independently, on the build's threads
        sph.resize((size_t)ns[refs.size()]); lsph.resize(sph.size());
        msph.resize((size_t)nm[refs.size()]); lmsph.resize(msph.size());
        bez.resize((size_t)nb[refs.size()]); lbez.resize(bez.size());
        COMMIT_MARK("resize");
        parallel_for(refs.size(), bb.threads, [&](const size_t b, const size_t e) {
            for (size_t i = b; i < e; ++i) {
                const PrimRef& r = refs[i];
                const LeafTmp& L = f.leaves[r.leaf];
                const Obj& o = s->objs[L.obj];
                LeafInfo li{};
                li.type = L.type; li.chain = -1; li.mat = o.mat; li.flip = L.flip;
                if (r.type == LEAF_SPHERE) {
                    li.inv_r = 1.0 / o.r;
                    li.local = ns[i];
                    sph[(size_t)ns[i]] = SphereRec{o.c0[0], o.c0[1], o.c0[2], o.r * o.r};
                    lsph[(size_t)ns[i]] = li;
                } else if (r.type == LEAF_MSPHERE) {
                    li.inv_r = 1.0 / o.r;
                    li.local = nm[i];
                    MSphereRec m{};
                    m.c0x = o.c0[0]; m.c0y = o.c0[1]; m.c0z = o.c0[2]; m.rr = o.r * o.r;
                    m.dcx = o.c1[0] - o.c0[0]; m.dcy = o.c1[1] - o.c0[1]; m.dcz = o.c1[2] - o.c0[2];
                    m.t0 = o.t0; m.den = o.t1 - o.t0;
                    msph[(size_t)nm[i]] = m;
                    lmsph[(size_t)nm[i]] = li;
                } else {
                    li.local = nb[i];
                    bez[(size_t)nb[i]] = bezier_rec(o);
                    bez[(size_t)nb[i]].order = (uint32_t)r.leaf;      // the flattened list position
                    lbez[(size_t)nb[i]] = li;
                }
            }
        });
        // Time-0 BVH.  Every scattered ray has time 0 (make-ray, ray.scm:8-9,
        // Q4), so for those rays a moving sphere sits at center(0) exactly:
        // the second tree bounds each moving sphere at that one position
        // instead of over the whole shutter, and stores it as a plain sphere
        // whose center is computed here with the kernel's own operations
        // (c0 + dc * ((0 - t0) / den), IEEE f64, no contraction), so the
        // primitive test it runs is bit-for-bit the moving-sphere test.
        // (Built for every sphere tree: with no moving spheres it equals the
        // all-times tree and serves every ray, tree0_any_time.)
        tree0_any_time = nm[refs.size()] == 0;
        if (!bvh_has_bez && !std::getenv("RTAMD_NO_BVH0")) {
            std::vector<PrimRef> refs0;
            for (size_t i = 0; i < refs.size(); ++i) {
                PrimRef r = refs[i];
                r.leaf = (int)i;                     // index into refs (-> fsph / fid below)
                if (r.type == LEAF_MSPHERE) {
                    const MSphereRec& m = msph[(size_t)nm[i]];
                    const double frac = (0.0 - m.t0) / m.den;
                    const double c[3] = {m.c0x + m.dcx * frac, m.c0y + m.dcy * frac, m.c0z + m.dcz * frac};
                    const double rad = std::sqrt(m.rr) * (1 + 1e-15) + 1e-300;
                    const bool fin = std::isfinite(c[0]) && std::isfinite(c[1]) && std::isfinite(c[2]);
                    for (int k = 0; k < 3; ++k) {
                        r.lo[k] = fin ? c[k] - rad : -1e300;
                        r.hi[k] = fin ? c[k] + rad : 1e300;
                    }
                    pad_box(r.lo, r.hi);
                    for (int k = 0; k < 3; ++k) r.c[k] = 0.5 * (r.lo[k] + r.hi[k]);
                }
                refs0.push_back(r);
            }
            BvhBuild b0{refs0, {}};
            b0.leaf_max = bb.leaf_max;
            b0.trav_cost = bb.trav_cost;
            b0.sweep_max = bb.sweep_max;
            b0.singles = b0.leaf_max == 1;           // direct leaves (below) need one sphere per leaf
            b0.threads = bb.threads;
            const auto t0s = std::chrono::steady_clock::now();
            b0.build(0, (int)refs0.size(), 0);
            s->commit_sah_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0s).count();
            // fsph in refs0 order; each entry remembers which sphere / moving sphere it is
            for (const PrimRef& r : refs0) {
                const size_t i = (size_t)r.leaf;
                if (r.type == LEAF_SPHERE) {
                    fsph.push_back(sph[(size_t)ns[i]]);
                    fsrc.push_back({LEAF_SPHERE, ns[i]});
                } else {
                    const MSphereRec& m = msph[(size_t)nm[i]];
                    const double frac = (0.0 - m.t0) / m.den;
                    fsph.push_back({m.c0x + m.dcx * frac, m.c0y + m.dcy * frac, m.c0z + m.dcz * frac, m.rr});
                    fsrc.push_back({LEAF_MSPHERE, nm[i]});
                }
            }
            flatten_bvh2(b0.nodes, margin, [&](int b, int e) { return BvhLeaf{b, e - b, 0, 0, 0, 0, 0, 0}; },
                         fbvh2, fbleaf, fbvh2_root, lane_stack);
            // Direct leaves: when every time-0 leaf holds exactly one sphere, put
            // fsph (and its leaf-id map) in leaf order, so leaf k is sphere k and
            // the SOLO LDS kernels need no leaf records (DevScene::bvh_solo).
            tree0_direct = std::all_of(fbleaf.begin(), fbleaf.end(), [](const BvhLeaf& L) { return L.sn == 1; });
            if (tree0_direct) {
                std::vector<SphereRec> fs2(fbleaf.size());
                std::vector<std::pair<int, int>> src2(fbleaf.size());
                for (size_t k = 0; k < fbleaf.size(); ++k) {
                    fs2[k] = fsph[(size_t)fbleaf[k].sb];
                    src2[k] = fsrc[(size_t)fbleaf[k].sb];
                    fbleaf[k].sb = (int32_t)k;
                }
                fsph.swap(fs2);
                fsrc.swap(src2);
            }
        }
    }
    COMMIT_MARK("records");
    std::vector<MediumRec> med;
    std::vector<LeafInfo> lmed;
    std::vector<Group> bgroups;
    // records of one leaf.  Leaf id = leaf_base[type] + index in the type's
    // record array, so every record gets a LeafInfo; boundary leaves (never a
    // closest hit) get a placeholder.
    auto add_record = [&](const LeafTmp& L, LeafInfo* li_world) {
        const Obj& o = s->objs[L.obj];
        LeafInfo placeholder{};
        placeholder.type = L.type; placeholder.chain = -1; placeholder.mat = 0;
        LeafInfo* li = li_world ? li_world : &placeholder;
        if (L.type == LEAF_SPHERE) {
            li->local = (int)sph.size(); li->inv_r = 1.0 / o.r;  lsph.push_back(*li);
            sph.push_back({o.c0[0], o.c0[1], o.c0[2], o.r * o.r});
        } else if (L.type == LEAF_MSPHERE) {
            MSphereRec m{};
            m.c0x = o.c0[0]; m.c0y = o.c0[1]; m.c0z = o.c0[2]; m.rr = o.r * o.r;
            m.dcx = o.c1[0] - o.c0[0]; m.dcy = o.c1[1] - o.c0[1]; m.dcz = o.c1[2] - o.c0[2];
            m.t0 = o.t0; m.den = o.t1 - o.t0;
            li->local = (int)msph.size(); li->inv_r = 1.0 / o.r;  lmsph.push_back(*li);
            msph.push_back(m);
        } else if (L.type == LEAF_BEZIER) {
            li->local = (int)bez.size(); lbez.push_back(*li);
            bez.push_back(bezier_rec(o));
            {   // the flattened list position (medium boundaries come from f.bounds: order 0, ties irrelevant)
                const uintptr_t p = reinterpret_cast<uintptr_t>(&L), b0 = reinterpret_cast<uintptr_t>(f.leaves.data());
                const bool in_list = p >= b0 && p < b0 + f.leaves.size() * sizeof(LeafTmp);
                bez.back().order = in_list ? (uint32_t)((p - b0) / sizeof(LeafTmp)) : 0u;
            }
        } else if (L.type == LEAF_KLEIN) {
            li->local = (int)klein.size(); lklein.push_back(*li);
            klein.push_back({o.c0[0], o.c0[1], o.c0[2], 0.0});
        } else {
            RectRec r{};
            r.a0 = o.a0; r.a1 = o.a1; r.b0 = o.b0; r.b1 = o.b1; r.k = o.k;
            li->local = (int)rect.size(); lrect[L.type - LEAF_RECT_XY].push_back(*li);
            rect.push_back(r);
        }
    };
    auto type_size = [&](int type) {
        return (type == LEAF_SPHERE) ? sph.size() : (type == LEAF_MSPHERE) ? msph.size()
             : (type == LEAF_BEZIER) ? bez.size() : (type == LEAF_KLEIN) ? klein.size() : rect.size();
    };
    // group a leaf subset by (chain, type) into `out`; world leaves also get LeafInfo
    auto emit_groups = [&](const std::vector<const LeafTmp*>& ls, std::vector<Group>& out, bool world, bool skip_bvh) {
        for (int ch : chain_order) {
            for (int type = LEAF_SPHERE; type <= LEAF_KLEIN; ++type) {
                if (type == LEAF_MEDIUM) continue;
                if (skip_bvh && ch == -1 && (type == LEAF_SPHERE || type == LEAF_MSPHERE || type == LEAF_BEZIER)) continue;
                Group g{type, ch, 0, 0};
                const size_t before = type_size(type);
                g.begin = (int)before;
                for (const LeafTmp* L : ls) {
                    if (L->chain != ch || L->type != type) continue;
                    if (world) {
                        LeafInfo li{};
                        li.type = type; li.chain = ch; li.mat = s->objs[L->obj].mat; li.flip = L->flip;
                        add_record(*L, &li);
                    } else {
                        add_record(*L, nullptr);
                    }
                }
                const size_t after = type_size(type);
                g.end = (int)after;
                if (after > before) out.push_back(g);
            }
        }
    };
    for (int sg = 0; sg < nseg; ++sg) {
        std::vector<const LeafTmp*> ls;
        const LeafTmp* medium = nullptr;
        for (size_t i = 0; i < f.leaves.size(); ++i) {
            if (seg[i] != sg) continue;
            if (f.leaves[i].type == LEAF_MEDIUM) medium = &f.leaves[i];
            else ls.push_back(&f.leaves[i]);
        }
        emit_groups(ls, groups, true, use_bvh && sg == 0);
        COMMIT_MARK("emit");
        if (!medium) continue;
        const Obj& o = s->objs[medium->obj];
        MediumRec m{};
        m.bg_begin = (int)bgroups.size();
        std::vector<const LeafTmp*> bl;
        for (const LeafTmp& L : f.bounds[medium->aux]) bl.push_back(&L);
        emit_groups(bl, bgroups, false, false);
        m.bg_end = (int)bgroups.size();
        m.neg_inv_density = -(1 / o.r);             // (- (/ 1 density)), geometry.scm:564
        LeafInfo li{};
        li.type = LEAF_MEDIUM; li.chain = medium->chain; li.local = (int)med.size();
        li.mat = o.mat; li.flip = medium->flip;
        groups.push_back(Group{LEAF_MEDIUM, medium->chain, (int)med.size(), (int)med.size() + 1});
        med.push_back(m);
        lmed.push_back(li);
    }
    if (lsph.size() != sph.size() || lmsph.size() != msph.size() || lbez.size() != bez.size() ||
        lklein.size() != klein.size() ||
        lrect[0].size() + lrect[1].size() + lrect[2].size() != rect.size())
        return fail("internal: leaf records and leaf infos out of step");
    // leaf ids: spheres, moving spheres, then all rects (rect locals index the shared rect array)
    // rect arrays are shared between the three axis types; leaf id = rect_base + local
    std::vector<LeafInfo> rl(rect.size());
    for (int a = 0; a < 3; ++a) for (auto& li : lrect[a]) rl[li.local] = li;
    int32_t base[kLeafTypes];
    base[LEAF_SPHERE] = 0;
    base[LEAF_MSPHERE] = base[LEAF_SPHERE] + (int32_t)lsph.size();
    base[LEAF_RECT_XY] = base[LEAF_RECT_XZ] = base[LEAF_RECT_YZ] = base[LEAF_MSPHERE] + (int32_t)lmsph.size();
    base[LEAF_BEZIER] = base[LEAF_RECT_XY] + (int32_t)rl.size();
    base[LEAF_MEDIUM] = base[LEAF_BEZIER] + (int32_t)lbez.size();
    base[LEAF_KLEIN] = base[LEAF_MEDIUM] + (int32_t)lmed.size();
    HostVec<LeafInfo> leaves;
    leaves.resize((size_t)base[LEAF_KLEIN] + lklein.size());
    auto put = [&](const LeafInfo* src, const size_t n, const int32_t at) {
        parallel_for(n, threads, [&](const size_t b, const size_t e) { std::copy(src + b, src + e, leaves.data() + at + b); });
    };
    put(lsph.data(), lsph.size(), base[LEAF_SPHERE]);
    put(lmsph.data(), lmsph.size(), base[LEAF_MSPHERE]);
    put(rl.data(), rl.size(), base[LEAF_RECT_XY]);
    put(lbez.data(), lbez.size(), base[LEAF_BEZIER]);
    put(lmed.data(), lmed.size(), base[LEAF_MEDIUM]);
    put(lklein.data(), lklein.size(), base[LEAF_KLEIN]);
    COMMIT_MARK("leaves");
    // the shade-side fields: material, texture shortcut, sphere centre (LeafInfo)
    parallel_for(leaves.size(), threads, [&](const size_t lb, const size_t le) {
      for (size_t lk = lb; lk < le; ++lk) {
        LeafInfo& li = leaves[lk];
        if (li.mat < 0 || li.mat >= (int)s->mats.size()) continue;     // boundary placeholders
        const DevMaterial& m = s->mats[li.mat];
        li.mtype = m.type;
        li.tex = m.tex;
        li.mparam = (m.type == MAT_METAL) ? m.fuzz : m.ref_idx;
        li.tex_kind = TK_GENERIC;
        auto constant = [&](int t) { return t >= 0 && t < (int)s->texs.size() && s->texs[t].type == TEX_CONSTANT; };
        if (constant(m.tex)) {
            const DevTexture& T = s->texs[m.tex];
            li.tex_kind = TK_CONSTANT;
            li.albedo[0] = T.r; li.albedo[1] = T.g; li.albedo[2] = T.bl;
        } else if (m.tex >= 0 && m.tex < (int)s->texs.size() && s->texs[m.tex].type == TEX_CHECKER &&
                   constant(s->texs[m.tex].a) && constant(s->texs[m.tex].b)) {
            const DevTexture& E = s->texs[s->texs[m.tex].a];       // even (texture.scm:20-23)
            const DevTexture& O = s->texs[s->texs[m.tex].b];       // odd
            li.tex_kind = TK_CHECKER_CONST;
            li.albedo[0] = E.r; li.albedo[1] = E.g; li.albedo[2] = E.bl;
            li.albedo2[0] = O.r; li.albedo2[1] = O.g; li.albedo2[2] = O.bl;
        }
        if (li.type == LEAF_SPHERE) {
            const SphereRec& S = sph[(size_t)li.local];
            li.c[0] = S.cx; li.c[1] = S.cy; li.c[2] = S.cz;
        } else if (li.type == LEAF_MSPHERE) {                   // center(0), the kernel's own operations
            const MSphereRec& M = msph[(size_t)li.local];
            const double frac = (0.0 - M.t0) / M.den;
            li.c[0] = M.c0x + M.dcx * frac; li.c[1] = M.c0y + M.dcy * frac; li.c[2] = M.c0z + M.dcz * frac;
        }
      }
    });

    std::vector<Chain> chains;
    for (auto& cv : f.chains) {
        Chain c{};
        c.n = (int)cv.size();
        for (size_t k = 0; k < cv.size(); ++k) c.ops[k] = cv[k];
        chains.push_back(c);
    }
    DevScene& d = s->dev;
    std::memset(&d, 0, sizeof d);
    COMMIT_MARK("groups");
    if (int rc = upload(s->d_sph, sph, &d.sph)) return rc;
    if (int rc = upload(s->d_msph, msph, &d.msph)) return rc;
    if (int rc = upload(s->d_rect, rect, &d.rect)) return rc;
    if (int rc = upload(s->d_groups, groups, &d.groups)) return rc;
    if (int rc = upload(s->d_bez, bez, &d.bez)) return rc;
    d.n_bez = (int)bez.size();
    if (int rc = upload(s->d_klein, klein, &d.klein)) return rc;
    d.n_klein = (int)klein.size();
    if (int rc = upload(s->d_med, med, &d.med)) return rc;
    d.n_med = (int)med.size();
    if (int rc = upload(s->d_bgroups, bgroups, &d.bgroups)) return rc;
    d.n_bgroups = (int)bgroups.size();
    d.bvh_has_bez = bvh_has_bez ? 1 : 0;
    d.bez_groups = 0;
    for (const Group& G : groups) d.bez_groups += G.type == LEAF_BEZIER ? 1 : 0;
    d.bvh_pad = bvh_pad;
    if (int rc = upload(s->d_bvh2, bvh2, &d.bvh2)) return rc;
    if (int rc = upload(s->d_bleaf, bleaf, &d.bleaf)) return rc;
    d.n_bvh2 = (int)bvh2.size();
    d.bvh2_root = bvh2_root;
    if (!fbvh2.empty()) {
        std::vector<int32_t> fid;
        for (const auto& sl : fsrc) fid.push_back(base[sl.first] + sl.second);
        if (int rc = upload(s->d_fbvh2, fbvh2, &d.fbvh2)) return rc;
        if (int rc = upload(s->d_fbleaf, fbleaf, &d.fbleaf)) return rc;
        if (int rc = upload(s->d_fsph, fsph, &d.fsph)) return rc;
        if (int rc = upload(s->d_fid, fid, &d.fid)) return rc;
        d.fbvh2_root = fbvh2_root;
        d.n_fbvh2 = (int)fbvh2.size(); d.n_fbleaf = (int)fbleaf.size(); d.n_fsph = (int)fsph.size();
        d.tree0_any_time = tree0_any_time ? 1 : 0;
    }
    d.n_bleaf = (int)bleaf.size();
    d.lane_stack = lane_stack;
    if (lane_stack > kLaneStack) return fail("internal: BVH deeper than the traversal stack");
    if (!bvh4.empty()) {
        if (int rc = upload(s->d_bvh4, bvh4, &d.bvh4)) return rc;
        d.n_bvh4 = (int)bvh4.size();
        d.bvh4_root = bvh4_root;
        d.stack4 = stack4;
        // the walk's LDS stack column: kCurveLdsStack entries (a walk rarely holds more; the rest go to the
        // overflow area), so the curve kernel's blocks stay small.  RTAMD_CURVE_LDS_STACK (tests): fewer
        // entries, so the walk exercises its overflow area
        const char* ce = std::getenv("RTAMD_CURVE_LDS_STACK");
        d.lds4 = std::min(lane_stack, ce ? std::max(1, std::atoi(ce)) : kCurveLdsStack);
        {                                            // survivor rings: RT_CURVE_WAVES 256-thread blocks per CU
            int dev = 0, cus = 0;
            HIPCHK(hipGetDevice(&dev));
            HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            d.ring_waves = (uint32_t)std::max(cus, 1) * 4u * (uint32_t)RT_CURVE_WAVES;
            HIPCHK(s->d_bez_ring.ensure((size_t)kLanes * d.ring_waves * kBezRing * 128u));
            d.bez_ring = s->d_bez_ring.as<double>();
            HIPCHK(s->d_fuse_ring.ensure((size_t)kLanes * d.ring_waves * kFuseWaveBytes));
            d.fuse_ring = s->d_fuse_ring.as<uint8_t>();
        }
        if (stack4 > d.lds4) {                       // the walk's deepest stacks spill past the LDS columns
            int dev = 0, cus = 0;
            HIPCHK(hipGetDevice(&dev));
            HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            d.ovf_lanes = (uint32_t)std::max(cus, 1) * 2048u;     // any resident grid of 256-thread blocks
            HIPCHK(s->d_stk_ovf.ensure((size_t)kLanes * d.ovf_lanes * (size_t)(stack4 - d.lds4) * sizeof(uint32_t)));
            d.stk_ovf = s->d_stk_ovf.as<uint32_t>();
        }
    }
    if (int rc = upload(s->d_chains, chains, &d.chains)) return rc;
    if (int rc = upload(s->d_leaves, leaves, &d.leaves)) return rc;
    {
        std::vector<uint8_t> lc((leaves.size() + 15) / 16 * 16 + 16, 0);
        for (size_t k = 0; k < leaves.size(); ++k) lc[k] = (uint8_t)leaves[k].mtype;
        if (int rc = upload(s->d_leaf_cls, lc, &d.leaf_cls)) return rc;
    }
    if (int rc = upload(s->d_mats, s->mats, &d.mats)) return rc;
    if (int rc = upload(s->d_texs, s->texs, &d.texs)) return rc;
    d.n_sph = (int)sph.size(); d.n_msph = (int)msph.size(); d.n_rect = (int)rect.size();
    d.n_groups = (int)groups.size(); d.n_chains = (int)chains.size(); d.n_leaves = (int)leaves.size();
    d.msph_shared = 0;
    if (!msph.empty()) {
        bool same = true;
        for (const MSphereRec& m : msph)
            same = same && std::memcmp(&m.t0, &msph[0].t0, sizeof(double)) == 0 &&
                   std::memcmp(&m.den, &msph[0].den, sizeof(double)) == 0;
        if (same) { d.msph_shared = 1; d.msph_t0 = msph[0].t0; d.msph_den = msph[0].den; }
    }
    d.bvh_solo = (groups.size() == 1 && groups[0].type == GROUP_BVH && !bvh_has_bez && tree0_direct &&
                  !std::getenv("RTAMD_NO_SOLO")) ? 1 : 0;
    d.n_mats = (int)s->mats.size(); d.n_texs = (int)s->texs.size();
    for (int k = 0; k < kLeafTypes; ++k) d.leaf_base[k] = base[k];
    d.has_perlin = s->have_perlin ? 1 : 0;
    d.has_noise_tex = 0;
    for (const auto& t : s->texs) if (t.type == TEX_NOISE || t.type == TEX_MARBLE) d.has_noise_tex = 1;
    if (s->have_perlin) {
        if (int rc = upload(s->d_ranvec, s->ranvec, &d.ranvec)) return rc;
        if (int rc = upload(s->d_perm, s->perm, &d.perm)) return rc;
    }
    d.sky = s->sky;
    std::memset(&d.light, 0, sizeof d.light);
    if (s->light >= 0) {
        const Obj* L = &s->objs[s->light];
        while (L->type == O_FLIP) L = &s->objs[L->child];
        if (L->type == O_RECT) {
            d.light.type = LIGHT_RECT; d.light.axis = L->axis;
            d.light.a0 = L->a0; d.light.a1 = L->a1; d.light.b0 = L->b0; d.light.b1 = L->b1; d.light.k = L->k;
        } else {
            d.light.type = LIGHT_SPHERE;
            d.light.cx = L->c0[0]; d.light.cy = L->c0[1]; d.light.cz = L->c0[2]; d.light.r = L->r;
        }
    }
    d.mat_mask = 0;
    for (const auto& m : s->mats) d.mat_mask |= 1 << m.type;
    const double* cm = s->cam;
    for (int k = 0; k < 3; ++k) {
        d.cam.llc[k] = cm[k]; d.cam.hor[k] = cm[3 + k]; d.cam.ver[k] = cm[6 + k];
        d.cam.origin[k] = cm[9 + k]; d.cam.w[k] = cm[12 + k]; d.cam.u[k] = cm[15 + k]; d.cam.v[k] = cm[18 + k];
    }
    d.cam.lens = cm[21]; d.cam.t0 = cm[22]; d.cam.t1 = cm[23];
    for (const Obj& o : s->objs)
        if (o.mat >= (int)s->mats.size()) return fail("object refers to an unknown material");
    // LDS footprints of the persistent kernels: only now is every count and
    // the stack depth in `d` final (the kernels carve their LDS from the same fields)
    s->ext_lds = 0;
    s->ext_lds_blocks = 0;
    if (!std::getenv("RTAMD_NO_EXTEND_LDS")) {
        const size_t lds = extend_lds_bytes(d);
        uint32_t mb = 0;
        if (lds > 0 && lds <= extend_lds_budget() && extend_lds_prepare(d, lds, &mb) == hipSuccess && mb >= 256) {
            s->ext_lds = lds;
            s->ext_lds_blocks = mb;           // every resident block (50-88 % of them: -0.3 .. -3 %, profiles/r02/pct)
        }
        (void)hipGetLastError();
    }
    s->cam_lds = 0;
    s->cam_blocks = 0;
    if (!std::getenv("RTAMD_NO_CAMERA_LDS")) {
        const size_t lds = camera_lds_bytes(d);
        uint32_t mb = 0;
        if (lds > 0 && lds <= extend_lds_budget() && camera_prepare(d, lds, &mb) == hipSuccess && mb >= 256) {
            s->cam_lds = lds;
            s->cam_blocks = mb;
        }
        (void)hipGetLastError();
    }
    HIPCHK(s->d_dev.ensure(sizeof(DevScene)));
    COMMIT_MARK("upload");
    HIPCHK(hipMemcpy(s->d_dev.p, &d, sizeof(DevScene), hipMemcpyHostToDevice));
    s->committed = true;
    g_reaper.reap(std::move(f), std::move(refs), std::move(bvh_nodes), std::move(bvh2), std::move(bleaf), std::move(bvh4),
                  std::move(sph), std::move(msph), std::move(bez), std::move(lsph), std::move(lmsph), std::move(lbez),
                  std::move(leaves), std::move(fbvh2), std::move(fbleaf), std::move(fsph));
    return 0;
}

// -------------------------------------------------------------- render
// The pixels a render covers: rows [y0, y1) of the frame (trace-all: every
// row; trace-line, main.scm:452-469: one row), restricted to shard `shard` of
// `nshard` interleaved 16x16 tiles (row-major tile order; tile t -> shard
// t % nshard).  Listed tile by tile, pixel j = y*nx + x.
struct PixSel { int y0, y1, shard, nshard; };
PixSel full_frame(int ny) { return PixSel{0, ny, 0, 1}; }
// The diagonal tile deal's row stride: the smallest odd prime coprime with the shard count (3 for every
// count not divisible by 3, so 1, 2, 4 and 8 shards keep the round-5 deal; 5 for 3 or 6 shards).  With a
// stride sharing a factor with the count, shard r would only ever get the columns tx = r mod that factor.
int tile_stride(const int nshard) {
    for (int k : {3, 5, 7, 11, 13, 17, 19, 23, 29, 31})
        if (nshard % k != 0) return k;
    return 37;                               // a product of the primes to 31 exceeds any int shard count
}
std::vector<uint32_t> make_pixlist(int nx, int ny, const PixSel& ps) {
    const int T = 16;
    const int tx = (nx + T - 1) / T, ty = (ny + T - 1) / T;
    std::vector<uint32_t> out;
    out.reserve((size_t)nx * (size_t)(ps.y1 - ps.y0) / (size_t)ps.nshard + T * T);
    // tile (x, y) belongs to shard (x + k y) % nshard, k = tile_stride(nshard).  Plain t % nshard degenerates
    // into vertical 16-px stripes whenever nshard divides the tiles per row (C2: 120, C4: 64): every rank then
    // renders the same columns of every row, and the Cornell box's walls are not alike (shard balance at C4,
    // one GPU per shard: max / mean 1.0385 for 8 shards, 1.0247 for 4; profiles/r05/balance.log).  The
    // diagonal deal with k coprime to nshard gives every shard one tile of each nshard consecutive ones along
    // a row and along a column.
    const int k = tile_stride(ps.nshard);
    for (int t = 0; t < tx * ty; ++t) {
        if (((t % tx) + k * (t / tx)) % ps.nshard != ps.shard) continue;
        const int bx = (t % tx) * T, by = (t / tx) * T;
        for (int yy = std::max(by, ps.y0); yy < std::min(std::min(by + T, ny), ps.y1); ++yy)
            for (int xx = bx; xx < std::min(bx + T, nx); ++xx) out.push_back((uint32_t)(yy * nx + xx));
    }
    return out;
}

// (re)build the gather plan for a frame size and world; the root's device list and receive buffer too
int gather_plan(GatherPlan& g, int nx, int ny, int world, bool root) {
    if (g.nx == nx && g.ny == ny && g.world == world && g.root == root) return 0;
    g.nx = -1;
    g.world = world;
    g.root = root;
    g.count.assign(world, 0);
    g.off.assign(world, 0);
    std::vector<uint32_t> all;
    int64_t total = 0;
    for (int r = 0; r < world; ++r) {
        const std::vector<uint32_t> pl = make_pixlist(nx, ny, PixSel{0, ny, r, world});
        g.off[r] = total;
        g.count[r] = (int64_t)pl.size();
        total += g.count[r];
        if (root) all.insert(all.end(), pl.begin(), pl.end());
    }
    if (root) {
        HIPCHK(g.pix.ensure(std::max<size_t>(1, all.size()) * sizeof(uint32_t)));
        if (!all.empty()) HIPCHK(hipMemcpy(g.pix.p, all.data(), all.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        HIPCHK(g.recv.ensure(std::max<size_t>(1, (size_t)g.others()) * 3 * sizeof(double)));
    }
    g.nx = nx;
    g.ny = ny;
    return 0;
}
// the root's placement: its own compact accumulator, then the received shards, into the y-up frame
int gather_place(const GatherPlan& g, const double* own, double* frame, hipStream_t st) {
    const uint32_t* pix = g.pix.as<const uint32_t>();
    if (g.count[0] > 0) HIPCHK(launch_scatter_pixels(own, pix, (uint32_t)g.count[0], frame, st));
    HIPCHK(launch_scatter_pixels(g.recv.as<const double>(), pix + g.count[0], (uint32_t)g.others(), frame, st));
    return 0;
}

std::string fault_text(uint32_t f) {
    std::string m = "device fault (flags " + std::to_string(f) + "):";
    if (f & RT_FAULT_REJECT) m += " a rejection sampler exceeded its attempt cap;";
    if (f & RT_FAULT_CURVE) m += " a curve walk exceeded its step bound or a curve needed more subdivision levels than the walk supports;";
    if (f & RT_FAULT_PATH) m += " a persistent kernel's path or ray exceeded its step bound;";
    if (f & RT_FAULT_SHARD) m += " a queue shard overflowed (the append was dropped);";
    if (f & RT_FAULT_LDS) m += " a persistent kernel's LDS allocation was too small;";
    return m;
}

// Path-pool cap (paths per chunk).  Bigger pools mean fewer chunks, each
// with its own narrow tail: C2 (1920x1080x1024 spp) 13 383 Mrays/s with 96M
// paths (22 chunks), 13 675 with 200M (12), 13 742 with 330M (8 chunks;
// profiles/r02/pool/); round 5, with the first frame on new pools excluded (a re-allocated pool's first frame
// waits for the driver to clear the memory it reuses, tools/realloc_probe.py): 8 chunks (288Mi- or 320Mi-path
// cap) 13 804–13 888, 10 / 12 chunks 13 657–13 711, 6 chunks (354Mi) 13 927 / 13 957 (profiles/r05/ab/pool/).
// Default 384Mi paths, but at most what lets the render lanes' pools (~272 B per path: two path-state
// pools, four hit queues, the sample buffer) take 65 % of the device's free memory — on a 288-GB MI355X
// C2's frame then cuts into 6 chunks (193 GB of pools).  RT_OPT_MAX_PATHS overrides.
size_t max_paths(const Context& c, const int lanes) {
    if (c.opt_max_paths > 0) return c.opt_max_paths < 1024 ? 1024 : (size_t)c.opt_max_paths;
    size_t v = (size_t)384 << 20;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
        const size_t fit = free_b / 100 * 65 / ((size_t)std::max(1, lanes) * 272);
        if (fit < v) v = fit;
    } else {
        (void)hipGetLastError();
    }
    return v < ((size_t)1 << 20) ? ((size_t)1 << 20) : v;
}

int lanes_wanted(const Context& c) {   // RT_OPT_LANES: path pools kept in flight (1 = no overlap)
    return c.opt_lanes > 0 ? (int)std::min<int64_t>(c.opt_lanes, kLanes) : 2;
}
// The persistent curve kernels serve scenes whose world BVH holds every curve (launch_extend)
bool curve_kernel_scene(const DevScene& d) {
    return d.n_bez > 0 && d.bvh_has_bez && d.bez_groups == 0 && d.n_med == 0 && d.n_klein == 0;
}
// Scenes whose world BVH holds curves run the persistent curve kernel, whose
// grid fills the chip by itself: a second lane's kernels only queue behind it
// and its narrow tails, so one lane is faster (C5 at 64 spp: 200.3 vs 164.1
// Mrays/s, profiles/r03/ab/ab_lanes_c5.log; round 5, 398.0 vs 304.9 at 32 spp and
// 409.1 vs 306.5 at 256 spp, profiles/r05/ab/lanes/).  RT_OPT_LANES overrides.
int lanes_for(const Context& c, const DevScene& d) {
    if (c.opt_lanes > 0) return lanes_wanted(c);
    return curve_kernel_scene(d) ? 1 : lanes_wanted(c);
}

// The fused curve extend (rt_kernels.hip k_extend_curves<FUSE>: every depth >= 1 of a chunk in one launch)
// serves curve-kernel scenes whose hits it can shade itself: no Perlin tables (the fused kernel keeps no
// LDS copy of them) and no light mixture (f2).  It pays where the per-depth launches are small: each
// persistent launch drains once (~1.1 ms at C5), which a depth-1 launch of n rays amortises over n.  C5,
// fused vs one launch per depth (profiles/r05/ab/fuse/): 1 spp 275.2 vs 189.5 Mrays/s, 8 spp 380.4 vs
// 356.1, 32 spp 394.8 vs 395.8, 256 spp (128-spp chunks) 402.9 vs 407.8 — so it is taken for depth-1
// launches of at most kFuseMaxRays rays (full frames below ~16 spp per chunk, e.g. the progressive
// one-pass-at-a-time loop, main.scm:533-544).  RTAMD_CURVE_FUSE=0 / 1: never / always (A/B, tests).
// (2^23 / 2^25: the same within noise at 32 and 256 spp, profiles/r06/fuse_max/)
constexpr uint32_t kFuseMaxRays = 1u << 24;
bool curve_fuse(const DevScene& d, const uint32_t n) {
    if (!(curve_kernel_scene(d) && curve_persistent() && !d.has_perlin && d.light.type == LIGHT_OFF)) return false;
    if (!d.fuse_ring || d.n_leaves >= (1 << kFuseLeafBits) - 1) return false;    // FuseHit packs leaf + 1 in 25 bits
    const char* e = std::getenv("RTAMD_CURVE_FUSE");   // read per render: tests switch it inside one process
    if (e && e[0] == '0') return false;
    if (e && e[0] == '1') return true;
    return n <= kFuseMaxRays;
}

// A chunk's live paths at or below max(tail_threshold, B / tail_divisor) go to
// the tail kernel; RT_OPT_TAIL_OFF keeps every depth in the wavefront.
// Without those options the threshold also follows the render's shape (round 5, C2's scene, same images;
// profiles/r05/ab/tail/): a render of one chunk has no second lane to fill its narrow depths, so the tail
// kernel takes over at B/4, at most 524 288 paths (1 spp per frame, the progressive loop: 2.60 → 2.13 ms); renders of a few
// small chunks take it at up to B/64, at most 262 144 paths (4 spp: 4.85 → 4.17 ms; 16 spp: 12.7 → 11.3 ms);
// large chunks keep B/256 (the 8-GPU per-rank share, 680×381×1024 spp: 73.6 ms at B/256, 75.1 at B/64; C2:
// B/256 over B/128, rounds 2–3).  Curve-kernel scenes keep the fixed rule (their tail kernel walks curves
// per ray; the fused curve extend serves their small launches).
uint32_t tail_paths(const Context& c, const uint32_t B, const int nchunks, const bool curves) {
    if (c.wavefront_only) return 0u;
    if (c.opt_tail_paths <= 0 && c.opt_tail_div <= 0 && !curves) {
        // (bounded: a large single chunk — one render lane, e.g. Cornell at 256 spp, 268M paths — keeps B/256;
        // B/4 there handed a quarter of the paths to the tail kernel: 100.6 of 213 ms)
        if (nchunks == 1) return std::max<uint32_t>(std::max<uint32_t>(32768u, std::min<uint32_t>(B / 4u, 524288u)), B / 256u);
        return std::max<uint32_t>(std::max<uint32_t>(32768u, std::min<uint32_t>(B / 64u, 262144u)), B / 256u);
    }
    const uint32_t thr = c.opt_tail_paths > 0 ? (uint32_t)std::min<int64_t>(c.opt_tail_paths, 0xFFFFFFFFll) : 32768u;
    // B/256 with 288M-path pools (+0.9 % over B/128, profiles/r02/tail*/; B/128 was best with 96M pools)
    const uint32_t div = c.opt_tail_div > 0 ? (uint32_t)std::min<int64_t>(c.opt_tail_div, 0xFFFFFFFFll) : 256u;
    return std::max<uint32_t>(thr, B / div);
}

constexpr size_t kStateBytesPerPath = sizeof(RayRec) + sizeof(PathRec) + sizeof(double) + sizeof(uint32_t);

PathState carve_state(void* base, size_t cap) {
    PathState st;
    char* p = static_cast<char*>(base);
    st.ray = reinterpret_cast<RayRec*>(p);
    p += cap * sizeof(RayRec);
    st.path = reinterpret_cast<PathRec*>(p);
    p += cap * sizeof(PathRec);
    st.tm = reinterpret_cast<double*>(p);
    p += cap * sizeof(double);
    st.rng0 = reinterpret_cast<uint32_t*>(p);
    return st;
}

// Render passes spp_begin .. spp_begin+spp_count-1 of the pixels `ps` selects
// into accum (indexed by image pixel j, or by the selection's own pixel index
// q when `compact`).
int render_impl(Scene* s, int nx, int ny, const PixSel& ps, int spp_begin, int spp_count, uint64_t seed,
                double* accum, bool compact, hipStream_t stream) {
    if (!s->committed) return fail("scene not committed (rt_scene_commit)");
    if (nx <= 0 || ny <= 0) return fail("image size must be positive");
    if (spp_begin < 0 || spp_count < 0) return fail("spp_begin/spp_count must be >= 0");
    if ((uint64_t)spp_begin + (uint64_t)spp_count > 0xFFFFFFFFull) return fail("sample index out of range");
    if (ps.nshard <= 0 || ps.shard < 0 || ps.shard >= ps.nshard) return fail("invalid shard index/count");
    if (ps.y0 < 0 || ps.y1 < ps.y0 || ps.y1 > ny) return fail("row range outside the image");
    if ((uint64_t)nx * (uint64_t)ny >= (1ull << 31)) return fail("image too large");
    Context* c = get_ctx(s->ctx);
    if (!c) return fail("scene's context was destroyed");
    HIPCHK(hipSetDevice(c->device));
    if (!stream) stream = c->stream;
    auto t_start = std::chrono::steady_clock::now();
    std::memset(&s->stats, 0, sizeof s->stats);
    {
        uint32_t stale = 0;
        HIPCHK(take_fault(&stale));                  // a fault word left by another context's failed launch
        unsigned long long cs[2];
        HIPCHK(take_curve_stats(cs));                // counters start at zero for this render
        // tests: drive a sampler / the curve kernel's per-ray loop into its cap
        const char* e = std::getenv("RTAMD_REJECT_CAP");
        const char* rc = std::getenv("RTAMD_CURVE_RAY_CAP");
        HIPCHK(set_test_caps(e ? std::max(0, std::atoi(e)) : 4096, rc ? (uint32_t)std::strtoul(rc, nullptr, 10) : 0u));
    }
    if (spp_count == 0) return 0;

    if (s->pix_nx != nx || s->pix_ny != ny || s->pix_y0 != ps.y0 || s->pix_y1 != ps.y1 || s->pix_shard != ps.shard ||
        s->pix_nshard != ps.nshard) {
        std::vector<uint32_t> pl = make_pixlist(nx, ny, ps);
        s->pix_nx = -1;                              // stale until the upload below succeeds
        HIPCHK(s->pixlist.ensure(std::max<size_t>(1, pl.size()) * sizeof(uint32_t)));
        if (!pl.empty()) HIPCHK(hipMemcpy(s->pixlist.p, pl.data(), pl.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        s->pix_nx = nx; s->pix_ny = ny; s->pix_y0 = ps.y0; s->pix_y1 = ps.y1;
        s->pix_shard = ps.shard; s->pix_nshard = ps.nshard;
        s->pix_n = (uint32_t)pl.size();
    }
    const uint32_t npix = s->pix_n;
    if (npix == 0) return 0;
    // Chunks of samples: as few as the pool cap allows, but at least two (one
    // per render lane) and an even count when the samples allow, so the two
    // lanes end together (a frame of three chunks would leave one lane alone
    // for a third of it).  A floor of four cost 6.5 % on a 1/8-frame shard
    // (680x381x1024 spp, the per-rank work at 8 GPUs) and 2.4 % at 1/4
    // (profiles/r02/mc/).
    // the cap is sized on the context's first render (before its pools exist), then kept; an option change
    // that resets it (RT_OPT_LANES, RT_OPT_MAX_PATHS) frees the old pools first, so the sizing sees the
    // memory they held and the lanes together stay within it
    if (!c->pool_cap) {
        for (auto& L : c->lanes)
            if (L && L->stream) HIPCHK(hipStreamSynchronize(L->stream));
        for (auto& L : c->lanes) L.reset();
        c->pool_lanes = std::min(kLanes, lanes_wanted(*c));
        c->pool_cap = max_paths(*c, c->pool_lanes);
    }
    const size_t cap_paths = c->pool_cap;
    uint32_t chunk = (uint32_t)std::max<size_t>(1, cap_paths / npix);
    if (chunk > (uint32_t)spp_count) chunk = (uint32_t)spp_count;
    {
        const int min_chunks = lanes_for(*c, s->dev);   // one chunk per lane at least
        int n = (int)((spp_count + chunk - 1) / chunk);
        if (n < min_chunks) n = std::min(min_chunks, spp_count);
        if (n > 1 && (n & 1) && n < spp_count) ++n;
        chunk = (uint32_t)((spp_count + n - 1) / n);
    }
    const int nchunks = (int)((spp_count + chunk - 1) / chunk);
    const int nlanes = std::max(1, std::min(std::min(kLanes, lanes_for(*c, s->dev)), nchunks));
    const size_t cap = (size_t)npix * chunk;
    s->stats.chunks = (uint32_t)nchunks;
    s->stats.lanes = (uint32_t)nlanes;
    // sharded compaction (rt_device.h kShards): shard capacity bounds what the
    // blocks of one shard can append in one wavefront step (extend: one item
    // per thread; the four shade kernels: grid-stride over at most 4096 blocks)
    const size_t gmax = std::min<size_t>(4096, (cap + 255) / 256 + kShards);
    size_t slack = 4 * 32 * gmax + 256;
    // test switch (RTAMD_SHARD_SLACK): a smaller slack drives k_extend_curves' hit appends past their wave's
    // shard (wave_append<true> spills into the next one); 256 still bounds the shade kernels' survivors
    if (const char* e = std::getenv("RTAMD_SHARD_SLACK")) slack = std::max<size_t>(256, std::strtoull(e, nullptr, 10));
    const size_t shard_cap = (cap + kShards - 1) / kShards + slack;
    const size_t scap = shard_cap * kShards;
    if (scap >= (1ull << 32)) return fail("path pool too large");
    constexpr int kCountsPerIter = 5 * kShards * kCntStride;   // 4 material hit queues + survivors, 8 shards each
    constexpr int kIters = kMaxDepth + 4;
    // callers' prior work on `stream` (e.g. zeroing accum) comes first
    hipEvent_t ev_in = nullptr;
    HIPCHK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    std::unique_ptr<void, void (*)(void*)> ev_in_guard(ev_in, [](void* e) { (void)hipEventDestroy((hipEvent_t)e); });
    HIPCHK(hipEventRecord(ev_in, stream));
    for (int li = 0; li < nlanes; ++li) {
        if (!c->lanes[li]) c->lanes[li].reset(new Lane());
        c->lanes[li]->index = li;
        Lane& L = *c->lanes[li];
        if (!L.stream) HIPCHK(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
        if (!L.ev_cnt) HIPCHK(hipEventCreateWithFlags(&L.ev_cnt, hipEventDisableTiming));
        if (!L.ev_acc) HIPCHK(hipEventCreateWithFlags(&L.ev_acc, hipEventDisableTiming));
        if (s->profiling && !L.ev[0]) for (auto& e : L.ev) HIPCHK(hipEventCreate(&e));
        HIPCHK(L.st_a.ensure(scap * kStateBytesPerPath));
        HIPCHK(L.st_b.ensure(scap * kStateBytesPerPath));
        HIPCHK(L.hit.ensure(4 * scap * sizeof(HitRec)));   // the 4 material hit queues (sharded like the survivors)
        HIPCHK(L.sb.ensure(cap * 3 * sizeof(double)));
        HIPCHK(L.counts.ensure(kIters * kCountsPerIter * sizeof(uint32_t)));
        // tail segments, next tail path / curve claim, LDS errors, the fused curve extend's continuation segments
        HIPCHK(L.seg_tail.ensure(4 * sizeof(unsigned long long)));
        if (!L.h_counts) HIPCHK(hipHostMalloc((void**)&L.h_counts, kIters * kCountsPerIter * sizeof(uint32_t)));
        HIPCHK(hipStreamWaitEvent(L.stream, ev_in, 0));
        HIPCHK(hipMemsetAsync(L.seg_tail.p, 0, 4 * sizeof(unsigned long long), L.stream));
        L.A = carve_state(L.st_a.p, scap);
        L.B = carve_state(L.st_b.p, scap);
        L.state = Lane::IDLE;
        L.n_fin = 0;
    }
    // An error return below leaves kernels queued on the lanes that may still
    // write the caller's accumulator: drain every lane before returning.
    struct Drain {
        Context* c; int n; bool armed = true;
        ~Drain() {
            if (!armed) return;
            for (int i = 0; i < n; ++i)
                if (c->lanes[i] && c->lanes[i]->stream) (void)hipStreamSynchronize(c->lanes[i]->stream);
            uint32_t f = 0;
            (void)take_fault(&f);                  // do not leak this render's fault bits into the next
        }
    } drain{c, nlanes};
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    // RT_OPT_EXACT_LIBM: auto = exact in scenes with curves or noise / marble textures ("libm"):
    // C3 (marble) frame rows with the device library's sin / cos were 0.79 % of pixels off by more than 1e-9;
    // exact there costs 1.7 % (profiles/r06/c3_libm/).  The cover scene keeps the device's: exact would cost it
    // 1.4 % (profiles/r06/c2_libm/) for 26 of 15 360 horizon pixels at 256 passes, all within 1e-7
    const bool exact_libm = c->opt_exact_libm == RT_LIBM_EXACT ||
                            (c->opt_exact_libm == RT_LIBM_AUTO && (s->dev.n_bez > 0 || s->dev.has_noise_tex));
    uint64_t seq = 0;

    // Enqueue the lane's next step for its current path count: one wavefront
    // iteration (extend + shades + the survivor-count readback), or, below
    // the tail threshold, the tail kernel that finishes every remaining path.
    auto step = [&](Lane& L) -> int {
        const uint32_t tail = tail_paths(*c, L.rp.B, nchunks, curve_kernel_scene(s->dev));
        if (L.n == 0) { L.state = Lane::DONE; return 0; }
        if (L.depth > kMaxDepth + 1) return fail("internal: path exceeded the depth cap");
        if (L.n <= tail) {
            std::pair<hipEvent_t, hipEvent_t>* fe = nullptr;
            if (s->profiling) {
                if (L.n_fin == L.ev_fin.size()) {
                    hipEvent_t e0 = nullptr, e1 = nullptr;
                    HIPCHK(hipEventCreate(&e0));
                    HIPCHK(hipEventCreate(&e1));
                    L.ev_fin.push_back({e0, e1});
                }
                fe = &L.ev_fin[L.n_fin++];
                HIPCHK(hipEventRecord(fe->first, L.stream));
            }
            HIPCHK(hipMemsetAsync(L.seg_tail.as<unsigned long long>() + 1, 0, sizeof(unsigned long long), L.stream));
            HIPCHK(launch_finish(s->dev, s->d_dev.as<const DevScene>(), L.rp, *L.cur, L.view, L.n, L.seg_tail.as<unsigned long long>(),
                                 s->ext_lds ? (size_t)32 << 10 : 0, (uint32_t)L.depth, L.stream));
            if (fe) HIPCHK(hipEventRecord(fe->second, L.stream));
            s->stats.finish_paths += L.n;
            L.state = Lane::DONE;
            return 0;
        }
        uint32_t* cnt = L.counts.as<uint32_t>() + L.depth * kCountsPerIter;   // [material][shard], survivors at 4
        bool fused = false;
        HitBuf hit{L.hit.as<HitRec>(), (uint32_t)scap};
        if (s->profiling) HIPCHK(hipEventRecord(L.ev[0], L.stream));
        if (L.depth == 0 && L.fused_camera)     // raygen + first closest hit in one kernel
            HIPCHK(launch_camera(s->dev, L.rp, *L.cur, L.n, hit, (uint32_t)shard_cap, cnt,
                                 s->cam_lds, s->cam_blocks, L.seg_tail.as<unsigned long long>() + 2, L.stream));
        else if (L.depth > 0 && s->ext_lds)     // every ray of a depth >= 1 launch has time +0.0
            HIPCHK(launch_extend_lds(s->dev, L.rp, *L.cur, L.view, L.n, hit, (uint32_t)shard_cap,
                                     cnt, s->ext_lds_blocks, L.seg_tail.as<unsigned long long>() + 2, L.stream));
        else {
            // the curve walk's stack overflow area: one region per render lane (lanes run concurrently)
            DevScene dl = s->dev;
            if (dl.stk_ovf) dl.stk_ovf += (size_t)L.index * dl.ovf_lanes * (size_t)(dl.stack4 - dl.lds4);
            if (dl.bez_ring) dl.bez_ring += (size_t)L.index * dl.ring_waves * kBezRing * 16u;
            if (dl.fuse_ring) dl.fuse_ring += (size_t)L.index * dl.ring_waves * kFuseWaveBytes;
            // the fused curve extend (k_extend_curves<FUSE>): every depth from 1 on in this one launch
            CurveFuse fz{L.seg_tail.as<unsigned long long>() + 3, (uint32_t)L.depth};
            fused = L.depth > 0 && curve_fuse(s->dev, L.n);
            HIPCHK(launch_extend(dl, s->d_dev.as<const DevScene>(), L.rp, *L.cur, L.view, L.n, hit,
                                 (uint32_t)shard_cap, cnt, L.depth == 0,
                                 reinterpret_cast<unsigned int*>(L.seg_tail.as<unsigned long long>() + 1),
                                 fused ? &fz : nullptr, L.stream));
        }
        if (s->profiling) HIPCHK(hipEventRecord(L.ev[1], L.stream));
        uint32_t* surv = cnt + 4 * kShards * kCntStride;
        for (int mt = 0; mt < 4 && !fused; ++mt) {         // (a fused launch shades its hits itself: no queues)
            if (!(s->dev.mat_mask & (1 << mt))) continue;
            const QView qv{cnt + mt * kShards * kCntStride, (uint32_t)shard_cap};
            HIPCHK(launch_shade(mt, s->dev, s->d_dev.as<const DevScene>(), L.rp, *L.cur, hit, qv, L.n, *L.nxt, surv,
                                (uint32_t)shard_cap, (uint32_t)L.depth, L.stream));
        }
        if (s->profiling) HIPCHK(hipEventRecord(L.ev[2], L.stream));
        HIPCHK(hipMemcpyAsync(L.h_counts + L.depth * kCountsPerIter, cnt, kCountsPerIter * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, L.stream));
        HIPCHK(hipEventRecord(L.ev_cnt, L.stream));
        L.state = Lane::RUNNING;
        L.seq = seq++;
        return 0;
    };
    // The iteration's counts have arrived: take its statistics, move on.
    auto advance = [&](Lane& L) -> int {
        if (s->profiling) {
            float a = 0, b = 0;
            HIPCHK(hipEventElapsedTime(&a, L.ev[0], L.ev[1]));
            HIPCHK(hipEventElapsedTime(&b, L.ev[1], L.ev[2]));
            s->stats.ms_extend += a; s->stats.ms_shade += b;
            s->stats.extend_launches += 1;
        }
        s->stats.extend_rays += L.n;
        s->stats.segments += L.n;
        if ((uint32_t)L.depth > s->stats.max_depth_seen) s->stats.max_depth_seen = (uint32_t)L.depth;
        const uint32_t* row = L.h_counts + L.depth * kCountsPerIter;
        uint32_t n = 0;
        for (int x = 0; x < kShards; ++x) {
            const uint32_t c_x = row[4 * kShards * kCntStride + x * kCntStride];
            if (c_x > shard_cap) return fail("internal: shard overflow");
            n += c_x;
        }
        uint64_t hits = 0;
        // a hit-queue counter can pass its shard's capacity (k_extend_curves' items then spill into the next
        // shard): what the queue holds is the clamped count
        for (int k = 0; k < 4 * kShards; ++k) hits += std::min<uint32_t>(row[k * kCntStride], (uint32_t)shard_cap);
        (L.depth == 0 ? s->stats.shade_hits_d0 : s->stats.shade_hits) += hits;
        s->stats.shade_survivors += n;
        L.view = QView{L.counts.as<uint32_t>() + L.depth * kCountsPerIter + 4 * kShards * kCntStride,
                       (uint32_t)shard_cap};
        std::swap(L.cur, L.nxt);
#ifdef RT_STATS
        static const bool dbg_depth = std::getenv("RTAMD_DEBUG_DEPTH") != nullptr;   // stats builds: live paths per depth
        if (dbg_depth) std::fprintf(stderr, "depth-count lane %d chunk %d depth %d in %u out %u\n", L.index, L.chunk,
                                    L.depth, L.n, n);
#endif
        L.n = n;
        ++L.depth;
        return step(L);
    };
    auto start = [&](Lane& L, int ch) -> int {
        const int done = ch * (int)chunk;
        L.chunk = ch;
        L.S = (uint32_t)std::min<int>((int)chunk, spp_count - done);
        RenderParams& rp = L.rp;
        rp = RenderParams{};
        rp.nx = (uint32_t)nx; rp.ny = (uint32_t)ny; rp.npix = npix;
        rp.inx = 1.0 / (double)nx; rp.iny = 1.0 / (double)ny;
        rp.spp0 = (uint32_t)(spp_begin + done); rp.k0 = k0; rp.k1 = k1;
        rp.pixlist = s->pixlist.as<const uint32_t>();
        rp.sb = L.sb.as<double>();
        rp.B = npix * L.S;
        rp.compact = compact ? 1u : 0u;
        rp.exact_libm = exact_libm ? 1u : 0u;
        HIPCHK(hipMemsetAsync(L.counts.p, 0, kIters * kCountsPerIter * sizeof(uint32_t), L.stream));
        const uint32_t tail = tail_paths(*c, rp.B, nchunks, curve_kernel_scene(s->dev));
        L.fused_camera = s->cam_lds != 0 && rp.B > tail;     // the tail kernel starts from raygen's state
        if (!L.fused_camera) HIPCHK(launch_raygen(s->dev, rp, L.A, L.stream));
        L.cur = &L.A;
        L.nxt = &L.B;
        L.view = QView{nullptr, (uint32_t)scap};         // raygen output: contiguous
        L.n = rp.B;
        L.depth = 0;
        s->stats.paths += rp.B;
        return step(L);
    };

    int next_chunk = 0, next_acc = 0;
    Lane* last_acc = nullptr;
    while (next_acc < nchunks) {
        bool progressed = false;
        for (int li = 0; li < nlanes; ++li) {           // accumulate in chunk order
            Lane& L = *c->lanes[li];
            if (L.state != Lane::DONE || L.chunk != next_acc) continue;
            if (last_acc && last_acc != &L) HIPCHK(hipStreamWaitEvent(L.stream, last_acc->ev_acc, 0));
            HIPCHK(launch_accumulate(L.rp, L.S, accum, L.stream));
            HIPCHK(hipEventRecord(L.ev_acc, L.stream));
            last_acc = &L;
            ++next_acc;
            L.state = Lane::IDLE;
            progressed = true;
            li = -1;                                     // the next chunk may sit on an earlier lane
        }
        for (int li = 0; li < nlanes; ++li) {           // idle lanes take the next chunk
            Lane& L = *c->lanes[li];
            if (L.state != Lane::IDLE || next_chunk >= nchunks) continue;
            if (int rc = start(L, next_chunk++)) return rc;
            progressed = true;
        }
        for (int li = 0; li < nlanes; ++li) {           // lanes whose counts have arrived
            Lane& L = *c->lanes[li];
            if (L.state != Lane::RUNNING) continue;
            const hipError_t q = hipEventQuery(L.ev_cnt);
            if (q == hipErrorNotReady) continue;
            HIPCHK(q);
            if (int rc = advance(L)) return rc;
            progressed = true;
        }
        if (progressed) continue;
        Lane* oldest = nullptr;                          // nothing to do: wait for the oldest pending step
        for (int li = 0; li < nlanes; ++li) {
            Lane& L = *c->lanes[li];
            if (L.state == Lane::RUNNING && (!oldest || L.seq < oldest->seq)) oldest = &L;
        }
        if (!oldest) return fail("internal: render lanes stalled");
        HIPCHK(hipEventSynchronize(oldest->ev_cnt));
    }
    for (int li = 0; li < nlanes; ++li) HIPCHK(hipStreamSynchronize(c->lanes[li]->stream));
    drain.armed = false;
    {
        uint32_t f = 0;
        HIPCHK(take_fault(&f));
        if (f) return fail(fault_text(f));
        unsigned long long cs[2];
        HIPCHK(take_curve_stats(cs));
        s->stats.curve_pooled_batches = cs[0];
        s->stats.curve_flat_pooled = cs[1];
    }
    for (int li = 0; li < nlanes; ++li) {
        Lane& L = *c->lanes[li];
        unsigned long long ctl[4] = {0, 0, 0, 0};
        HIPCHK(hipMemcpy(ctl, L.seg_tail.p, sizeof ctl, hipMemcpyDeviceToHost));
        if (ctl[2]) return fail("internal: a persistent kernel's LDS allocation was too small (flags " +
                                std::to_string(ctl[2]) + ")");
        s->stats.segments += ctl[0] + ctl[3];
        s->stats.extend_rays += ctl[3];                // the fused curve extend's segments past its launch's rays
        for (size_t k = 0; k < L.n_fin; ++k) {
            float a = 0;
            HIPCHK(hipEventElapsedTime(&a, L.ev_fin[k].first, L.ev_fin[k].second));
            s->stats.ms_finish += a;
        }
    }
    // later work on the caller's stream sees the finished accumulator
    HIPCHK(hipStreamSynchronize(stream));
    s->stats.ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return 0;
}

}  // namespace

// =================================================================== C ABI
extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_err.c_str(); }

int rt_device_count(int* out) {
    if (!out) return fail("null out pointer");
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    *out = n;
    return 0;
}

int rt_context_create(int device, int* out_ctx) {
    if (!out_ctx) return fail("null out pointer");
    int n = 0;
    HIPCHK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail("device " + std::to_string(device) + " out of range (" + std::to_string(n) + " devices)");
    HIPCHK(hipSetDevice(device));
    auto c = std::make_unique<Context>();
    c->device = device;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    std::lock_guard<std::mutex> lk(g_mu);
    int h = g_next_ctx++;
    g_ctx[h] = std::move(c);
    *out_ctx = h;
    return 0;
}

int rt_context_destroy(int ctx) {
    std::lock_guard<std::mutex> lk(g_mu);
    Context* c = get_ctx(ctx);
    if (!c) return fail("invalid context handle");
    for (auto it = g_scene.begin(); it != g_scene.end();) {
        if (it->second->ctx == ctx) it = g_scene.erase(it); else ++it;
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    g_ctx.erase(ctx);
    return 0;
}

int rt_context_release_pools(int ctx) {
    std::lock_guard<std::mutex> lk(g_mu);
    Context* c = get_ctx(ctx);
    if (!c) return fail("invalid context handle");
    HIPCHK(hipSetDevice(c->device));
    for (auto& L : c->lanes)
        if (L && L->stream) HIPCHK(hipStreamSynchronize(L->stream));
    for (auto& L : c->lanes) L.reset();
    c->pool_cap = 0;                               // the next render sizes them again
    return 0;
}

int rt_context_set_option(int ctx, int option, int64_t value) {
    std::lock_guard<std::mutex> lk(g_mu);
    Context* c = get_ctx(ctx);
    if (!c) return fail("invalid context handle");
    if (value < 0) return fail("option value must be >= 0 (0 = automatic)");
    switch (option) {
    case RT_OPT_LANES: {
        if (value > kLanes) return fail("RT_OPT_LANES: at most " + std::to_string(kLanes) + " render lanes");
        // more lanes than the pools were sized for: size them again for the lanes together (the next render
        // frees them first); otherwise the lanes kept hold pools of the right size, so keep them — a re-allocated pool's
        // first frame waits for the driver to clear the memory it reuses (4.7–6.6 s for C2's ~150 GB,
        // profiles/r05/ab/realloc/), which a lane-count dip (bench.py's single-lane profiling frame) need not pay
        const int64_t new_n = value > 0 ? std::min<int64_t>(value, kLanes) : 2;
        if (new_n > c->pool_lanes) c->pool_cap = 0;
        c->opt_lanes = value;
        break;
    }
    case RT_OPT_MAX_PATHS:
        if (value > ((int64_t)1 << 32)) return fail("RT_OPT_MAX_PATHS: at most 2^32 paths per pool");
        c->opt_max_paths = value;
        c->pool_cap = 0;                           // the next render sizes the pools again
        break;
    case RT_OPT_TAIL_PATHS: c->opt_tail_paths = value; break;
    case RT_OPT_TAIL_DIV: c->opt_tail_div = value; break;
    case RT_OPT_TAIL_OFF: c->wavefront_only = value != 0; break;
    case RT_OPT_EXACT_LIBM:
        if (value > RT_LIBM_DEVICE) return fail("RT_OPT_EXACT_LIBM: RT_LIBM_AUTO, RT_LIBM_EXACT or RT_LIBM_DEVICE");
        c->opt_exact_libm = value;
        break;
    default: return fail("unknown context option " + std::to_string(option));
    }
    return 0;
}

int rt_context_get_option(int ctx, int option, int64_t* out) {
    if (!out) return fail("null out pointer");
    std::lock_guard<std::mutex> lk(g_mu);
    Context* c = get_ctx(ctx);
    if (!c) return fail("invalid context handle");
    switch (option) {
    case RT_OPT_LANES: *out = c->opt_lanes; break;
    case RT_OPT_MAX_PATHS: *out = c->opt_max_paths; break;
    case RT_OPT_TAIL_PATHS: *out = c->opt_tail_paths; break;
    case RT_OPT_TAIL_DIV: *out = c->opt_tail_div; break;
    case RT_OPT_TAIL_OFF: *out = c->wavefront_only ? 1 : 0; break;
    case RT_OPT_EXACT_LIBM: *out = c->opt_exact_libm; break;
    default: return fail("unknown context option " + std::to_string(option));
    }
    return 0;
}

int rt_scene_begin(int ctx, int* out_scene) {
    if (!out_scene) return fail("null out pointer");
    std::lock_guard<std::mutex> lk(g_mu);
    if (!get_ctx(ctx)) return fail("invalid context handle");
    auto s = std::make_unique<Scene>();
    s->ctx = ctx;
    int h = g_next_scene++;
    g_scene[h] = std::move(s);
    *out_scene = h;
    return 0;
}

int rt_scene_destroy(int scene) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_scene.erase(scene)) return fail("invalid scene handle");
    return 0;
}

#define OUT_OR_FAIL(p) if (!(p)) return fail("null out pointer")

int rt_add_texture_constant(int scene, const double rgb[3], int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    DevTexture t{};
    t.type = TEX_CONSTANT; t.r = rgb[0]; t.g = rgb[1]; t.bl = rgb[2];
    s->texs.push_back(t);
    *out = (int)s->texs.size() - 1;
    return 0;
}
int rt_add_texture_checker(int scene, int even, int odd, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (check_tex(s, even) || check_tex(s, odd)) return 1;
    DevTexture t{};
    t.type = TEX_CHECKER; t.a = even; t.b = odd;
    s->texs.push_back(t);
    *out = (int)s->texs.size() - 1;
    return 0;
}
static int add_scaled_tex(int scene, int type, double sc, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    DevTexture t{};
    t.type = type; t.scale = sc;
    s->texs.push_back(t);
    *out = (int)s->texs.size() - 1;
    return 0;
}
int rt_add_texture_noise(int scene, double sc, int* out) { return add_scaled_tex(scene, TEX_NOISE, sc, out); }
int rt_add_texture_marble(int scene, double sc, int* out) { return add_scaled_tex(scene, TEX_MARBLE, sc, out); }

static int add_mat(int scene, int type, int tex, double fuzz, double ref, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (type != MAT_DIELECTRIC && check_tex(s, tex)) return 1;
    DevMaterial m{};
    m.type = type; m.tex = tex; m.fuzz = fuzz; m.ref_idx = ref;
    s->mats.push_back(m);
    *out = (int)s->mats.size() - 1;
    return 0;
}
int rt_add_material_lambertian(int scene, int tex, int* out) { return add_mat(scene, MAT_LAMBERTIAN, tex, 0, 0, out); }
int rt_add_material_metal(int scene, int tex, double fuzz, int* out) { return add_mat(scene, MAT_METAL, tex, fuzz, 0, out); }
int rt_add_material_dielectric(int scene, double ref, int* out) { return add_mat(scene, MAT_DIELECTRIC, -1, 0, ref, out); }
int rt_add_material_diffuse_light(int scene, int tex, int* out) { return add_mat(scene, MAT_DIFFUSE_LIGHT, tex, 0, 0, out); }

static int push_obj(Scene* s, Obj&& o, int* out) {
    s->objs.push_back(std::move(o));
    *out = (int)s->objs.size() - 1;
    return 0;
}

int rt_add_sphere(int scene, const double c[3], double r, int mat, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (check_mat(s, mat)) return 1;
    Obj o; o.type = O_SPHERE; o.mat = mat; o.r = r;
    for (int k = 0; k < 3; ++k) o.c0[k] = c[k];
    return push_obj(s, std::move(o), out);
}
int rt_add_moving_sphere(int scene, const double c0[3], const double c1[3], double t0, double t1, double r,
                         int mat, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (check_mat(s, mat)) return 1;
    Obj o; o.type = O_MSPHERE; o.mat = mat; o.r = r; o.t0 = t0; o.t1 = t1;
    for (int k = 0; k < 3; ++k) { o.c0[k] = c0[k]; o.c1[k] = c1[k]; }
    return push_obj(s, std::move(o), out);
}
int rt_add_rect(int scene, int axis, double a0, double a1, double b0, double b1, double k, int mat, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (axis < 0 || axis > 2) return fail("rect axis must be RT_RECT_XY/XZ/YZ");
    if (check_mat(s, mat)) return 1;
    Obj o; o.type = O_RECT; o.axis = axis; o.mat = mat;
    o.a0 = a0; o.a1 = a1; o.b0 = b0; o.b1 = b1; o.k = k;
    return push_obj(s, std::move(o), out);
}
int rt_add_bezier(int scene, const double a[3], const double b[3], const double c[3], const double d[3],
                  double width, int mat, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (!a || !b || !c || !d) return fail("rt_add_bezier: null control point");
    if (check_mat(s, mat)) return 1;
    // make-bezier has no check, but a width <= 0 makes converge's depth estimate the log of a number
    // <= 0 (eps = width / 20, bezier.scm:179-192): Gauche's log returns a complex (or -inf for 0) and
    // ceiling->exact raises, so the reference fails on the first ray that tests such a curve
    if (!(width > 0.0) || !std::isfinite(width))
        return fail("rt_add_bezier: width must be positive and finite (the reference's depth estimate fails otherwise)");
    Obj o; o.type = O_BEZIER; o.mat = mat; o.width = width;
    const double* p[4] = {a, b, c, d};
    for (int i = 0; i < 4; ++i) for (int k = 0; k < 3; ++k) o.cp[3 * i + k] = p[i][k];
    return push_obj(s, std::move(o), out);
}
int rt_add_bezier_array(int scene, const double* cps, int n, double width, int mat, int* out_first) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out_first);
    if (n < 0 || (n > 0 && !cps)) return fail("rt_add_bezier_array: invalid curve array");
    if (check_mat(s, mat)) return 1;
    // make-bezier has no check, but a width <= 0 makes converge's depth estimate the log of a number
    // <= 0 (eps = width / 20, bezier.scm:179-192): Gauche's log returns a complex (or -inf for 0) and
    // ceiling->exact raises, so the reference fails on the first ray that tests such a curve
    if (!(width > 0.0) || !std::isfinite(width))
        return fail("rt_add_bezier_array: width must be positive and finite (the reference's depth estimate fails otherwise)");
    *out_first = (int)s->objs.size();
    s->objs.reserve(s->objs.size() + (size_t)n);
    for (int i = 0; i < n; ++i) {
        Obj o; o.type = O_BEZIER; o.mat = mat; o.width = width;
        for (int k = 0; k < 12; ++k) o.cp[k] = cps[(size_t)i * 12 + k];
        s->objs.push_back(std::move(o));
    }
    return 0;
}
int rt_add_klein(int scene, const double center[3], int mat, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (!center) return fail("rt_add_klein: null centre");
    if (check_mat(s, mat)) return 1;
    Obj o; o.type = O_KLEIN; o.mat = mat;
    for (int k = 0; k < 3; ++k) o.c0[k] = center[k];
    return push_obj(s, std::move(o), out);
}
int rt_add_constant_medium(int scene, int boundary, double density, int albedo_tex, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (check_obj(s, boundary)) return 1;
    if (check_tex(s, albedo_tex)) return 1;
    if (!(density > 0.0) || !std::isfinite(density)) return fail("rt_add_constant_medium: density must be positive and finite");
    // the phase function is (m:make-lambertian a), geometry.scm:546
    DevMaterial m{};
    m.type = MAT_LAMBERTIAN; m.tex = albedo_tex;
    s->mats.push_back(m);
    Obj o; o.type = O_MEDIUM; o.child = boundary; o.r = density; o.mat = (int)s->mats.size() - 1;
    return push_obj(s, std::move(o), out);
}
int rt_set_light_sampling(int scene, int light_obj) {
    SCENE_OR_FAIL(s, scene);
    if (light_obj < 0) { s->light = -1; return 0; }
    if (check_obj(s, light_obj)) return 1;
    const Obj* L = &s->objs[light_obj];
    while (L->type == O_FLIP) L = &s->objs[L->child];
    if (L->type != O_RECT && L->type != O_SPHERE)
        return fail("rt_set_light_sampling: the light must be a rect or a sphere (optionally flipped)");
    s->light = light_obj;
    return 0;
}
int rt_add_flip_normals(int scene, int child, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (check_obj(s, child)) return 1;
    Obj o; o.type = O_FLIP; o.child = child; o.mat = s->objs[child].mat;
    return push_obj(s, std::move(o), out);
}
int rt_add_box(int scene, const double p0[3], const double p1[3], int mat, int* out) {
    // geometry.scm:444-463 — six rects, back faces flipped, in this order
    int r[6], tmp;
    if (rt_add_rect(scene, RT_RECT_XY, p0[0], p1[0], p0[1], p1[1], p1[2], mat, &r[0])) return 1;
    if (rt_add_rect(scene, RT_RECT_XY, p0[0], p1[0], p0[1], p1[1], p0[2], mat, &tmp)) return 1;
    if (rt_add_flip_normals(scene, tmp, &r[1])) return 1;
    if (rt_add_rect(scene, RT_RECT_XZ, p0[0], p1[0], p0[2], p1[2], p1[1], mat, &r[2])) return 1;
    if (rt_add_rect(scene, RT_RECT_XZ, p0[0], p1[0], p0[2], p1[2], p0[1], mat, &tmp)) return 1;
    if (rt_add_flip_normals(scene, tmp, &r[3])) return 1;
    if (rt_add_rect(scene, RT_RECT_YZ, p0[1], p1[1], p0[2], p1[2], p1[0], mat, &r[4])) return 1;
    if (rt_add_rect(scene, RT_RECT_YZ, p0[1], p1[1], p0[2], p1[2], p0[0], mat, &tmp)) return 1;
    if (rt_add_flip_normals(scene, tmp, &r[5])) return 1;
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    Obj o; o.type = O_BOX; o.mat = mat; o.kids.assign(r, r + 6);
    for (int k = 0; k < 3; ++k) { o.c0[k] = p0[k]; o.c1[k] = p1[k]; }
    return push_obj(s, std::move(o), out);
}
int rt_add_translate(int scene, int child, const double off[3], int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (check_obj(s, child)) return 1;
    Obj o; o.type = O_TRANSLATE; o.child = child; o.mat = s->objs[child].mat;
    for (int k = 0; k < 3; ++k) o.c0[k] = off[k];
    return push_obj(s, std::move(o), out);
}
int rt_add_rotate_y(int scene, int child, double angle, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (check_obj(s, child)) return 1;
    Obj o; o.type = O_ROTATE_Y; o.child = child; o.mat = s->objs[child].mat;
    const double radians = (kPi / 180.0) * angle;     // geometry.scm:484
    o.sin_t = std::sin(radians); o.cos_t = std::cos(radians);
    return push_obj(s, std::move(o), out);
}
int rt_add_list(int scene, const int* objs, int n, int* out) {
    SCENE_OR_FAIL(s, scene);
    OUT_OR_FAIL(out);
    if (n < 0 || (n > 0 && !objs)) return fail("invalid object list");
    Obj o; o.type = O_LIST;
    for (int i = 0; i < n; ++i) { if (check_obj(s, objs[i])) return 1; o.kids.push_back(objs[i]); }
    return push_obj(s, std::move(o), out);
}
int rt_add_bvh(int scene, const int* objs, int n, double t0, double t1, int sah, int* out) {
    (void)t0; (void)t1; (void)sah;
    if (rt_add_list(scene, objs, n, out)) return 1;
    std::lock_guard<std::mutex> lk(g_mu);
    get_scene(scene)->objs[*out].type = O_BVH;
    return 0;
}

int rt_make_camera(const double from[3], const double at[3], const double vup[3], double vfov, double aspect,
                   double aperture, double focus, double t0, double t1, double out[RT_CAMERA_DOUBLES]) {
    if (!out) return fail("null out pointer");
    // camera.scm:63-78 in the reference's evaluation order
    auto sub = [](const double* a, const double* b, double* r) { for (int k = 0; k < 3; ++k) r[k] = a[k] - b[k]; };
    auto unit = [](const double* a, double* r) {
        double d = 0.0; d += a[0] * a[0]; d += a[1] * a[1]; d += a[2] * a[2];
        const double k = 1.0 / std::sqrt(d);
        for (int i = 0; i < 3; ++i) r[i] = a[i] * k;
    };
    auto cross = [](const double* a, const double* b, double* r) {
        r[0] = a[1] * b[2] - b[1] * a[2]; r[1] = a[2] * b[0] - b[2] * a[0]; r[2] = a[0] * b[1] - b[0] * a[1];
    };
    const double theta = vfov * (kPi / 180.0);
    const double hh = std::tan(theta / 2);
    const double hw = aspect * hh;
    double w[3], u[3], v[3], tmp[3];
    sub(from, at, tmp); unit(tmp, w);
    cross(vup, w, tmp); unit(tmp, u);
    cross(w, u, v);
    for (int k = 0; k < 3; ++k) {
        double llc = from[k] - u[k] * (hw * focus);
        llc = llc - v[k] * (hh * focus);
        llc = llc - w[k] * focus;
        out[k] = llc;
        out[3 + k] = u[k] * (2 * hw * focus);
        out[6 + k] = v[k] * (2 * hh * focus);
        out[9 + k] = from[k];
        out[12 + k] = w[k]; out[15 + k] = u[k]; out[18 + k] = v[k];
    }
    out[21] = aperture / 2; out[22] = t0; out[23] = t1;
    return 0;
}

int rt_set_camera(int scene, const double cam[RT_CAMERA_DOUBLES]) {
    SCENE_OR_FAIL(s, scene);
    if (!cam) return fail("null camera");
    std::memcpy(s->cam, cam, sizeof s->cam);
    s->have_cam = true;
    return 0;
}
int rt_set_sky(int scene, int sky) {
    SCENE_OR_FAIL(s, scene);
    if (sky != RT_SKY_GRADIENT && sky != RT_SKY_BLACK) return fail("sky must be RT_SKY_GRADIENT or RT_SKY_BLACK");
    s->sky = sky;
    return 0;
}
int rt_set_perlin_tables(int scene, const double ranvec[768], const int32_t px[256], const int32_t py[256],
                         const int32_t pz[256]) {
    SCENE_OR_FAIL(s, scene);
    if (!ranvec || !px || !py || !pz) return fail("null Perlin table");
    s->ranvec.assign(ranvec, ranvec + 768);
    s->perm.resize(768);
    for (int i = 0; i < 256; ++i) {
        if (px[i] < 0 || px[i] > 255 || py[i] < 0 || py[i] > 255 || pz[i] < 0 || pz[i] > 255)
            return fail("Perlin permutation entries must be in 0..255");
        s->perm[i] = px[i]; s->perm[256 + i] = py[i]; s->perm[512 + i] = pz[i];
    }
    s->have_perlin = true;
    return 0;
}
int rt_scene_commit(int scene, int world) {
    SCENE_OR_FAIL(s, scene);
    if (check_obj(s, world)) return 1;
    const auto t0 = std::chrono::steady_clock::now();
    tl_upload_ms = 0.0;
    const int rc = commit_scene(s, world);
#ifdef RT_COMMIT_PROFILE
    std::fprintf(stderr, "commit %-12s %9.1f ms\n", "return",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
#endif
    s->commit_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    s->commit_upload_ms = tl_upload_ms;
    return rc;
}

int rt_set_profiling(int scene, int enabled) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    s->profiling = enabled != 0;
    return 0;
}

int rt_get_stats(int scene, rt_stats* out) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!out) return fail("null out pointer");
    *out = s->stats;
    return 0;
}

int rt_get_scene_info(int scene, rt_scene_info* out) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!out) return fail("null out pointer");
    if (!s->committed) return fail("scene not committed (rt_scene_commit)");
    Context* c = get_ctx(s->ctx);
    if (!c) return fail("scene's context was destroyed");
    const DevScene& d = s->dev;
    std::memset(out, 0, sizeof *out);
    out->leaves = d.n_leaves;
    out->groups = d.n_groups;
    out->bvh_nodes = d.n_bvh2;
    out->bvh0_nodes = d.n_fbvh2;
    out->tree_depth = d.lane_stack;
    out->bvh_solo = d.bvh_solo;
    out->extend_lds_bytes = (uint32_t)s->ext_lds;
    out->extend_lds_blocks = s->ext_lds_blocks;
    out->camera_lds_bytes = (uint32_t)s->cam_lds;
    out->camera_lds_blocks = s->cam_blocks;
    int cus = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    out->cus = cus;
    out->curve_stack = d.bvh4 ? d.stack4 : 0;
    out->commit_ms = s->commit_ms;
    out->commit_upload_ms = s->commit_upload_ms;
    out->commit_sah_ms = s->commit_sah_ms;
    out->commit_threads = s->commit_threads;
    return 0;
}

int rt_hit_rays(int scene, int n, const double* rays, double* out_t, int32_t* out_mat) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!s->committed) return fail("scene not committed (rt_scene_commit)");
    if (n < 0) return fail("ray count must be >= 0");
    if (n > 0 && (!rays || !out_t || !out_mat)) return fail("null pointer");
    if (s->dev.n_med > 0) return fail("rt_hit_rays: the scene has constant media, whose hit test draws random numbers");
    Context* c = get_ctx(s->ctx);
    if (!c) return fail("scene's context was destroyed");
    if (n == 0) return 0;
    HIPCHK(hipSetDevice(c->device));
    uint32_t stale = 0;
    HIPCHK(take_fault(&stale));
    DevBuf d_rays, d_t, d_mat;
    HIPCHK(d_rays.ensure((size_t)n * 7 * sizeof(double)));
    HIPCHK(d_t.ensure((size_t)n * sizeof(double)));
    HIPCHK(d_mat.ensure((size_t)n * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(d_rays.p, rays, (size_t)n * 7 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_hit_rays(s->dev, d_rays.as<const double>(), (uint32_t)n, d_t.as<double>(), d_mat.as<int32_t>(),
                           c->stream));
    HIPCHK(hipMemcpyAsync(out_t, d_t.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(out_mat, d_mat.p, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    uint32_t f = 0;
    HIPCHK(take_fault(&f));
    if (f) return fail(fault_text(f));
    return 0;
}

int rt_curve_depth_probe(int ctx, int n, const double* cps, const double* eps8, int32_t* out_depth) {
    std::lock_guard<std::mutex> lk(g_mu);
    Context* c = get_ctx(ctx);
    if (!c) return fail("invalid context handle");
    if (n < 0) return fail("curve count must be >= 0");
    if (n == 0) return 0;
    if (!cps || !eps8 || !out_depth) return fail("null pointer");
    HIPCHK(hipSetDevice(c->device));
    DevBuf d_cps, d_eps, d_out;
    HIPCHK(d_cps.ensure((size_t)n * 12 * sizeof(double)));
    HIPCHK(d_eps.ensure((size_t)n * sizeof(double)));
    HIPCHK(d_out.ensure((size_t)n * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(d_cps.p, cps, (size_t)n * 12 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_eps.p, eps8, (size_t)n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_curve_depth(d_cps.as<const double>(), d_eps.as<const double>(), (uint32_t)n, d_out.as<int32_t>(),
                              c->stream));
    HIPCHK(hipMemcpyAsync(out_depth, d_out.p, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int rt_render_device(int scene, int nx, int ny, int spp_begin, int spp_count, uint64_t seed, int shard,
                     int nshard, double* accum, void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!accum) return fail("null accum");
    if (ny <= 0) return fail("image size must be positive");
    return render_impl(s, nx, ny, PixSel{0, ny, shard, nshard}, spp_begin, spp_count, seed, accum, false,
                       (hipStream_t)stream);
}

int rt_render_shard_device(int scene, int nx, int ny, int spp_begin, int spp_count, uint64_t seed, int shard,
                           int nshard, double* accum_compact, void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!accum_compact) return fail("null accum");
    if (ny <= 0) return fail("image size must be positive");
    return render_impl(s, nx, ny, PixSel{0, ny, shard, nshard}, spp_begin, spp_count, seed, accum_compact, true,
                       (hipStream_t)stream);
}

int rt_render_rows_device(int scene, int nx, int ny, int y_begin, int y_count, int spp_begin, int spp_count,
                          uint64_t seed, double* accum, void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!accum) return fail("null accum");
    if (y_begin < 0 || y_count < 0 || (int64_t)y_begin + y_count > ny) return fail("row range outside the image");
    return render_impl(s, nx, ny, PixSel{y_begin, y_begin + y_count, 0, 1}, spp_begin, spp_count, seed, accum, false,
                       (hipStream_t)stream);
}

namespace {
// rows [y0, y0+yn) of a host accumulator through the context's device copy
int render_rows_host(Scene* s, int nx, int ny, int y0, int yn, int spp_begin, int spp_count, uint64_t seed,
                     double* accum_host) {
    if (nx <= 0 || ny <= 0) return fail("image size must be positive");
    if (y0 < 0 || yn < 0 || (int64_t)y0 + yn > ny) return fail("row range outside the image");
    Context* c = get_ctx(s->ctx);
    if (!c) return fail("scene's context was destroyed");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(c->accum_tmp.ensure((size_t)nx * ny * 3 * sizeof(double)));
    const size_t off = (size_t)y0 * nx * 3, cnt = (size_t)yn * nx * 3;
    double* dev = c->accum_tmp.as<double>();
    HIPCHK(hipMemcpyAsync(dev + off, accum_host + off, cnt * sizeof(double), hipMemcpyHostToDevice, c->stream));
    if (int rc = render_impl(s, nx, ny, PixSel{y0, y0 + yn, 0, 1}, spp_begin, spp_count, seed, dev, false, c->stream))
        return rc;
    HIPCHK(hipMemcpyAsync(accum_host + off, dev + off, cnt * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}
}  // namespace

int rt_render_rows(int scene, int nx, int ny, int y_begin, int y_count, int spp_begin, int spp_count, uint64_t seed,
                   double* accum_host) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!accum_host) return fail("null accum");
    return render_rows_host(s, nx, ny, y_begin, y_count, spp_begin, spp_count, seed, accum_host);
}

int rt_trace_line(int scene, int nx, int ny, int y, int sample_count, uint64_t seed, double* raw_data,
                  uint8_t* image) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!raw_data || !image) return fail("null buffer");
    if (sample_count < 1) return fail("sample_count is 1-based (main.scm:452)");
    if (int rc = render_rows_host(s, nx, ny, y, 1, sample_count - 1, 1, seed, raw_data)) return rc;
    // main.scm:462-469: correct-gamma of sum/sample-count, floor(255.99*min(1,c)), for row y only
    const size_t b = (size_t)y * nx * 3, e = b + (size_t)nx * 3;
    for (size_t i = b; i < e; ++i) {
        const double c = std::sqrt(raw_data[i] / sample_count);
        const double m = (1.0 < c) ? 1.0 : c;
        image[i] = (uint8_t)std::floor(255.99 * m);
    }
    return 0;
}

int rt_render(int scene, int nx, int ny, int spp_begin, int spp_count, uint64_t seed, double* accum_host) {
    std::lock_guard<std::mutex> lk(g_mu);
    Scene* s = get_scene(scene);
    if (!s) return fail("invalid scene handle");
    if (!accum_host) return fail("null accum");
    if (nx <= 0 || ny <= 0) return fail("image size must be positive");
    Context* c = get_ctx(s->ctx);
    if (!c) return fail("scene's context was destroyed");
    HIPCHK(hipSetDevice(c->device));
    const size_t bytes = (size_t)nx * ny * 3 * sizeof(double);
    HIPCHK(c->accum_tmp.ensure(bytes));
    HIPCHK(hipMemcpyAsync(c->accum_tmp.p, accum_host, bytes, hipMemcpyHostToDevice, c->stream));
    if (int rc = render_impl(s, nx, ny, full_frame(ny), spp_begin, spp_count, seed, c->accum_tmp.as<double>(), false,
                             c->stream))
        return rc;
    HIPCHK(hipMemcpyAsync(accum_host, c->accum_tmp.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int rt_shard_pixels(int nx, int ny, int shard, int nshard, uint32_t* out_pix, int64_t* out_count) {
    if (nx <= 0 || ny <= 0) return fail("image size must be positive");
    if (nshard <= 0 || shard < 0 || shard >= nshard) return fail("invalid shard index/count");
    if (!out_count) return fail("null out pointer");
    const std::vector<uint32_t> pl = make_pixlist(nx, ny, PixSel{0, ny, shard, nshard});
    *out_count = (int64_t)pl.size();
    if (out_pix && !pl.empty()) std::memcpy(out_pix, pl.data(), pl.size() * sizeof(uint32_t));
    return 0;
}

int rt_resolve_u8(const double* accum, int nx, int ny, int count, uint8_t* out) {
    if (!accum || !out) return fail("null buffer");
    if (count <= 0) return fail("sample_count must be positive");
    const size_t n = (size_t)nx * ny * 3;
    for (size_t i = 0; i < n; ++i) {
        const double c = std::sqrt(accum[i] / count);
        const double m = (1.0 < c) ? 1.0 : c;
        out[i] = (uint8_t)std::floor(255.99 * m);
    }
    return 0;
}

// ---- multi-GPU frame: the frame-end gather over RCCL (include/rt.h) ----
#define NCCLCHK(expr)                                                                  \
    do {                                                                               \
        ncclResult_t r_ = (expr);                                                      \
        if (r_ != ncclSuccess) return fail(std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

int rt_comm_unique_id(uint8_t out_id[RT_COMM_ID_BYTES]) {
    if (!out_id) return fail("null out pointer");
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "RT_COMM_ID_BYTES is RCCL's unique id size");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    std::memcpy(out_id, &id, sizeof id);
    return 0;
}

int rt_comm_create(int ctx, const uint8_t unique_id[RT_COMM_ID_BYTES], int rank, int world, int* out_comm) {
    if (!unique_id || !out_comm) return fail("null pointer");
    if (world <= 0 || rank < 0 || rank >= world) return fail("invalid rank / world size");
    int device = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        Context* c = get_ctx(ctx);
        if (!c) return fail("invalid context handle");
        device = c->device;
    }
    HIPCHK(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof id);
    auto m = std::make_shared<Comm>();
    m->ctx = ctx; m->rank = rank; m->world = world; m->device = device;
    // collective: returns once every rank has called it (outside the lock: it waits for the other processes)
    NCCLCHK(ncclCommInitRank(&m->nc, world, id, rank));
    std::lock_guard<std::mutex> lk(g_mu);
    const int h = g_next_comm++;
    g_comm[h] = std::move(m);
    *out_comm = h;
    return 0;
}

int rt_comm_destroy(int comm) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comm.find(comm);
    if (it == g_comm.end()) return fail("invalid communicator handle");
    Context* c = get_ctx(it->second->ctx);
    if (c) HIPCHK(hipSetDevice(c->device));
    g_comm.erase(it);
    return 0;
}

int rt_gather_shards(int comm, int nx, int ny, const double* accum_compact, double* frame_device, void* stream) {
    if (nx <= 0 || ny <= 0) return fail("image size must be positive");
    if ((uint64_t)nx * (uint64_t)ny >= (1ull << 31)) return fail("image too large");
    std::shared_ptr<Comm> keep;                       // alive through the call, whatever rt_comm_destroy does
    hipStream_t st = (hipStream_t)stream;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_comm.find(comm);
        if (it == g_comm.end()) return fail("invalid communicator handle");
        keep = it->second;
        Context* c = get_ctx(keep->ctx);
        if (!c) return fail("the communicator's context was destroyed");
        if (!st) st = c->stream;                      // (the context must outlive the call: rt.h)
    }
    Comm* m = keep.get();
    HIPCHK(hipSetDevice(m->device));
    if (int rc = gather_plan(m->plan, nx, ny, m->world, m->rank == 0)) return rc;
    const GatherPlan& g = m->plan;
    const int64_t mine = g.count[m->rank];
    if (mine > 0 && !accum_compact) return fail("null compact accumulator");
    if (m->rank == 0 && !frame_device) return fail("rank 0 needs the frame buffer");
    // RCCL has no gather: every other rank sends its compact accumulator (its exact size, no padding) to
    // rank 0, which posts one receive per rank into its buffer at recv_at(r), in one group.
    // The group is always closed, also after a failed call inside it (an open group poisons the thread's
    // later RCCL calls).
    if (m->world > 1) {
        ncclResult_t r0 = ncclGroupStart();
        if (r0 != ncclSuccess) return fail(std::string("ncclGroupStart: ") + ncclGetErrorString(r0));
        ncclResult_t bad = ncclSuccess;
        if (m->rank != 0) {
            if (mine > 0) bad = ncclSend(accum_compact, (size_t)(3 * mine), ncclDouble, 0, m->nc, st);
        } else {
            double* recv = g.recv.as<double>();
            for (int r = 1; r < m->world && bad == ncclSuccess; ++r)
                if (g.count[r] > 0) bad = ncclRecv(recv + g.recv_at(r), (size_t)(3 * g.count[r]), ncclDouble, r, m->nc, st);
        }
        const ncclResult_t end = ncclGroupEnd();
        if (bad != ncclSuccess) return fail(std::string("ncclSend / ncclRecv: ") + ncclGetErrorString(bad));
        if (end != ncclSuccess) return fail(std::string("ncclGroupEnd: ") + ncclGetErrorString(end));
    }
    if (m->rank == 0)                                  // place every shard's pixels into the y-up frame
        if (int rc = gather_place(g, accum_compact, frame_device, st)) return rc;
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

int rt_gather_layout(int nx, int ny, int world, int64_t* out_count, int64_t* out_offset) {
    if (nx <= 0 || ny <= 0) return fail("image size must be positive");
    if ((uint64_t)nx * (uint64_t)ny >= (1ull << 31)) return fail("image too large");
    if (world <= 0) return fail("invalid world size");
    if (!out_count || !out_offset) return fail("null out pointer");
    GatherPlan g;
    if (int rc = gather_plan(g, nx, ny, world, false)) return rc;
    for (int r = 0; r < world; ++r) { out_count[r] = g.count[r]; out_offset[r] = g.off[r]; }
    return 0;
}

int rt_gather_shards_local(int ctx, int nx, int ny, int world, const double* const* accum_compact,
                           double* frame_device, void* stream) {
    if (nx <= 0 || ny <= 0) return fail("image size must be positive");
    if ((uint64_t)nx * (uint64_t)ny >= (1ull << 31)) return fail("image too large");
    if (world <= 0) return fail("invalid world size");
    if (!accum_compact || !frame_device) return fail("null pointer");
    std::lock_guard<std::mutex> lk(g_mu);
    Context* c = get_ctx(ctx);
    if (!c) return fail("invalid context handle");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (int rc = gather_plan(c->gplan, nx, ny, world, true)) return rc;
    const GatherPlan& g = c->gplan;
    for (int r = 0; r < world; ++r)
        if (g.count[r] > 0 && !accum_compact[r]) return fail("null compact accumulator for shard " + std::to_string(r));
    // what the RCCL gather's receives do: shard r's compact accumulator at recv_at(r)
    double* recv = g.recv.as<double>();
    for (int r = 1; r < world; ++r)
        if (g.count[r] > 0)
            HIPCHK(hipMemcpyAsync(recv + g.recv_at(r), accum_compact[r], (size_t)g.count[r] * 3 * sizeof(double),
                                  hipMemcpyDeviceToDevice, st));
    if (int rc = gather_place(g, accum_compact[0], frame_device, st)) return rc;
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

int rt_resolve_u8_device(int ctx, const double* accum, int nx, int ny, int count, uint8_t* out, void* stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    Context* c = get_ctx(ctx);
    if (!c) return fail("invalid context handle");
    if (!accum || !out) return fail("null buffer");
    if (count <= 0) return fail("sample_count must be positive");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(launch_resolve_u8(accum, (uint32_t)((size_t)nx * ny * 3), count, out, st));
    HIPCHK(hipStreamSynchronize(st));
    return 0;
}

}  // extern "C"
