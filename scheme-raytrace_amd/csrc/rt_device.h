// rt_device.h — device-side scene and wavefront-state layout (HBM).
//
// The reference evaluates closest hit by calling one closure per object of a
// linked list (geometry.scm:33-50) and nested closures for flip / box /
// translate / rotate-y (geometry.scm:433-543).  Here the host flattens that
// object tree into *leaf primitives*, each tagged with an instance chain
// (translate / rotate-y ops, outermost first) and a flip parity, and groups
// leaves of one type under one chain so the extend kernel runs one uniform,
// type-specialised loop per group with the primitive parameters read through
// the scalar unit (every lane of a wave tests the same primitive).
#pragma once
#include <stdint.h>

#include "../../include/rt.h"

namespace rtamd {

constexpr int kMaxDepth = 100;                 // main.scm:26
constexpr double kTmin = 0.001;                // main.scm:104
constexpr double kTmax = 999999999999.0;       // constant.scm:6
constexpr double kPi = 3.141592653589793;      // math.const pi
constexpr int kMaxChain = 4;                   // instance ops per leaf chain
// device fault bits: RT_FAULT_* (include/rt.h); rt_kernels.hip g_fault, reported by render_impl

enum TexType : int32_t { TEX_CONSTANT = 0, TEX_CHECKER = 1, TEX_NOISE = 2, TEX_MARBLE = 3 };
enum MatType : int32_t { MAT_LAMBERTIAN = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2, MAT_DIFFUSE_LIGHT = 3 };
enum LeafType : int32_t { LEAF_SPHERE = 0, LEAF_MSPHERE = 1, LEAF_RECT_XY = 2, LEAF_RECT_XZ = 3,
                          LEAF_RECT_YZ = 4, LEAF_BEZIER = 5, LEAF_MEDIUM = 6, LEAF_KLEIN = 7 };
constexpr int kLeafTypes = 8;
constexpr int32_t GROUP_BVH = 8;               // group type: BVH over world-level spheres / curves
// closest-hit kernel variants: scene features compiled in (extra = constant media, Klein limit sets)
constexpr int kFeatCurves = 1, kFeatExtra = 2;
enum ChainOp : int32_t { OP_TRANSLATE = 0, OP_ROTATE_Y = 1 };

struct DevTexture {            // texture.scm:12-34
    int32_t type, a, b, pad;   // checker: a = even, b = odd
    double r, g, bl, scale;
};
struct DevMaterial {           // material.scm:24-111
    int32_t type, tex;
    double fuzz, ref_idx;
};

// Extend-side records: only what the closest-hit test reads, 16-B aligned so
// the scalar unit fetches each with one s_load_dwordx8 / x16.
struct alignas(32) SphereRec { double cx, cy, cz, rr; };             // rr = r*r
struct alignas(32) MSphereRec {                                        // center(t) = c0 + dc*((t-t0)/den), 96 B
    double c0x, c0y, c0z, rr, dcx, dcy, dcz, t0;
    double den, pad0, pad1, pad2;
};
struct alignas(64) RectRec { double a0, a1, b0, b1, k, pad0, pad1, pad2; };
// Cubic Bezier curve of a given width (bezier.scm:61-66): control points,
// width1 = width/2, width2 = width1^2, eps8 = 8*(width/20).
// order: the curve's position in the flattened object list (ties between curves at one z go to the later one)
struct alignas(64) BezierRec { double cp[12]; double w1, w2, eps8; uint32_t order, pad; };
constexpr int kBezMaxDepth = 24;               // subdivision levels the curve test supports
// Constant medium (geometry.scm:545-578): its boundary is the closest hit over
// the boundary groups [bg_begin, bg_end) of DevScene::bgroups; neg_inv_density
// = (- (/ 1 density)).  The phase function is a lambertian material.
// Kleinian limit set (geometry.scm:590-673): its centre; the six inversion
// spheres and radii are the module's constants.
struct alignas(32) KleinRec { double cx, cy, cz, pad; };
struct MediumRec { int32_t bg_begin, bg_end, pad0, pad1; double neg_inv_density, pad; };

// BVH over the world-level spheres, moving spheres and curves, per-lane
// traversal layout (Aila & Laine style BVH2): both child boxes live in the
// parent so one visit tests two boxes.  Boxes are padded outward so culling is
// conservative: the primitive tests are the exact f64 ones, the BVH only skips
// primitives that cannot report a hit.  Child refs: >= 0 inner node, < 0 leaf
// ~index into BvhLeaf.  Boxes are f32, rounded outward and widened by an
// absolute margin that covers the f32 slab test's rounding for any ray whose
// origin lies within the scene's radius (see commit_scene), so culling stays
// conservative.
// Child boxes interleaved left/right per plane, b = {lx0, rx0, ly0, ry0, lz0,
// rz0, lx1, rx1, ly1, ry1, lz1, rz1}: the kernel tests both children with
// packed f32 FMAs (v_pk_fma_f32) on adjacent register pairs.
struct alignas(64) BvhNode2 { float b[12]; int32_t l, r, pad0, pad1; };
struct BvhLeaf { int32_t sb, sn, mb, mn, bb, bn, pad0, pad1; };   // sphere / moving / curve ranges
// Trees that hold curves: a leaf holding exactly one curve k (and nothing
// else) is referenced as ~(kDirectCurve + k), so a walk queues the curve from
// the child ref itself instead of fetching a BvhLeaf record.
constexpr int32_t kDirectCurve = 1 << 30;
// The curve tree as a BVH4 for the persistent curve kernel (k_extend_curves):
// each BVH2 inner node with an inner child replaced by that child's two
// children (the BVH2's own f32 boxes, so culling stays as conservative), so a
// walk through a tree far larger than the L2 pays one dependent 128-B fetch
// per two levels.  Planes as [axis][child]; child refs as in BvhNode2 (>= 0
// an inner BvhNode4, < 0 a leaf / direct curve); children [n, 4) are empty.
struct alignas(128) BvhNode4 { float lo[3][4]; float hi[3][4]; int32_t ref[4]; int32_t n, pad0, pad1, pad2; };
static_assert(sizeof(BvhNode4) == 128, "BvhNode4 is one 128-B line");
constexpr int kLaneStack = 32;                 // max per-lane traversal stack (dynamic LDS, stride = block size)

// Shade-side per-leaf record (indexed by leaf id): what a shade kernel reads
// for a hit, in one 128-B record, so a hit costs one dependent load instead
// of the chain leaf -> group -> primitive -> material -> texture.
enum TexKind : int32_t { TK_GENERIC = 0, TK_CONSTANT = 1, TK_CHECKER_CONST = 2 };
struct alignas(16) LeafInfo {
    int32_t type, chain, local, flip;  // local = index in the type's array; chain: instance chain (-1 world)
    int32_t mat, mtype, tex, tex_kind; // material id and type, its texture id and TexKind
    double mparam;                     // fuzz (metal) / ref_idx (dielectric)
    double inv_r;                      // sphere / moving sphere: (/ 1 radius) as a double
    double c[3];                       // sphere center; moving sphere: center(0), for time-0 rays
    double albedo[3];                  // TK_CONSTANT colour / TK_CHECKER_CONST even colour
    double albedo2[3];                 // TK_CHECKER_CONST odd colour
    double pad;
};

struct ChainOpRec { int32_t op, pad; double x, y, z; };   // translate: (x,y,z); rotate: x=sin, y=cos
struct Chain { int32_t n, pad; ChainOpRec ops[kMaxChain]; };

// One group = leaves [begin, end) of one type under one chain (-1 = world).
struct Group { int32_t type, chain, begin, end; };   // begin/end index the type array
                                                      // leaf id = leaf_base[type] + local

// Light sampling target for the pdf.scm mixture (extension f2): an axis rect
// (axis as LeafType rect order) or a sphere.  type 0 = off.
struct DevLight {
    int32_t type, axis, pad0, pad1;          // type: 0 off, 1 rect, 2 sphere
    double a0, a1, b0, b1, k;                // rect
    double cx, cy, cz, r;                    // sphere
};
enum { LIGHT_OFF = 0, LIGHT_RECT = 1, LIGHT_SPHERE = 2 };

struct DevCamera {            // camera.scm:33-78 (the 10 slots)
    double llc[3], hor[3], ver[3], origin[3], w[3], u[3], v[3];
    double lens, t0, t1;
};

// k_extend_curves' BVH4 stack entries per lane in LDS (the rest of a deep walk's stack goes to the
// overflow area).  15 is the most that keeps two 256-thread blocks (the register-bound occupancy) on a
// 160-KiB CU beside the blocks' BezWave state; C5 at 8 spp: 8 -> 320, 12 -> 337, 15 -> 340 Mrays/s
// (profiles/r04/ab_stack.log)
constexpr int kBezRing = 256;                  // survivor ring entries per wave (> the survivors a wave holds)
#ifndef RT_CURVE_WAVES
#define RT_CURVE_WAVES 2               // waves per SIMD k_extend_curves is compiled for (VGPR budget 512 / waves)
#endif
#ifndef RT_CURVE_LDS_STACK
#define RT_CURVE_LDS_STACK 15
#endif

struct DevScene {
    const SphereRec* sph;  int32_t n_sph;
    const MSphereRec* msph; int32_t n_msph;
    const RectRec* rect;   int32_t n_rect;
    const BezierRec* bez;  int32_t n_bez;
    const MediumRec* med;  int32_t n_med;
    const KleinRec* klein; int32_t n_klein;
    const Group* bgroups;  int32_t n_bgroups;     // medium boundaries (not part of the world loop)
    const Group* groups;   int32_t n_groups;
    const BvhNode2* bvh2;  int32_t n_bvh2;
    const BvhLeaf* bleaf;  int32_t bvh2_root;      // root child ref (may be a leaf)
    int32_t bvh_has_bez;                           // curves in the BVH: widen the box t range (see bvh_closest)
    int32_t bez_groups;                            // curve groups outside the world BVH (k_extend_curves needs none)
    float bvh_pad;                                 // the margin baked into the f32 boxes (diagnostic)
    int32_t lane_stack;                            // deepest BVH2 level (stack entries a traversal needs)
    // BVH4 of the same tree (curve trees only, else nullptr): its walk pushes up to three children per
    // node, stack4 entries at most; entries past the LDS stack (lds4) go to stk_ovf, stack4 - lds4
    // words per lane of a grid of at most ovf_lanes lanes (entry e of lane g at e * lanes + g);
    // the buffer holds one such region per render lane and each launch gets its lane's (rt_api.cpp)
    const BvhNode4* bvh4;  int32_t n_bvh4;
    // k_extend_curves' survivor rings: per resident wave kBezRing entries of 128 B (a root-culled curve's
    // ray-space control points and widths, written by stage A, read by stage B's refills and takes)
    double* bez_ring;  uint32_t ring_waves;
    // the fused curve extend's per-wave hand-off rings (k_extend_curves<FUSE>): kFuseRing parked hits
    // (FuseHit, waiting for a whole-wave shading round) then kFuseRing ready paths (FuseReady, scattered
    // rays waiting for a lane), kFuseWaveBytes per resident wave
    uint8_t* fuse_ring;
    int32_t bvh4_root, stack4;
    int32_t lds4;                                  // the walk's stack entries in LDS (lane_stack; tests lower it)
    uint32_t* stk_ovf;     uint32_t ovf_lanes;
    // Time-0 tree over the same primitives (nullptr = none): every moving
    // sphere frozen at center(0), so rays with time +0.0 (all scattered rays,
    // Q4) traverse tighter boxes.  Leaves index fsph (plain sphere records in
    // tree order); fid maps an fsph entry to its leaf id.
    const BvhNode2* fbvh2; const BvhLeaf* fbleaf; int32_t fbvh2_root;
    const SphereRec* fsph; const int32_t* fid;
    int32_t n_fbvh2, n_fbleaf, n_fsph;
    int32_t tree0_any_time;                        // no moving spheres in the tree: the time-0 tree serves every ray
    int32_t n_bleaf;                               // leaves of the all-times tree
    int32_t msph_shared;                           // every moving sphere has the same (t0, den = t1 - t0): the
    double msph_t0, msph_den;                      // tree walk computes (time - t0) / den once per ray
    int32_t bvh_solo;                              // the world is exactly one BVH group (no other groups) and
                                                   // every time-0 leaf is one sphere, fsph in leaf order: the
                                                   // LDS kernels compile only the tree walk, with direct leaves
    const Chain* chains;   int32_t n_chains;
    const LeafInfo* leaves; int32_t n_leaves;
    const uint8_t* leaf_cls;                   // leaf id -> material type (a byte per leaf, padded to 16)
    int32_t leaf_base[kLeafTypes];             // first leaf id of each LeafType
    const DevMaterial* mats; int32_t n_mats;
    const DevTexture* texs;  int32_t n_texs;
    const double* ranvec;                      // 256*3 (Perlin)
    const int32_t* perm;                       // 3*256 (x, y, z)
    int32_t has_perlin;
    int32_t has_noise_tex;                     // some texture is noise / marble
    int32_t sky;                               // 0 gradient, 1 black
    int32_t mat_mask;                          // bit t set <=> some material of type t exists
    DevCamera cam;
    DevLight light;
};

// Wavefront path state, SoA, one slot per live path (ping-pong buffers).
// A path's pixel and absolute sample index follow from its work id (wid =
// s_rel * npix + q: pixel pixlist[q], sample spp0 + s_rel), so they are not
// stored.  Depth-0 state (raygen output) holds only what varies per camera
// ray — o, d, time, draw counter (throughput is 1, wid is the slot, depth 0);
// scattered rays all have time 0 (Q4), so deeper state has no time.
// Records, not one array per field: a lane reads its ray with three 16-B
// loads, and a kernel holds 4 base pointers instead of 13 (scalar registers).
#ifdef RT_F32_RECORDS
// Measurement build only ("f32 records"): ray and throughput
// records stored in f32, all arithmetic still f64 — the record traffic an f32
// perf mode would save, at the cost of parity.  Never the product build.
struct alignas(8) RayRec { float ox, oy, oz, dx, dy, dz; };                   // 24 B
struct alignas(8) PathRec { float tr, tg, tb; uint32_t wid, rng, pad; };
static_assert(sizeof(PathRec) == 24, "PathRec layout");
#else
struct alignas(16) RayRec { double ox, oy, oz, dx, dy, dz; };                 // 48 B
#endif
// depth >= 1: throughput, work id, draw counter (32 B).  The depth is not
// stored: every path of a wavefront iteration has the iteration's depth.
#ifndef RT_F32_RECORDS
struct alignas(8) PathRec { double tr, tg, tb; uint32_t wid, rng; };
static_assert(sizeof(PathRec) == 32, "PathRec layout");
#endif
struct PathState {
    RayRec* ray;          // origin, direction
    PathRec* path;        // depth >= 1: throughput, work id, draw counter
    double* tm;           // depth 0: time
    uint32_t* rng0;       // depth 0: draw counter
};
// The hit queues, one per material type: one record per ray that hit
// something, appended by the closest-hit kernels in (block-)compaction order —
// distance t, leaf id and the path's slot in the state pool — so a shade
// kernel reads its queue front to back (no gather of a separate hit array).
// Queue c starts at h + c * stride.
struct alignas(16) HitRec { double t; int32_t leaf; uint32_t slot; };
struct HitBuf { HitRec* h; uint32_t stride; };

// Sharded queues.  Stream compaction appends through one atomic per block
// and class on a counter chosen by blockIdx % kShards (8 XCDs), so no single
// counter word serialises the chip; shard x of a queue holds counts[x] entries
// at [x*cap, x*cap + counts[x]).  Consumers see a virtual index space
// 0..sum(counts)-1 (QView; counts == nullptr means "contiguous").
constexpr int kShards = 8;
// Counter k of a counter array lives at [k * kCntStride] (uint32 units): each
// shard counter gets its own 128-B line, so the shards' atomics do not meet
// in one L2 line.
#ifndef RT_CNT_STRIDE
#define RT_CNT_STRIDE 32
#endif
constexpr int kCntStride = RT_CNT_STRIDE;
struct QView { const uint32_t* counts; uint32_t cap; };

// The fused curve extend's hand-off records (DevScene::fuse_ring).  A lane whose ray is resolved parks
// its hit (slot, leaf + 1 with the path depth above it, closest t); once a wave has 64 parked, every lane
// shades one (a whole-wave round) and the paths that go on are listed as ready (slot, depth) for the next
// free lanes.  A wave owns at most 64 walking + 63 parked paths when it claims new ones (and claims only
// with no ready path left), so 128 entries per ring cannot overflow; kFuseRing leaves a margin.
struct alignas(16) FuseHit { uint32_t slot, leaf_dep; double t; };      // leaf_dep = (leaf + 1) | depth << 25
struct alignas(8) FuseReady { uint32_t slot, depth; };
constexpr int kFuseRing = 256;
constexpr size_t kFuseWaveBytes = (size_t)kFuseRing * (sizeof(FuseHit) + sizeof(FuseReady));
constexpr int kFuseLeafBits = 25;                                    // leaves below 2^25 - 1 (launch_extend checks)

// The fused curve extend's launch (launch_extend, k_extend_curves<FUSE>): every depth from `depth` on in
// one launch; continuation segments are counted into *segs
struct CurveFuse {
    unsigned long long* segs;
    uint32_t depth;
};

// Per-render-chunk parameters shared by the kernels.
struct RenderParams {
    uint32_t nx, ny;
    uint32_t npix;            // pixels of this shard
    uint32_t spp0;            // absolute sample index of the chunk's first sample
    uint32_t k0, k1;          // RNG key (seed)
    const uint32_t* pixlist;  // shard pixel q -> image pixel j
    double* sb;               // sample colours [B][3] (one rgb record per work id), B = npix * chunk_spp
    uint32_t B;
    uint32_t compact;         // accumulator indexed by shard pixel q (rt_render_shard_device), not image pixel j
    uint32_t exact_libm;      // host side: lambertian bounce directions with rt_libm.h's sin / cos (RT_OPT_EXACT_LIBM;
                              // launch_shade / launch_finish pick the kernel instance by it)
    double inx, iny;          // RN(1/nx), RN(1/ny): trace-all's (/ (+ i r) nx) as div_ia (rt_kernels.hip)
};

}  // namespace rtamd
