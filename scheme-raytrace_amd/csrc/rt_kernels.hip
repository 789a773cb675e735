// rt_kernels.hip — CDNA4 (gfx950) wavefront path-tracing kernels.
//
// The reference's recursive `color` (main.scm:100-121) becomes an iterative
// wavefront over a pool of paths kept SoA in HBM:
//
//   k_raygen    trace-all jitter + cam:get-ray      main.scm:476-478, camera.scm:80-92
//   k_extend<F> closest hit over the flattened       geometry.scm:14-56,146-215,376-673,
//               object tree (one segment per path):  bezier.scm:13-223; main.scm:91-95,120
//               per-lane BVH traversal, brute-force
//               groups, wave-batched curve tests;
//               misses finish with the sky, hits are
//               appended to per-material queues
//   k_shade<M>  hit record + material M's scatter /  material.scm:15-111, texture.scm,
//               emission; survivors compacted with   perlin.scm, pdf.scm (f2), main.scm:100-121
//               a wave64 ballot + mbcnt prefix, an
//               LDS scan and one atomic per block
//   k_finish<F> the depth tail: extend+shade looped  (same code; persistent lanes refill
//               per lane for the last paths           from the remaining path list)
//   k_accumulate per-pixel running sum in sample     main.scm:480,488
//               order (deterministic, no atomics)
//   k_resolve_u8 correct-gamma + quantise            main.scm:481-491
//
// F selects the closest-hit features compiled in (kFeatCurves: curve batching
// state; kFeatExtra: constant media and Klein limit sets, which draw random
// numbers / march inside the hit test), so sphere scenes run lean kernels.
//
// All arithmetic is f64 like the reference's flonums.  Random numbers come
// from a Philox4x32-10 stream keyed by (seed, pixel, sample) with a per-path
// draw counter, consumed in the reference's order.
#include <hip/hip_runtime.h>
#include "rt_device.h"
#include "rt_libm.h"
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace rtamd {

// --------------------------------------------------------------- faults
// Device fault word (one per device).  Every loop that waits on data — the
// rejection samplers, the curve subdivision walk, the persistent kernels'
// per-path / per-ray loops — carries an iteration cap that a valid stream
// cannot reach; a kernel that hits one, or would append past a queue shard,
// sets a bit here and leaves the loop instead of hanging the device.
// render_impl reads and clears the word after every render and fails the
// call with rt_last_error naming the bits (rt_api.cpp fault_text).
__device__ unsigned int g_fault;
__device__ __forceinline__ void raise_fault(const unsigned int bit) { atomicOr(&g_fault, bit); }
constexpr int kRejectCap = 4096;               // rejection sampler attempts (P(reject) <= 0.48 per attempt)
// the cap the samplers use: kRejectCap unless a test lowers it (RTAMD_REJECT_CAP, set_test_caps) to
// drive the fault path of a real sampler loop without a degenerate stream
__device__ int g_reject_cap = kRejectCap;
// k_extend_curves' per-ray iteration cap; 0 = the scene's bound (tests lower it: RTAMD_CURVE_RAY_CAP)
__device__ uint32_t g_curve_ray_cap = 0;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;      // block_append / wave_append: the shard is full

// ------------------------------------------------------------------ RNG
__device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                         uint32_t k0, uint32_t k1) {
    // Philox4x32-10: ten rounds define the stream the oracle restates
    // (oracle/rt_oracle.c philox4x32_10); no build may change them
    constexpr int kPhiloxRounds = 10;
#pragma unroll
    for (int r = 0; r < kPhiloxRounds; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        // one 32x32->64 product per word (v_mad_u64_u32) instead of separate
        // low / high multiplies: 1.36x the Philox rate (tools micro-benchmark)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
}

// (hi,lo) -> (2k+1)*2^-53 with k = (hi>>12)<<32 | lo; every step is exact.
__device__ __forceinline__ double u32pair_unit(uint32_t hi, uint32_t lo) {
    const double k = (double)(hi >> 12) * 4294967296.0 + (double)lo;
    return (k * 2.0 + 1.0) * (1.0 / 9007199254740992.0);
}

struct Rng {
    uint32_t k0, k1, pix, smp, ctr, blk, w0, w1, w2, w3;
    __device__ __forceinline__ void init(uint32_t a, uint32_t b, uint32_t p, uint32_t s, uint32_t c) {
        k0 = a; k1 = b; pix = p; smp = s; ctr = c; blk = 0xFFFFFFFFu;
    }
    // srfi-27 random-real replacement: draw number `ctr` of the path's stream
    __device__ __forceinline__ double next() {
        const uint32_t d = ctr++;
        const uint32_t b = d >> 1;
        if (b != blk) {
            uint32_t c0 = b, c1 = smp, c2 = pix, c3 = 0u;
            philox10(c0, c1, c2, c3, k0, k1);
            w0 = c0; w1 = c1; w2 = c2; w3 = c3; blk = b;
        }
        return (d & 1u) ? u32pair_unit(w2, w3) : u32pair_unit(w0, w1);
    }
};

// x / a, correctly rounded, from ia = RN(1/a) (one true division per ray
// instead of one per root).  q0 = RN(x*ia) is within 1.5 ulp of x/a; one
// residual step makes it faithful, and the second is Markstein's: with ia =
// RN(1/a), q1 faithful and the residual x - a*q1 exact (fma), RN(q1 + r*ia)
// = RN(x/a).  So the quotient is the IEEE one the reference's `/` gives,
// for every a the scenes produce (|d|^2 far from the f64 under/overflow
// range); 5 f64 ops instead of the 11-op division sequence.
__device__ __forceinline__ double div_ia(const double x, const double a, const double ia) {
    const double q0 = x * ia;
    const double q1 = fma(fma(-q0, a, x), ia, q0);
    return fma(fma(-q1, a, x), ia, q1);
}

// ------------------------------------------------------------ vec.scm
// sin / cos as the reference's libm computes them (rt_libm.h); OCML beyond the
// reference algorithm's reduction range (|x| >= 0x1.921fbp+26 = 105414336, inf, nan)
__device__ __forceinline__ double rt_sin(const double x) { return rtlibm::sin_full(x); }
__device__ __forceinline__ double rt_cos(const double x) { return rtlibm::cos_full(x); }
// cos(a) and sin(b), one evaluation after the other: inlined side by side, the two would hold their
// temporaries at once (the shade kernels' register budget).  Bounce angles only: a, b = 2 pi u with u in
// (0, 1) lie inside the restated reduction range (rtlibm::in_range), so the platform fallback that
// sincos_full carries for huge arguments (the device library's Payne-Hanek path) is not compiled in —
// it cost the lambertian shade 27 VGPRs (154 vs 127, 3 waves instead of 4)
__device__ __forceinline__ void rt_cos_sin(const double a, const double b, double& c, double& s, const double* tab) {
    double v0 = 0.0, v1 = 0.0;
#pragma unroll 1
    for (int j = 0; j < 2; ++j) {
        const double v = rtlibm::sincos_(j == 0 ? a : b, j == 0, tab);
        if (j == 0) v0 = v; else v1 = v;
    }
    c = v0;
    s = v1;
}
// The bounce directions' cos / sin (random-cosine-direction, util.scm:37-44; the light mixture's
// random-to-sphere): EX = libm's own bits (rt_libm.h), else OCML's (within 1 ulp).  The render's
// RT_OPT_EXACT_LIBM picks the kernel instance (RenderParams::exact_libm); by default scenes with curves
// take EX: a grazing ribbon hit turns a 1-ulp direction change into another path (the dense flat-curve
// test); elsewhere OCML's ulps move pixels by ~1e-16 (C2 band RMS 1.6e-13, a few horizon pixels by up
// to 1e-6) and EX costs C2 ~4.5 % (profiles/r04/ab_libm_c2.log).  Marble textures use rt_libm.h in
// every scene (checker_odd needs only a sine's sign).
template <bool EX>
__device__ __forceinline__ void bounce_cos_sin(const double a, const double b, double& c, double& s, const double* tab) {
    if (EX) {
        rt_cos_sin(a, b, c, s, tab);
    } else {
        c = cos(a);
        s = sin(b);
    }
}
struct v3 { double x, y, z; };
__device__ __forceinline__ v3 mk(double x, double y, double z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 operator*(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 operator*(v3 a, double k) { return mk(a.x * k, a.y * k, a.z * k); }
__device__ __forceinline__ double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double length(v3 a) { return sqrt(dot(a, a)); }
__device__ __forceinline__ v3 unit(v3 a) { const double k = 1.0 / length(a); return a * k; }
#ifdef RT_F32_RECORDS
__device__ __forceinline__ RayRec ray_rec(const v3 o, const v3 d) {
    return RayRec{(float)o.x, (float)o.y, (float)o.z, (float)d.x, (float)d.y, (float)d.z};
}
__device__ __forceinline__ PathRec path_rec(const v3 T, const uint32_t wid, const uint32_t rng) {
    return PathRec{(float)T.x, (float)T.y, (float)T.z, wid, rng, 0u};
}
#else
__device__ __forceinline__ RayRec ray_rec(const v3 o, const v3 d) { return RayRec{o.x, o.y, o.z, d.x, d.y, d.z}; }
__device__ __forceinline__ PathRec path_rec(const v3 T, const uint32_t wid, const uint32_t rng) {
    return PathRec{T.x, T.y, T.z, wid, rng};
}
#endif
__device__ __forceinline__ v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}

// --------------------------------------------------------- instancing
// translate (geometry.scm:467-469) and rotate-y (:512-522): ray into the
// instance, outermost op first.
__device__ __forceinline__ void chain_ray(const Chain& c, v3& o, v3& d) {
    for (int k = 0; k < c.n; ++k) {
        const ChainOpRec& op = c.ops[k];
        if (op.op == OP_TRANSLATE) {
            o = o - mk(op.x, op.y, op.z);
        } else {
            const double sn = op.x, cs = op.y;
            o = mk(cs * o.x - sn * o.z, o.y, sn * o.x + cs * o.z);
            d = mk(cs * d.x - sn * d.z, d.y, sn * d.x + cs * d.z);
        }
    }
}
// hit record back out of the instance (:473, :526-535), innermost op first.
__device__ __forceinline__ void chain_hit(const Chain& c, v3& p, v3& n) {
    for (int k = c.n - 1; k >= 0; --k) {
        const ChainOpRec& op = c.ops[k];
        if (op.op == OP_TRANSLATE) {
            p = p + mk(op.x, op.y, op.z);
        } else {
            const double sn = op.x, cs = op.y;
            p = mk(cs * p.x + sn * p.z, p.y, (-sn) * p.x + cs * p.z);
            n = mk(cs * n.x + sn * n.z, n.y, (-sn) * n.x + cs * n.z);
        }
    }
}

// =====================================================================
// k_raygen — one camera sample per work item w = s_rel*npix + q
// =====================================================================
// trace-all's per-pixel jitter + cam:get-ray for work item w (main.scm:476-478,
// camera.scm:80-92); returns the ray and leaves g after its draws.
__device__ __forceinline__ void camera_ray(const DevScene& sc, const RenderParams& rp, const uint32_t w, v3& o, v3& d,
                                           double& time, Rng& g) {
    const uint32_t s_rel = w / rp.npix;
    const uint32_t q = w - s_rel * rp.npix;
    const uint32_t j = rp.pixlist[q];
    const uint32_t y = j / rp.nx, x = j - y * rp.nx;
    const uint32_t smp = rp.spp0 + s_rel;
    g.init(rp.k0, rp.k1, j, smp, 0u);
    // main.scm:476-477 (let* order: u then v)
    const double u = div_ia((double)x + g.next(), (double)rp.nx, rp.inx);
    const double v = div_ia((double)y + g.next(), (double)rp.ny, rp.iny);
    // camera.scm:80-92
    const DevCamera& c = sc.cam;
    v3 p;
    for (int it = 0;; ++it) {   // util.scm:17-23 random-in-unit-disk
        const double a = g.next(), b = g.next();
        p = mk(a * 2.0 - 1.0, b * 2.0 - 1.0, 0.0 * 2.0 - 0.0);
        if (dot(p, p) < 1.0) break;
        if (it >= g_reject_cap) { raise_fault(RT_FAULT_REJECT); p = mk(0.0, 0.0, 0.0); break; }
    }
    const v3 rd = p * c.lens;
    const v3 cu = mk(c.u[0], c.u[1], c.u[2]), cv = mk(c.v[0], c.v[1], c.v[2]);
    const v3 offset = cu * rd.x + cv * rd.y;
    time = c.t0 + g.next() * (c.t1 - c.t0);
    const v3 origin = mk(c.origin[0], c.origin[1], c.origin[2]);
    o = origin + offset;
    d = ((mk(c.llc[0], c.llc[1], c.llc[2]) + mk(c.hor[0], c.hor[1], c.hor[2]) * u) +
         mk(c.ver[0], c.ver[1], c.ver[2]) * v) - origin - offset;
}

__global__ __launch_bounds__(256) void k_raygen(const DevScene sc, const RenderParams rp,
                                                PathState st) {
    const uint32_t w = blockIdx.x * 256u + threadIdx.x;
    if (w >= rp.B) return;
    v3 o, d;
    double time;
    Rng g;
    camera_ray(sc, rp, w, o, d, time, g);
    st.ray[w] = ray_rec(o, d);                             // depth-0 state (rt_device.h PathState)
    st.tm[w] = time;
    st.rng0[w] = g.ctr;
}

// ---------------------------------------------------------- closest hit
// hit-obj-list semantics (geometry.scm:33-50): shrinking t-max, strict
// (tmin, closest) for spheres, non-strict for rects.  Every lane of a wave
// walks the same group / primitive sequence, so the primitive records are
// fetched once per wave through the scalar unit.
constexpr double kInvPi = 1.0 / kPi;           // RN(1/pi): (/ x pi) = div_ia(x, kPi, kInvPi)
// sphere test (geometry.scm:146-171); updates closest/best on a hit.
// a = (dot d d), ia = 1/a (div_ia)
__device__ __forceinline__ void sphere_test(const v3 o, const v3 d, const double a, const double ia, const v3 c,
                                            const double rr, const int32_t id, double& closest, int32_t& best) {
    const v3 oc = o - c;
    const double b = dot(oc, d);
    const double cc = dot(oc, oc) - rr;
    const double disc = b * b - a * cc;
    if (disc > 0.0) {
        const double sq = sqrt(disc);
        double t = div_ia(-b - sq, a, ia);
        if (!(kTmin < t && t < closest)) t = div_ia(-b + sq, a, ia);
        if (kTmin < t && t < closest) { closest = t; best = id; }
    }
}


// ------------------------------------------------------------- curves
// Cubic Bezier curve test (bezier.scm:13-214).  The ray is moved to a frame
// where it starts at the origin and runs along +z (get-projection-mat); the
// curve is subdivided at 0.5 down to a depth estimated from its flatness and
// each surviving leaf segment is intersected in the xy plane.  The reference's
// `converge` gives both children of a split the t it was called with, so the
// curve's answer is min z over all leaf hits with z <= t; the recursion
// becomes an explicit per-lane stack (private memory).
// rows 0..3, columns 0..2 of the 4x4 projection matrix without its entry (1, 0), which both branches of
// get-projection-mat make 0 (m[k] for k < 3, m[k - 1] after: 11 doubles in the wave's LDS per lane)
struct BezRay { double m[11]; };

__device__ __forceinline__ void bez_ray(const v3 o, const v3 d, BezRay& R) {
    const double ox = -o.x, oy = -(-o.z), oz = -o.y;
    const v3 rd = unit(d);
    const double lx = rd.x, ly = -rd.z, lz = rd.y;
    const double dd = sqrt(lx * lx + lz * lz);
    double r[9];
    if (dd == 0.0) {
        // ang = -pi/2 or pi/2: libm's cos / sin of those doubles (rt_libm.h), as constants
        const double cs = 0x1.1a62633145c07p-54, sn = (ly >= 0.0) ? -1.0 : 1.0;
        r[0] = 1.0; r[1] = 0.0; r[2] = 0.0;
        r[3] = 0.0; r[4] = cs;  r[5] = -sn;
        r[6] = 0.0; r[7] = sn;  r[8] = cs;
    } else {
        r[0] = lz / dd;   r[1] = (-1.0 * lx * ly) / dd; r[2] = lx;
        r[3] = 0.0;       r[4] = dd;                    r[5] = ly;
        r[6] = (-lx) / dd; r[7] = (-1.0 * ly * lz) / dd; r[8] = lz;
    }
    // array-mul with the translation: rows 0..2 are the rotation, row 3 = o' R
#pragma unroll
    for (int k = 0; k < 9; ++k) if (k != 3) R.m[k < 3 ? k : k - 1] = r[k];
#pragma unroll
    for (int j = 0; j < 3; ++j) R.m[8 + j] = ((ox * r[j] + oy * r[3 + j]) + oz * r[6 + j]) + 0.0;
}
// transform (bezier.scm:49-55): row vector (x, -z, y, 1) times the matrix
__device__ __forceinline__ v3 bez_xf(const BezRay& R, const double x, const double y, const double z) {
    const double a = x, b = -z, c = y;
    // b * 0.0 kept as an operation: it is -0 for negative b, and a * m0 + (-0) keeps a -0 product's sign
    return mk(((a * R.m[0] + b * 0.0) + c * R.m[5]) + R.m[8],
              ((a * R.m[1] + b * R.m[3]) + c * R.m[6]) + R.m[9],
              ((a * R.m[2] + b * R.m[4]) + c * R.m[7]) + R.m[10]);
}
struct Bez4 { v3 p0, p1, p2, p3; };
__device__ __forceinline__ v3 bez_point(const Bez4& c, const double t) {       // bez-p :67-77
    const double t2 = t * t, t3 = t2 * t;
    const double u = 1.0 - t, u2 = u * u, u3 = u2 * u;
    return ((c.p0 * u3 + c.p1 * (3.0 * u2 * t)) + c.p2 * (3.0 * u * t2)) + c.p3 * t3;
}
// internally-divide (:45-47) at t = 0.5 is (v:sum (v:scale a 0.5) (v:scale b 0.5)) = RN(a/2 + b/2): both
// halvings are exact (a power of two, outside the subnormal range), and RN((a + b) / 2) = RN(a + b) / 2 for the
// same reason, so (a + b) * 0.5 gives the same bits with one multiply less per component (15 per split;
// C5 at 8 spp +0.75 %, same image, profiles/r06/ab_halfsum/)
__device__ __forceinline__ v3 half_div(const v3 a, const v3 b) { return (a + b) * 0.5; }
// bez-p at t = 0.5: ((p0 0.125 + p1 0.375) + p2 0.375) + p3 0.125 (bez_point's products and sums).  The
// products by 0.125 are exact, RN(p 0.375) = RN(3 p) / 8, and RN(x / 8 + y / 8) = RN(x + y) / 8 (scaling by
// a power of two commutes with rounding outside the subnormal range): the same bits as
// RN(RN(RN(p0 + RN(3 p1)) + RN(3 p2)) + p3) / 8, one operation less per component
__device__ __forceinline__ v3 bez_mid(const Bez4& c) { return (((c.p0 + c.p1 * 3.0) + c.p2 * 3.0) + c.p3) * 0.125; }
__device__ __forceinline__ void bez_split(const Bez4& c, Bez4& l, Bez4& r) {    // split :78-87
    const v3 sp = bez_mid(c);
    const v3 nbc = half_div(c.p1, c.p2);
    const v3 lb = half_div(c.p0, c.p1);
    const v3 lc = half_div(lb, nbc);
    const v3 rc = half_div(c.p2, c.p3);
    const v3 rb = half_div(nbc, rc);
    l.p0 = c.p0; l.p1 = lb; l.p2 = lc; l.p3 = sp;
    r.p0 = sp; r.p1 = rb; r.p2 = rc; r.p3 = c.p3;
}
__device__ __forceinline__ v3 bez_tan(const Bez4& c, const bool one) {         // bez-tan-vec :106-117
    const v3 ca = ((c.p1 * 3.0 + c.p3) + c.p2 * -3.0) + c.p0 * -1.0;
    const v3 cb = ((c.p0 + c.p1 * -2.0) + c.p2) * 3.0;
    const v3 cc = (c.p1 - c.p0) * 3.0;
    const double k2 = one ? 3.0 : 0.0, k1 = one ? 2.0 : 0.0;
    return unit((ca * k2 + cb * k1) + cc);
}
__device__ __forceinline__ double dot2d(const v3 a, const v3 b) { return (a.x * b.x + a.y * b.y) + 0.0 * 0.0; }

__device__ __forceinline__ void bez_load(const BezierRec& B, const BezRay& R, Bez4& c) {   // bezier-transform :99-105
    c.p0 = bez_xf(R, B.cp[0], B.cp[1], B.cp[2]);
    c.p1 = bez_xf(R, B.cp[3], B.cp[4], B.cp[5]);
    c.p2 = bez_xf(R, B.cp[6], B.cp[7], B.cp[8]);
    c.p3 = bez_xf(R, B.cp[9], B.cp[10], B.cp[11]);
}
// bounding-box cull of converge (:123-128) against the ray-space cylinder
__device__ __forceinline__ bool bez_culled(const Bez4& c, const double w1, const double t) {
    const double zmn = fmin(fmin(c.p0.z, c.p1.z), fmin(c.p2.z, c.p3.z)) - w1;
    const double zmx = fmax(fmax(c.p0.z, c.p1.z), fmax(c.p2.z, c.p3.z)) + w1;
    const double xmn = fmin(fmin(c.p0.x, c.p1.x), fmin(c.p2.x, c.p3.x)) - w1;
    const double xmx = fmax(fmax(c.p0.x, c.p1.x), fmax(c.p2.x, c.p3.x)) + w1;
    const double ymn = fmin(fmin(c.p0.y, c.p1.y), fmin(c.p2.y, c.p3.y)) - w1;
    const double ymx = fmax(fmax(c.p0.y, c.p1.y), fmax(c.p2.y, c.p3.y)) + w1;
    return zmn >= t || zmx <= 0.000001 || xmn >= w1 || xmx <= -w1 || ymn >= w1 || ymx <= -w1;
}
// Hull culls (not in the reference; they change no result, only the work).
// converge reports a leaf hit only at a point p = (bez-p leaf v) with
// |p.xy|^2 < width2 (bezier.scm:156-164); v lies in [0, 1], so p is a convex
// combination of the leaf's control points, and every sub-curve's control
// points are convex combinations of its parent's (split, :78-87): p lies in
// the convex hull of every ancestor's control points.  A node whose hull (in
// the ray-space xy plane) stays farther than width1 from the ray axis
// therefore holds no hit, and neither walking it nor culling it changes the
// answer.  The box cull above keeps many such nodes (the box of a diagonal
// curve is mostly empty: at C5 two thirds of the root-box survivors).  The
// test is a separating axis: the normal of a hull edge along which every
// control point lies more than r from the origin.  The computed points drift
// from the exact sub-curves by a few ulps of their magnitude s per level (and
// bez-p by a few more), so r = width1 (1 + 1e-9) + 1e-9 s keeps the cull
// conservative by orders of magnitude; NaNs and a zero edge never cull.
#ifndef RT_BEZ_HULL
#define RT_BEZ_HULL 1
#endif
__device__ __forceinline__ bool bez_sep_axis(const Bez4& c, const v3 a, const v3 b, const double r2) {
    const double nx = a.y - b.y, ny = b.x - a.x;                 // normal of the edge a -> b
    const double d0 = fma(c.p0.x, nx, c.p0.y * ny), d1 = fma(c.p1.x, nx, c.p1.y * ny);
    const double d2 = fma(c.p2.x, nx, c.p2.y * ny), d3 = fma(c.p3.x, nx, c.p3.y * ny);
    const double mn = fmin(fmin(d0, d1), fmin(d2, d3)), mx = fmax(fmax(d0, d1), fmax(d2, d3));
    const double lim = r2 * fma(nx, nx, ny * ny);
    return (mn > 0.0 && mn * mn > lim) || (mx < 0.0 && mx * mx > lim);
}
// EDGES = 1: the chord p0 -> p3 only (the walk's splits: sub-curves are nearly
// straight); 4: the chord and the three legs of the control polygon (roots;
// the two diagonals as well cut C5's survivors by another ~10 % in a host
// simulation but cost more in stage A than they save: -1.2 % at 8 spp)
// r^2 for the control points c; a sub-curve's points are convex combinations of its root's (a few ulps
// aside), so the root's r bounds every node's and the walk computes it once (BezWalk::hr2)
__device__ __forceinline__ double bez_hull_r2(const Bez4& c, const double w1) {
    const double s = fmax(fmax(fmax(fabs(c.p0.x), fabs(c.p0.y)), fmax(fabs(c.p1.x), fabs(c.p1.y))),
                          fmax(fmax(fabs(c.p2.x), fabs(c.p2.y)), fmax(fabs(c.p3.x), fabs(c.p3.y))));
    const double aw = fabs(w1);         // a hit needs |p.xy|^2 < width2 = w1^2 (the ABI refuses widths <= 0)
    const double r = fma(aw, 1e-9, aw) + 1e-9 * s;
    return r * r;
}
template <int EDGES>
__device__ __forceinline__ bool bez_hull_sep(const Bez4& c, const double r2) {
    if (!RT_BEZ_HULL) return false;
    bool sep = bez_sep_axis(c, c.p0, c.p3, r2);
    if (EDGES > 1)
        sep = sep || bez_sep_axis(c, c.p0, c.p1, r2) || bez_sep_axis(c, c.p1, c.p2, r2) || bez_sep_axis(c, c.p2, c.p3, r2);
    return sep;
}
template <int EDGES>
__device__ __forceinline__ bool bez_hull_culled(const Bez4& c, const double w1) {
    return RT_BEZ_HULL && bez_hull_sep<EDGES>(c, bez_hull_r2(c, w1));
}
// converge's box cull plus the hull cull
template <int EDGES>
__device__ __forceinline__ bool bez_culled_hull(const Bez4& c, const double w1, const double t) {
    return bez_culled(c, w1, t) || bez_hull_culled<EDGES>(c, w1);
}

// The subdivision walk of converge (bezier.scm:121-175) as a per-lane state
// machine: one node per step, so the batched curve kernels (stage B) can hand
// a lane whose curve is finished the next survivor while the others keep
// walking; bezier_test runs it to the end.
//
// The answer does not depend on the order of the recursion: a leaf hit at
// z <= tmax lies on its sub-curve, inside every ancestor's box, so no
// ancestor culls it and converge's result is min z over all leaf hits with
// z <= tmax.  The walk therefore also culls with the best z found so far (it
// cannot hide a smaller z, and culling only gets stronger as the best z
// drops), which only removes work.
//
// Depth-first, without a stack: node (L, idx) is the sub-curve reached from
// the root by L splits at 0.5 taking the halves given by idx's bits (MSB
// first); its parameter range is [idx, idx + 1] * 2^-L.  A split culls both
// halves at once: the walk goes into the left half if it survives, else
// straight into the right one (already in registers), and remembers in rmask
// whether a left half's right sibling survived.  Only a right sibling that
// survived next to a surviving left half is revisited later, re-derived from
// the root by the same split sequence, so every sub-curve carries the exact
// values the reference's recursion computes.  (Keeping the deepest pending
// right half in registers instead cut the re-derivation splits per curve from
// 15 to 5 at C5, but the persistent curve kernel then spills: 120.6 vs 137.8
// Mrays/s at 4 spp.)
//
// The walk's calls: bez_walk_split (one split: a descent split, both halves
// culled, or one level of a right sibling's re-derivation from the root),
// bez_walk_node (a pending right sibling re-derived in one go, then split)
// and bez_walk_leaf (a leaf segment's test).  Stage B calls node / leaf, and
// holds lanes at leaf segments until enough of them test together
// (RT_BEZ_LEAF_PHASE); the per-lane bezier_test calls split / leaf.
// RING (k_extend_curves' stage B): the root is not held in registers — the walk re-reads it from the
// survivor's ring line when it re-derives a node (24 VGPRs less at the kernel's peak)
template <bool RING> struct BezRootOf { Bez4 root; };
template <> struct BezRootOf<true> { const Bez4* rootp; };
template <bool RING = false>
struct BezWalkT : BezRootOf<RING> {
    Bez4 c;
    double best, tmax, w1, w2;
    double hr2;                     // the hull cull's r^2 from the root (bez_hull_r2)
    int L, leaf_level, base;        // base: the level the walk started at (a donated subtree's root; else 0)
    int rl;                         // re-derivation (!fresh): c is the path node at level rl < L
    uint32_t idx, it, cap;
    uint32_t rmask;                 // bit L: the right sibling of the level-L left half was culled at the split
    int pl;                         // the level of the pending right sibling held in the lane's LDS slot (-1: none)
    bool fresh, found;              // fresh: c is node (L, idx) and passed the cull
};
using BezWalk = BezWalkT<false>;
template <bool RING>
__device__ __forceinline__ Bez4 bez_root(const BezWalkT<RING>& s) {
    if constexpr (RING) return *s.rootp;
    else return s.root;
}
// converge's subdivision depth from the transformed curve's flatness (:180-193)
__device__ __forceinline__ int bez_maxd(const Bez4& c, const double eps8) {
    double l0 = -kTmax;
    const double x0 = fabs((c.p0.x + -2.0 * c.p1.x) + c.p2.x), y0 = fabs((c.p0.y + -2.0 * c.p1.y) + c.p2.y);
    l0 = fmax(fmax(x0, y0), l0);
    const double x1 = fabs((c.p1.x + -2.0 * c.p2.x) + c.p3.x), y1 = fabs((c.p1.y + -2.0 * c.p2.y) + c.p3.y);
    l0 = fmax(fmax(x1, y1), l0);
    const double md = log((((1.4142135623730951 * 4.0) * 3.0) * l0) / eps8) / log(4.0);
    // saturates at kBezMaxDepth + 1: the caller faults on anything deeper than the walk supports
    return (md == -INFINITY) ? 0 : (md > (double)(kBezMaxDepth + 1) ? kBezMaxDepth + 1 : (int)ceil(md));
}
// set up the walk of root-transformed curve `root` for t-max tmax (the root
// has passed the cull) down to leaf level leaf_level = max(0, maxd + 1): a
// negative maxd (a flat curve) makes the root a leaf (:130, 189-193)
template <bool RING>
__device__ __forceinline__ void bez_walk_init(BezWalkT<RING>& s, const Bez4& root, const double w1, const double w2,
                                              const double tmax, const int leaf_level, const Bez4* rootp = nullptr) {
    if constexpr (RING) s.rootp = rootp;
    else s.root = root;
    s.c = root;
    s.w1 = w1; s.w2 = w2; s.tmax = tmax;
    s.hr2 = bez_hull_r2(root, w1);
    s.leaf_level = leaf_level;
    // each of the <= 2^(leaf_level+1) nodes is visited at most once, for at
    // most leaf_level re-derivation splits and one split or leaf test
    s.cap = (uint32_t)(s.leaf_level + 2) << (s.leaf_level + 1);
    s.L = 0; s.base = 0; s.rl = 0; s.idx = 0; s.it = 0; s.rmask = 0; s.pl = -1;
    s.fresh = true; s.found = false; s.best = tmax;
}
// at a leaf segment: the next call is bez_walk_leaf
template <bool RING>
__device__ __forceinline__ bool bez_walk_at_leaf(const BezWalkT<RING>& s) { return s.fresh && s.L >= s.leaf_level; }
// set up the walk of curve B for t-max tmax, whose leaf level (maxd + 1, from
// stage A's root cull) is given; false if the whole curve is culled
__device__ __forceinline__ bool bez_walk_begin(BezWalk& s, const BezierRec& B, const BezRay& R, const double tmax,
                                               const int leaf_level) {
    Bez4 root;
    bez_load(B, R, root);
    if (bez_culled(root, B.w1, tmax)) return false;
    bez_walk_init(s, root, B.w1, B.w2, tmax, leaf_level);
    return true;
}
// past the current node: climb past right halves and past left halves whose
// right sibling was culled at the split, then aim at the surviving right
// sibling (re-derived from the root); true once the walk is over
template <bool RING>
__device__ __forceinline__ bool bez_walk_next(BezWalkT<RING>& s) {
    while (s.L > s.base && ((s.idx & 1u) || ((s.rmask >> s.L) & 1u))) { --s.L; s.idx >>= 1; }
    if (s.L == s.base) return true;
    ++s.idx;
    if constexpr (!RING) s.c = s.root;              // (RING walks re-derive in bez_walk_node only)
    s.rl = 0; s.fresh = false;
    return false;
}
// one split (not at a leaf: !bez_walk_at_leaf); true once the walk is over
// slot (stage B only; nullptr in the per-lane walk): the lane's LDS copy of the latest pending right
// sibling.  Depth first, that sibling is the next pending node the walk turns to (every later one lies in
// its left brother's subtree and is visited first), so the walk takes it from the slot instead of
// re-deriving it from the root, bit for bit the same values; older ones are overwritten and re-derived.
template <bool SLOT = false, bool RING = false>
__device__ __forceinline__ bool bez_walk_split(BezWalkT<RING>& s, Bez4* slot = nullptr) {
    if (++s.it > s.cap + 1u) { raise_fault(RT_FAULT_CURVE); return true; }
    Bez4 l, r;
    bez_split(s.c, l, r);                                       // split, left first (:167-175)
    if (!s.fresh) {                                             // one level toward the right sibling (L, idx)
        const bool right = (s.idx >> (s.L - 1 - s.rl)) & 1u;
        s.c = right ? r : l;
        if (++s.rl < s.L) return false;
        if (!bez_culled(s.c, s.w1, s.best)) { s.fresh = true; return false; }  // it survives the cull: visit it
        return bez_walk_next(s);                                // (its hull passed at its first split)
    }
    // (:123-128) with the best z so far
    const bool kl = !(bez_culled(l, s.w1, s.best) || bez_hull_sep<1>(l, s.hr2));
    const bool kr = !(bez_culled(r, s.w1, s.best) || bez_hull_sep<1>(r, s.hr2));
    if (kl || kr) {
        ++s.L;
        if (kl) {
            s.c = l; s.idx <<= 1;
            s.rmask = kr ? (s.rmask & ~(1u << s.L)) : (s.rmask | (1u << s.L));
            if (SLOT && kr) { *slot = r; s.pl = s.L; }
        } else {
            s.c = r; s.idx = (s.idx << 1) | 1u;
        }
        return false;
    }
    return bez_walk_next(s);
}
// one node (not at a leaf): a pending right sibling is re-derived from the
// root in one go, then split; true once the walk is over
template <bool SLOT = false, bool RING = false>
__device__ __forceinline__ bool bez_walk_node(BezWalkT<RING>& s, Bez4* slot = nullptr) {
    if (!s.fresh) {
        if (++s.it > s.cap + 1u) { raise_fault(RT_FAULT_CURVE); return true; }
        if (SLOT && s.pl == s.L) {                              // the pending sibling kept in the slot
            s.c = *slot;
            s.pl = -1;
        } else {
            s.c = bez_root(s);
            for (int k = s.L - 1; k >= 0; --k) {
                Bez4 l, r;
                bez_split(s.c, l, r);
                s.c = ((s.idx >> k) & 1u) ? r : l;
            }
        }
        if (bez_culled(s.c, s.w1, s.best)) return bez_walk_next(s);
        s.rl = s.L;
        s.fresh = true;
        if (s.L >= s.leaf_level) return false;                  // a leaf: tested in a leaf phase
    }
    return bez_walk_split<SLOT>(s, slot);
}
// the leaf segment's test (:130-166) (bez_walk_at_leaf); true once the walk is over
template <bool RING>
__device__ __forceinline__ bool bez_walk_leaf(BezWalkT<RING>& s) {
    if (++s.it > s.cap + 1u) { raise_fault(RT_FAULT_CURVE); return true; }
    const Bez4& c = s.c;
    const double v0 = ldexp((double)s.idx, -s.L), vn = v0 + ldexp(1.0, -s.L);
    const v3 dir = c.p3 - c.p0;
    v3 dp0 = bez_tan(c, false);
    if (dot2d(dir, dp0) < 0.0) dp0 = dp0 * -1.0;
    if (!(dot2d(dp0, c.p0 * -1.0) < 0.0)) {
        v3 dpn = bez_tan(c, true);
        if (dot2d(dir, dpn) < 0.0) dpn = dpn * -1.0;
        if (!(dot2d(dpn, c.p3) < 0.0)) {
            double w = dir.x * dir.x + dir.y * dir.y;
            if (w != 0.0) {
                w = (c.p0.x * dir.x + c.p0.y * dir.y) / (-w);
                w = (w < 0.0) ? 0.0 : ((w > 1.0) ? 1.0 : w);
                const double v = v0 * (1.0 - w) + vn * w;
                const v3 p = bez_point(c, v);                   // sub-curve at the global v (Q11)
                if (!(p.x * p.x + p.y * p.y >= s.w2 || p.z <= 0.0001 || s.tmax < p.z)) {
                    if (!s.found || p.z < s.best) s.best = p.z;
                    s.found = true;
                }
            }
        }
    }
    return bez_walk_next(s);
}
// one call of the walk (a leaf test or a split); true once the walk is over
__device__ __forceinline__ bool bez_walk_step(BezWalk& s) {
    return bez_walk_at_leaf(s) ? bez_walk_leaf(s) : bez_walk_split(s);
}

// Work sharing: the right siblings still pending on a walk's path (levels
// base+1 .. L whose path node is a left half whose right sibling survived its
// split), as a bit mask by level.
template <bool RING>
__device__ __forceinline__ uint32_t bez_walk_pending(const BezWalkT<RING>& s) {
    // level l's path node is a left half iff bit L - l of idx is 0: bit-reverse the complement so that
    // bit becomes bit l, keep levels base+1 .. L, drop the siblings culled at their split
    const uint32_t left = __builtin_bitreverse32(~s.idx & ((1u << s.L) - 1u)) >> (31 - s.L);
    return left & ~((2u << s.base) - 1u) & ~s.rmask;
}
// Hand the shallowest pending right sibling to another lane: returns its
// (level, index); this walk will skip it.
template <bool RING>
__device__ __forceinline__ void bez_walk_donate(BezWalkT<RING>& s, const uint32_t pend, uint32_t& l, uint32_t& ridx) {
    l = (uint32_t)__builtin_ctz(pend);
    ridx = (s.idx >> ((uint32_t)s.L - l)) | 1u;
    s.rmask |= 1u << l;
    if (s.pl == (int)l) s.pl = -1;                              // it is not this walk's any more
}
// A root-culled curve as stage A leaves it for stage B (k_extend_curves' survivor ring): the
// ray-space control points and the widths, so a refill reads 128 B the wave wrote itself (an L2 hit)
// instead of the curve record and the owner's matrix, and does not transform again
struct alignas(16) BezRoot { Bez4 c; double w1, w2, pad0, pad1; };
static_assert(sizeof(BezRoot) == 128, "BezRoot is one 128-B line");
__device__ __forceinline__ bool bez_walk_begin_root(BezWalkT<true>& s, const BezRoot& R, const double tmax,
                                                    const int leaf_level) {
    const Bez4 root = R.c;
    const double w1 = R.w1, w2 = R.w2;
    if (bez_culled(root, w1, tmax)) return false;
    bez_walk_init(s, root, w1, w2, tmax, leaf_level, &R.c);
    return true;
}
__device__ __forceinline__ void bez_walk_take_root(BezWalkT<true>& s, const BezRoot& R, const double tmax,
                                                   const int leaf_level, const uint32_t l, const uint32_t ridx) {
    bez_walk_init(s, R.c, R.w1, R.w2, tmax, leaf_level, &R.c);
    s.L = (int)l; s.base = (int)l; s.idx = ridx; s.fresh = false;
}
// Start a walk of the donated subtree rooted at node (l, ridx) of curve B
// (re-derived from the root at the first step; the walk ends back at level l).
__device__ __forceinline__ void bez_walk_take(BezWalk& s, const BezierRec& B, const BezRay& R, const double tmax,
                                              const int leaf_level, const uint32_t l, const uint32_t ridx) {
    Bez4 root;
    bez_load(B, R, root);
    bez_walk_init(s, root, B.w1, B.w2, tmax, leaf_level);
    s.L = (int)l; s.base = (int)l; s.idx = ridx; s.fresh = false;
}

// Returns true and the curve's t if it reports a hit for t-max `tmax`
// (bezier.scm:176-214): the root cull, the depth estimate, then the walk.
__device__ __forceinline__ bool bezier_test(const BezierRec& B, const BezRay& R, const double tmax, double& tout) {
    Bez4 c;
    bez_load(B, R, c);
    if (bez_culled_hull<4>(c, B.w1, tmax)) return false;
    const int maxd = bez_maxd(c, B.eps8);
    // converge has no depth limit (bezier.scm:189-193); a curve needing more
    // levels than the walk's 32-bit node index holds fails the render loudly
    if (maxd > kBezMaxDepth) { raise_fault(RT_FAULT_CURVE); return false; }
    BezWalk wk;
    bez_walk_init(wk, c, B.w1, B.w2, tmax, maxd + 1 > 0 ? maxd + 1 : 0);
    while (!bez_walk_step(wk)) {}
    if (!(wk.found && kTmin < wk.best)) return false;           // :201
    tout = wk.best;
    return true;
}

#ifdef RT_STATS
// traversal statistics (stats builds only): rays, node visits, leaf visits,
// sphere tests, moving-sphere tests, lane inner / outer loop iterations,
// waves, wave-max inner / outer iterations, lanes; [0..10] all-times tree,
// [16..26] time-0 tree; curve trees: [11] rays, [12] node visits, [13] leaf
// visits, [14] queued curve candidates, [15] root-cull survivors, [27] flushes,
// [28] wave loop iterations, [29] waves, [30] lanes
__device__ unsigned long long g_stats[48];
#define RT_STAT(k, v) atomicAdd(&g_stats[k], (unsigned long long)(v))
#else
#define RT_STAT(k, v) ((void)0)
#endif

// ------------------------------------------------- curve candidate batching
// Curve tests are long and their length varies per (ray, curve), so testing
// a curve in the lane that reached its BVH leaf leaves most of the wave idle.
// Instead the lanes of a wave traverse independently and append (curve,
// owner lane) candidates to a wave-local LDS queue; when 64 have gathered the
// wave tests them together: first the cheap root cull for every candidate,
// then the full subdivision for the survivors only, each lane taking one
// pair.  Per owner the smallest z wins; on a tie the later curve of the list
// (BezierRec::order), as hit-obj-list's scan reports a curve at
// z <= t-max (geometry.scm:41-46, bezier.scm:164) — bez_take_batch.  A
// curve's answer does not depend on the t-max it is tested with, beyond
// being reported only when z <= t-max (see bezier_test), so deferring the
// tests changes no result.
#ifndef RT_BEZ_REFILL
#define RT_BEZ_REFILL 8
#endif
constexpr int kBezRefill = RT_BEZ_REFILL;   // stage B: idle lanes that take the next survivors together
#ifndef RT_BEZ_DONATE
#define RT_BEZ_DONATE 16               // stage B: idle lanes (at least) that take pending subtrees together (0 = none)
#endif
#ifndef RT_BEZ_WAIT_FLUSH
#define RT_BEZ_WAIT_FLUSH 0            // k_extend_curves: lanes waiting on their curves that force a batch (0 = off)
#endif
#ifndef RT_BEZ_SLOT
#define RT_BEZ_SLOT 1                  // stage B: an LDS slot per lane for its latest pending right sibling
#endif
#ifndef RT_BEZ_QFLUSH
#define RT_BEZ_QFLUSH 48               // k_extend_curves: queued candidates that trigger a batch (stage A)
#endif
constexpr int kBezQ = (RT_BEZ_QFLUSH > 64 ? RT_BEZ_QFLUSH : 64) + 64;   // < the trigger before a step, + 1 per lane per step
#ifndef RT_BEZ_HOLD
#define RT_BEZ_HOLD 64                 // stage B runs once this many root-cull survivors wait (multiple of 64)
#endif
#ifndef RT_BEZ_LEAF_PHASE
#define RT_BEZ_LEAF_PHASE 40           // stage B: lanes at a leaf segment that test together
#endif
#ifndef RT_CURVE_FINISH_BATCH
#define RT_CURVE_FINISH_BATCH 20       // k_extend_curves: finished lanes written out and refilled together
#endif
constexpr int kBezS = RT_BEZ_HOLD + kBezQ;   // survivors: < RT_BEZ_HOLD carried over + one stage A's worth
static_assert(kBezS <= kBezRing && (kBezRing & (kBezRing - 1)) == 0,
              "k_extend_curves' survivor ring holds every survivor a wave can hold (slot = rtail + position)");
static_assert(2 * 64 <= kBezQ, "stage B's donation handover: two words per donor lane in W.q");
static_assert(kBezMaxDepth + 1 < 26, "the handover packs a level (6 bits) above a node index (26 bits)");
template <bool SLOT_>
struct BezWaveT {
    static constexpr bool SLOT = SLOT_;
    BezRay ray[64];                 // owner lane's ray-space matrix
    double cl[64];                  // owner's closest t when a batch runs
    double hz[64];                  // owner's best curve z from the batch
    unsigned long long hkey[64];    // and its curve: list order << 32 | curve index (ties: the later curve)
    uint32_t q[kBezQ];              // candidates: curve << 6 | owner
    uint32_t sv[kBezS];             // root-test survivors waiting for subdivision
    double sz[kBezS];               // their results (z or +inf)
    uint32_t done[64];              // persistent kernel: owner's candidates resolved so far
    Bez4 pend[SLOT_ ? 64 : 1];      // stage B: each lane's latest pending right sibling (bez_walk_split)
    uint8_t lev[kBezS];             // survivors' subdivision leaf levels (stage A)
};
using BezWave = BezWaveT<RT_BEZ_SLOT != 0>;
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Stage A: root cull of the qn queued candidates; survivors are appended to
// the survivor list (svn entries already there).  Returns the new count.
// Every active lane calls it with the same arguments.
// TRACK (k_extend_curves): survivors also go to the wave's ring (slot rtail + position, mod kBezRing)
template <bool TRACK = false, class WV = BezWave>
__device__ __forceinline__ uint32_t bez_stage_a(const DevScene& sc, WV& W, const uint32_t qn, uint32_t svn,
                                                BezRoot* __restrict__ ring = nullptr, const uint32_t rtail = 0u) {
    const unsigned long long act = __ballot(1);
    const uint32_t nact = (uint32_t)__popcll(act), rank = lanes_below(act);
    for (uint32_t base = 0; base < qn; base += nact) {
        const uint32_t i = base + rank;
        bool keep = false;
        uint32_t e = 0;
        uint8_t lev = 0;
        Bez4 c;
        if (i < qn) {
            e = W.q[i];
            const BezierRec& B = sc.bez[e >> 6];
            bez_load(B, W.ray[e & 63u], c);
            keep = !bez_culled_hull<4>(c, B.w1, W.cl[e & 63u]);
            // leaf level maxd + 1, at least 0: a flat curve's maxd is negative (its root is a leaf);
            // converge has no depth limit (bezier.scm:189-193): deeper than the walk supports fails loudly
            if (keep) {
                const int maxd = bez_maxd(c, B.eps8);
                if (maxd > kBezMaxDepth) { raise_fault(RT_FAULT_CURVE); keep = false; }
                else lev = (uint8_t)max(0, maxd + 1);
            }
            if (TRACK && !keep) atomicAdd(&W.done[e & 63u], 1u);
        }
        const unsigned long long m = __ballot(keep);
        if (keep) {
            const uint32_t pos = svn + lanes_below(m);
            W.sv[pos] = e; W.lev[pos] = lev;
            if (TRACK) {
                const BezierRec& B = sc.bez[e >> 6];
                ring[(rtail + pos) & (uint32_t)(kBezRing - 1)] = BezRoot{c, B.w1, B.w2, 0.0, 0.0};
            }
        }
        svn += (uint32_t)__popcll(m);
#ifdef RT_STATS
        if (rank == 0) RT_STAT(15, __popcll(m));
#endif
    }
    wave_sync();
    return svn;
}

// Stage B: full subdivision of the first nb survivors, one per lane, then per
// owner the smallest z (ties: the later curve of the list) into hz / hkey; the
// remaining svn - nb survivors move to the front.
// Pooled-curve counters (rt_stats.curve_pooled_batches / curve_flat_pooled):
// stage B passes over a full pool (>= RT_BEZ_HOLD survivors), and the
// survivors they walked whose root is already a leaf (a flat curve: converge's
// depth estimate is negative, bezier.scm:130,189-193).  One atomic per pass;
// read and cleared by take_curve_stats.
__device__ unsigned long long g_curve_stats[2];
template <bool TRACK = false, class WV = BezWave>
__device__ __forceinline__ void bez_stage_b(const DevScene& sc, WV& W, const uint32_t nb, const uint32_t svn,
                                            const BezRoot* __restrict__ ring = nullptr, const uint32_t rtail = 0u) {
    const unsigned long long act = __ballot(1);
    const uint32_t nact = (uint32_t)__popcll(act), rank = lanes_below(act);
    if (nb >= (uint32_t)RT_BEZ_HOLD) {
        uint32_t flat = 0;
        for (uint32_t base = 0; base < nb; base += nact)
            flat += (uint32_t)__popcll(__ballot(base + rank < nb && W.lev[base + rank] == 0));
        if (rank == 0) {
            atomicAdd(&g_curve_stats[0], 1ull);
            if (flat) atomicAdd(&g_curve_stats[1], (unsigned long long)flat);
        }
    }
    // Lanes take survivors one after the other from a wave-uniform cursor and
    // walk them a node per iteration (BezWalk): when at least kBezRefill
    // lanes are idle they take the next survivors together, so a lane is not
    // held by the longest walk of a fixed batch of 64.  Once the survivors are
    // all taken, idle lanes take pending right siblings (subtrees) from the
    // lanes still walking.  A survivor's z is the minimum over every lane
    // that walked part of it (atomicMin on the bits of the positive doubles),
    // then converge's (< t-min t) check (:201).
    {
        BezWalkT<TRACK> wk;
        bool busy = false;
        uint32_t si = 0, cursor = 0;
#ifdef RT_STATS
        // [31] passes [32] wave iterations [33] busy lane-iterations [34] walk steps [35] re-derived
        // nodes [36] re-derivation splits [37] leaf tests [38] survivors [39] stage B clock (lane 0)
        uint32_t n_it = 0, n_busy = 0, n_step = 0, n_red = 0, n_rsplit = 0, n_leaf = 0;
        unsigned long long n_clk_refill = 0;          // [45] stage B clock in refill / donation rounds (lane 0)
        unsigned long long n_clk_leaf = 0, n_clk_node = 0;   // [46] leaf tests, [47] node steps (splits, re-derivation)
        const unsigned long long clk0 = __builtin_amdgcn_s_memtime();
#endif
        const unsigned long long guard_cap = (unsigned long long)(nb + 2u) * (((unsigned long long)(kBezMaxDepth + 3) << (kBezMaxDepth + 2)) + 2ull);
        for (unsigned long long g = 0;; ++g) {                    // wave-uniform
            if (g > guard_cap) { raise_fault(RT_FAULT_CURVE); break; }
#ifdef RT_STATS
            ++n_it;
            n_busy += busy ? 1u : 0u;
            if (busy) {
                ++n_step;
                if (!wk.fresh) { ++n_red; n_rsplit += (uint32_t)wk.L; }
                if (bez_walk_at_leaf(wk)) ++n_leaf;     // lane-iterations at a leaf (tested or waiting)
            }
#endif
#ifdef RT_STATS
            const unsigned long long cr0 = __builtin_amdgcn_s_memtime();
#endif
            const unsigned long long idle = __ballot(!busy);
            if (cursor < nb && (__popcll(idle) >= kBezRefill || idle == act)) {
                if (!busy) {
                    const uint32_t i = cursor + lanes_below(idle);
                    if (i < nb) {
                        const uint32_t e = W.sv[i];
                        si = i;
                        W.sz[i] = INFINITY;
                        if constexpr (TRACK)
                            busy = bez_walk_begin_root(wk, ring[(rtail + i) & (uint32_t)(kBezRing - 1)], W.cl[e & 63u], W.lev[i]);
                        else
                            busy = bez_walk_begin(wk, sc.bez[e >> 6], W.ray[e & 63u], W.cl[e & 63u], W.lev[i]);
                    }
                }
                cursor += (uint32_t)__popcll(idle);
            } else if (RT_BEZ_DONATE > 0 && cursor >= nb && __popcll(idle) >= RT_BEZ_DONATE && idle != act) {
                // donation round: the candidate queue is empty during stage B, W.q carries the handover
                const uint32_t pend = busy ? bez_walk_pending(wk) : 0u;
                const unsigned long long dm = __ballot(pend != 0u);
                const uint32_t nd = min((uint32_t)__popcll(dm), (uint32_t)__popcll(idle));
                if (nd) {
                    const uint32_t dr = lanes_below(dm);
                    if (pend != 0u && dr < nd) {
                        uint32_t l, ridx;
                        bez_walk_donate(wk, pend, l, ridx);
                        W.q[2 * dr] = si; W.q[2 * dr + 1] = (l << 26) | ridx;     // l <= 25, ridx < 2^25
                    }
                    wave_sync();
                    const uint32_t ir = lanes_below(idle);
                    if (!busy && ir < nd) {
                        si = W.q[2 * ir];
                        const uint32_t e = W.sv[si], lr = W.q[2 * ir + 1];
                        if constexpr (TRACK)
                            bez_walk_take_root(wk, ring[(rtail + si) & (uint32_t)(kBezRing - 1)], W.cl[e & 63u], W.lev[si],
                                               lr >> 26, lr & ((1u << 26) - 1u));
                        else
                            bez_walk_take(wk, sc.bez[e >> 6], W.ray[e & 63u], W.cl[e & 63u], W.lev[si], lr >> 26,
                                          lr & ((1u << 26) - 1u));
                        busy = true;
                    }
                    wave_sync();
                }
            }
#ifdef RT_STATS
            n_clk_refill += __builtin_amdgcn_s_memtime() - cr0;
#endif
            const unsigned long long bm = __ballot(busy);
            if (bm == 0ull) {
                if (cursor >= nb) break;
                continue;
            }
            // lanes at a leaf segment wait until enough of them (or every busy lane) are there and
            // then test together; the others split this iteration either way
            const bool at_leaf = busy && bez_walk_at_leaf(wk);
            const unsigned long long lm = __ballot(at_leaf);
            bool over = false;
#ifdef RT_STATS
            const unsigned long long cl0 = __builtin_amdgcn_s_memtime();
#endif
            if (lm != 0ull && (__popcll(lm) >= RT_BEZ_LEAF_PHASE || lm == bm)) {
                if (at_leaf) over = bez_walk_leaf(wk);
            }
#ifdef RT_STATS
            const unsigned long long cl1 = __builtin_amdgcn_s_memtime();
            n_clk_leaf += cl1 - cl0;
#endif
            if constexpr (WV::SLOT) {
                if (busy && !at_leaf) over = bez_walk_node<true>(wk, &W.pend[threadIdx.x & 63u]);
            } else {
                if (busy && !at_leaf) over = bez_walk_node(wk);
            }
#ifdef RT_STATS
            n_clk_node += __builtin_amdgcn_s_memtime() - cl1;
#endif
            if (over) {
                if (wk.found)
                    atomicMin((unsigned long long*)&W.sz[si], (unsigned long long)__double_as_longlong(wk.best));
                busy = false;
            }
        }
#ifdef RT_STATS
        {   // per-lane counts summed in LDS first: 64 global atomics per counter and pass would load stage B itself
            __shared__ unsigned int s_st[4][5];
            unsigned int* ws = s_st[(threadIdx.x >> 6) & 3u];
            for (uint32_t j = rank; j < 5u; j += nact) ws[j] = 0u;
            wave_sync();
            atomicAdd(&ws[0], n_busy); atomicAdd(&ws[1], n_step); atomicAdd(&ws[2], n_red);
            atomicAdd(&ws[3], n_rsplit); atomicAdd(&ws[4], n_leaf);
            wave_sync();
            if (rank == 0) {
                RT_STAT(33, ws[0]); RT_STAT(34, ws[1]); RT_STAT(35, ws[2]); RT_STAT(36, ws[3]); RT_STAT(37, ws[4]);
            }
            wave_sync();
        }
        if (rank == 0) {
            RT_STAT(31, 1); RT_STAT(32, n_it); RT_STAT(38, nb);
            RT_STAT(39, __builtin_amdgcn_s_memtime() - clk0); RT_STAT(45, n_clk_refill);
            RT_STAT(46, n_clk_leaf); RT_STAT(47, n_clk_node);
        }
#endif
    }
    wave_sync();
    for (uint32_t base = 0; base < nb; base += nact) {
        const uint32_t i = base + rank;
        if (i < nb && !(kTmin < W.sz[i])) W.sz[i] = INFINITY;                // :201
        if (i < nb && W.sz[i] != INFINITY)
            atomicMin((unsigned long long*)&W.hz[W.sv[i] & 63u], (unsigned long long)__double_as_longlong(W.sz[i]));
    }
    wave_sync();
    for (uint32_t base = 0; base < nb; base += nact) {
        const uint32_t i = base + rank;
        if (i < nb && W.sz[i] != INFINITY) {
            const uint32_t e = W.sv[i], o = e & 63u;
            if (W.sz[i] == W.hz[o])
                atomicMax(&W.hkey[o], ((unsigned long long)sc.bez[e >> 6].order << 32) | (e >> 6));
        }
        if (TRACK && i < nb) atomicAdd(&W.done[W.sv[i] & 63u], 1u);
    }
    wave_sync();
    const uint32_t rest = svn - nb;             // < nact <= 64, disjoint from [0, rest) only if nb >= rest
    uint32_t e = 0;
    uint8_t lv = 0;
    if (rank < rest) { e = W.sv[nb + rank]; lv = W.lev[nb + rank]; }
    wave_sync();
    if (rank < rest) { W.sv[rank] = e; W.lev[rank] = lv; }
    wave_sync();
}

// The owner's result of a batch (hz, hid) against its closest hit so far: a
// curve reports z <= the t-max it was tested with (bezier.scm:164), so it
// takes the hit on a tie with a sphere or rect; between two curves at the
// same z the later one of the list (BezierRec::order) is the one the scan
// keeps, whichever batch tested it first.
template <class WV>
__device__ __forceinline__ void bez_take_batch(const DevScene& sc, const WV& W, const uint32_t lane,
                                               const int32_t bz, double& closest, int32_t& best) {
    const double z = W.hz[lane];
    if (z == INFINITY || z > closest) return;
    const uint32_t id = (uint32_t)W.hkey[lane];
    if (z == closest && best >= bz && best < bz + sc.n_bez && sc.bez[best - bz].order > (uint32_t)(W.hkey[lane] >> 32))
        return;
    closest = z;
    best = bz + (int32_t)id;
}

// Per-lane BVH traversal: every lane walks its own path through the BVH2
// (child boxes tested at the parent, nearer child first, LDS stack with a
// block-size stride so a wave's pushes hit 64 consecutive banks).
// f32 slab test on t = fma(box, 1/d, -o/d).  Each computed slab end is
// within 4 ulps * (|box| + |o|) * |1/d| of the exact one; the boxes carry an
// absolute margin above that bound for any origin inside the scene radius
// (commit_scene), so the test only culls boxes the ray misses.
struct BoxRay { float ix, iy, iz, px, py, pz; };     // 1/d and o/d
__device__ __forceinline__ float f32_up(const double x) {       // x >= 0 (a ray's t range)
    float f = (float)x;
    if ((double)f < x) f = __int_as_float(__float_as_int(f) + 1);
    return f;
}
__device__ __forceinline__ BoxRay box_ray(const v3 o, const v3 d) {
    const double lim = 1e30;
    const double ix = fmax(fmin(1.0 / d.x, lim), -lim);
    const double iy = fmax(fmin(1.0 / d.y, lim), -lim);
    const double iz = fmax(fmin(1.0 / d.z, lim), -lim);
    BoxRay b;
    b.ix = (float)ix; b.iy = (float)iy; b.iz = (float)iz;
    b.px = (float)(o.x * ix); b.py = (float)(o.y * iy); b.pz = (float)(o.z * iz);
    return b;
}
// Rays from anywhere (scenes with curves).  The box margin covers the slab ends' rounding only for an
// origin inside the scene radius, but a curve reports its hit at the distance along unit(dir) on the raw
// ray (Q10, bezier.scm:204-206), so a ray with |dir| != 1 (a reflection off a metal curve: |dir| grows
// ~quadratically per bounce) starts its next segment far outside the scene: at 1e9 from it, a C5-style
// scene's f32 slab ends err by more than the margin, and the walk culled a curve the ray hits
// (test_few_curves_among_spheres_large_launch, pixel 247288 sample 5, segment 70).  The rounding that
// depends on the origin is below 4 ulps of |o / d| per axis, so this box ray subtracts o/d - e from
// the near plane of each axis and o/d + e from the far one, e = 2^-20 |o / d| (about 8x that bound):
// each slab is widened by its own error, at no extra instruction in the node test (the lo and hi
// planes take different registers instead of one).
struct BoxRayW { float ix, iy, iz, lx, ly, lz, hx, hy, hz; };   // 1/d; o/d adjusted for the lo / hi planes
__device__ __forceinline__ BoxRayW box_ray_w(const v3 o, const v3 d) {
    const double lim = 1e30;
    const double i[3] = {fmax(fmin(1.0 / d.x, lim), -lim), fmax(fmin(1.0 / d.y, lim), -lim),
                         fmax(fmin(1.0 / d.z, lim), -lim)};
    const double oo[3] = {o.x, o.y, o.z};
    float lo[3], hi[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double p = oo[a] * i[a], e = 0x1p-20 * fabs(p);
        // ix >= 0: the lo plane gives the near end (subtract more), the hi plane the far one; else swapped
        lo[a] = (float)(i[a] >= 0.0 ? p + e : p - e);
        hi[a] = (float)(i[a] >= 0.0 ? p - e : p + e);
    }
    return BoxRayW{(float)i[0], (float)i[1], (float)i[2], lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]};
}
// Both child boxes of N (interleaved planes, BvhNode2): slab ends t = fma(box,
// 1/d, -o/d), near / far per child; hit iff near <= far.  (Packed v_pk_fma_f32
// pairs were measured slower here: the pairs raise register pressure.)
__device__ __forceinline__ void node_hit(const BvhNode2& N, const BoxRay& r, const float tcap, bool& hl, bool& hr,
                                         float& tl, float& tr) {
    auto one = [&](const int c, float& tn) {
        const float tx0 = fmaf(N.b[0 + c], r.ix, -r.px), tx1 = fmaf(N.b[6 + c], r.ix, -r.px);
        const float ty0 = fmaf(N.b[2 + c], r.iy, -r.py), ty1 = fmaf(N.b[8 + c], r.iy, -r.py);
        const float tz0 = fmaf(N.b[4 + c], r.iz, -r.pz), tz1 = fmaf(N.b[10 + c], r.iz, -r.pz);
        tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
        const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tcap));
        return tn <= tf;
    };
    hl = one(0, tl);
    hr = one(1, tr);
}
// the same with the widened slabs of a box ray from anywhere (BoxRayW)
__device__ __forceinline__ void node_hit(const BvhNode2& N, const BoxRayW& r, const float tcap, bool& hl, bool& hr,
                                         float& tl, float& tr) {
    auto one = [&](const int c, float& tn) {
        const float tx0 = fmaf(N.b[0 + c], r.ix, -r.lx), tx1 = fmaf(N.b[6 + c], r.ix, -r.hx);
        const float ty0 = fmaf(N.b[2 + c], r.iy, -r.ly), ty1 = fmaf(N.b[8 + c], r.iy, -r.hy);
        const float tz0 = fmaf(N.b[4 + c], r.iz, -r.lz), tz1 = fmaf(N.b[10 + c], r.iz, -r.hz);
        tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
        const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tcap));
        return tn <= tf;
    };
    hl = one(0, tl);
    hr = one(1, tr);
}

// Sign-selected slab planes (RT_SIGNED_SLAB, the LDS-tree walks): with the
// sign of 1/d known per lane, an axis's near plane is its lo plane for a
// positive component and its hi plane otherwise (fma(b, 1/d, -o/d) rounds
// monotonically in b), so the per-axis min / max pairs of node_hit go away
// and the results are node_hit's bit for bit.  SlabOff: byte offsets of the
// near / far plane pairs (left, right) in a BvhNode2.
#ifndef RT_SIGNED_SLAB
#define RT_SIGNED_SLAB 1
#endif
struct SlabOff { uint32_t nx, ny, nz, fx, fy, fz; };
__device__ __forceinline__ SlabOff slab_off(const BoxRay& r) {
    SlabOff o;                                              // far = near ^ (lo ^ hi offset)
    o.nx = r.ix < 0.0f ? 24u : 0u;  o.fx = o.nx ^ 24u;     // b[0..1] lo x, b[6..7] hi x
    o.ny = r.iy < 0.0f ? 32u : 8u;  o.fy = o.ny ^ 40u;     // b[2..3], b[8..9]
    o.nz = r.iz < 0.0f ? 40u : 16u; o.fz = o.nz ^ 56u;     // b[4..5], b[10..11]
    return o;
}
// The six plane-pair pointers of node 0 (nodes + the SlabOff offsets) are
// per-lane constants; node k's pair is at pointer + k * 64 (one shift-add per
// address).
struct SlabPtr { const char *nx, *ny, *nz, *fx, *fy, *fz; };
__device__ __forceinline__ SlabPtr slab_ptr(const BvhNode2* nodes, const SlabOff& so) {
    const char* B = reinterpret_cast<const char*>(nodes);
    return SlabPtr{B + so.nx, B + so.ny, B + so.nz, B + so.fx, B + so.fy, B + so.fz};
}
__device__ __forceinline__ void node_hit_signed(const SlabPtr& sp, const uint32_t k, const BoxRay& r,
                                                const float tcap, bool& hl, bool& hr, float& tl, float& tr) {
    static_assert(sizeof(BvhNode2) == 64, "node_hit_signed addresses 64-B nodes");
    auto pair = [&](const char* p) { return *reinterpret_cast<const float2*>(p + (k << 6)); };
    const float2 nx = pair(sp.nx), fx = pair(sp.fx), ny = pair(sp.ny), fy = pair(sp.fy);
    const float2 nz = pair(sp.nz), fz = pair(sp.fz);
    tl = fmaxf(fmaxf(fmaf(nx.x, r.ix, -r.px), fmaf(ny.x, r.iy, -r.py)), fmaxf(fmaf(nz.x, r.iz, -r.pz), 0.0f));
    tr = fmaxf(fmaxf(fmaf(nx.y, r.ix, -r.px), fmaf(ny.y, r.iy, -r.py)), fmaxf(fmaf(nz.y, r.iz, -r.pz), 0.0f));
    const float fl = fminf(fminf(fmaf(fx.x, r.ix, -r.px), fmaf(fy.x, r.iy, -r.py)), fminf(fmaf(fz.x, r.iz, -r.pz), tcap));
    const float fr = fminf(fminf(fmaf(fx.y, r.ix, -r.px), fmaf(fy.y, r.iy, -r.py)), fminf(fmaf(fz.y, r.iz, -r.pz), tcap));
    hl = tl <= fl;
    hr = tr <= fr;
}

// FROZEN: the time-0 tree (DevScene::fbvh2), whose leaves hold plain sphere
// records (moving spheres at center(0)); otherwise the all-times tree.
// nodes / leaves / fsph may point into LDS (k_extend_lds) or HBM.
__device__ __forceinline__ int32_t stack_ref(const uint32_t e) { return (int32_t)e; }
__device__ __forceinline__ int32_t stack_ref(const uint16_t e) { return (int32_t)(int16_t)e; }   // sign: leaf refs < 0
// SE: stack entry type — uint32_t, or uint16_t (k_extend_lds / k_camera, trees
// under 32768 nodes and leaves: child refs fit int16, halving the LDS stack).
// DIRECT (FROZEN only, DevScene::bvh_solo): every time-0 leaf holds one
// sphere and fsph is in leaf order, so leaf ref ~k tests fsph[k] directly
// (no leaf record to fetch or keep in LDS).
// WIDE: the box ray from anywhere (BoxRayW; scenes with curves, whose rays may start far outside)
template <bool FROZEN, class SE = uint32_t, bool DIRECT = false, bool WIDE = false>
__device__ __forceinline__ void bvh_closest_lane(const DevScene& sc, const v3 o, const v3 d, const double time,
                                                 double& closest, int32_t& best, SE* lstk, const int lmax,
                                                 const BvhNode2* __restrict__ nodes,
                                                 const BvhLeaf* __restrict__ leaves,
                                                 const SphereRec* __restrict__ fsph,
                                                 const SphereRec* __restrict__ sph = nullptr,
                                                 const MSphereRec* __restrict__ msph = nullptr,
                                                 const int32_t* __restrict__ fid = nullptr) {
    constexpr int32_t kDone = INT32_MIN;
    const double a = dot(d, d), ia = 1.0 / a;
    // 16-bit stacks: the LDS-tree walks; RT_SIGNED_SLAB 1 = the time-0 tree only, 2 = also the all-times tree
    constexpr bool SIGNED = sizeof(SE) == 2 && (RT_SIGNED_SLAB == 2 || (RT_SIGNED_SLAB == 1 && FROZEN));
    static_assert(!(WIDE && SIGNED), "the sign-selected LDS walks serve scenes without curves only");
    using BR = typename std::conditional<WIDE, BoxRayW, BoxRay>::type;
    BR br;
    if constexpr (WIDE) br = box_ray_w(o, d);
    else br = box_ray(o, d);
    SlabPtr slp{};
    if constexpr (SIGNED) slp = slab_ptr(nodes, slab_off(br));
    const int32_t bs = sc.leaf_base[LEAF_SPHERE], bm = sc.leaf_base[LEAF_MSPHERE];
    const uint32_t stride = blockDim.x;
    int32_t fbest = -1;                                       // FROZEN: fsph index of the best hit
    // moving spheres sharing one shutter: center(time)'s (time - t0) / den is
    // the same quotient for all of them, computed once (geometry.scm:181-184)
    const double frac_shared = (!FROZEN && sc.msph_shared) ? (time - sc.msph_t0) / sc.msph_den : 0.0;
    // stack pointer as an element offset (entries sit stride apart): push / pop
    // add or subtract stride instead of multiplying the depth by it
    uint32_t sp = 0;
    const uint32_t slim = (uint32_t)lmax * stride;
    int32_t node = FROZEN ? sc.fbvh2_root : sc.bvh2_root, pend = kDone;
    float tcap = f32_up(closest);                              // box t range, updated after each leaf
#ifdef RT_STATS
    uint32_t n_node = 0, n_leaf = 0, n_sph = 0, n_msph = 0, n_inner = 0, n_outer = 0;
#endif
    while (node != kDone || pend != kDone) {
#ifdef RT_STATS
        ++n_outer;
#endif
        while (node != kDone) {
#ifdef RT_STATS
            ++n_inner;
#endif
            if (node < 0) {                                   // a leaf
                if (pend != kDone) break;                     // one is already parked
                pend = node;
                node = sp ? stack_ref(lstk[sp -= stride]) : kDone;
            } else {
#ifdef RT_STATS
                ++n_node;
#endif
                float tl, tr;
                bool hl, hr;
                int2 N;                                       // child refs (l, r)
                if constexpr (SIGNED) {
                    node_hit_signed(slp, (uint32_t)node, br, tcap, hl, hr, tl, tr);
                    N = *reinterpret_cast<const int2*>(&nodes[node].l);
                } else {
                    const BvhNode2 M = nodes[node];
                    node_hit(M, br, tcap, hl, hr, tl, tr);
                    N = make_int2(M.l, M.r);
                }
                if (hl && hr) {
                    const bool lfirst = tl <= tr;
                    if (sp < slim) { lstk[sp] = (SE)(lfirst ? N.y : N.x); sp += stride; }
                    node = lfirst ? N.x : N.y;
                } else if (hl) {
                    node = N.x;
                } else if (hr) {
                    node = N.y;
                } else {
                    node = sp ? stack_ref(lstk[sp -= stride]) : kDone;
                }
            }
            // every active lane has a leaf parked
            if (__ballot(pend == kDone) == 0ull) break;
        }
        if (pend != kDone) {
            if constexpr (DIRECT) {
#ifdef RT_STATS
                ++n_leaf; ++n_sph;
#endif
                const SphereRec S = fsph[~pend];
                sphere_test(o, d, a, ia, mk(S.cx, S.cy, S.cz), S.rr, ~pend, closest, fbest);
            } else {
                const BvhLeaf L = leaves[~pend];
#ifdef RT_STATS
                ++n_leaf;
#endif
                if (FROZEN) {
                    for (int s = L.sb; s < L.sb + L.sn; ++s) {
#ifdef RT_STATS
                        ++n_sph;
#endif
                        const SphereRec S = fsph[s];
                        sphere_test(o, d, a, ia, mk(S.cx, S.cy, S.cz), S.rr, s, closest, fbest);
                    }
                } else {
                    for (int s = L.sb; s < L.sb + L.sn; ++s) {
#ifdef RT_STATS
                        ++n_sph;
#endif
                        const SphereRec S = sph[s];
                        sphere_test(o, d, a, ia, mk(S.cx, S.cy, S.cz), S.rr, bs + s, closest, best);
                    }
                    for (int s = L.mb; s < L.mb + L.mn; ++s) {
#ifdef RT_STATS
                        ++n_msph;
#endif
                        const MSphereRec S = msph[s];
                        const double frac = sc.msph_shared ? frac_shared : (time - S.t0) / S.den;
                        const v3 cen = mk(S.c0x, S.c0y, S.c0z) + mk(S.dcx, S.dcy, S.dcz) * frac;
                        sphere_test(o, d, a, ia, cen, S.rr, bm + s, closest, best);
                    }
                }
            }
            pend = kDone;
            tcap = f32_up(closest);
        }
    }
    if (FROZEN && fbest >= 0) best = fid[fbest];
#ifdef RT_STATS
    constexpr int so = FROZEN ? 16 : 0;
    RT_STAT(so + 0, 1); RT_STAT(so + 1, n_node); RT_STAT(so + 2, n_leaf); RT_STAT(so + 3, n_sph);
    RT_STAT(so + 4, n_msph); RT_STAT(so + 5, n_inner); RT_STAT(so + 6, n_outer);
    {   // wave-level iterations: the wave runs until its slowest lane is done
        const unsigned long long act = __ballot(1);
        uint32_t mi = 0, mo = 0;
        for (int l = 0; l < 64; ++l) {
            if (!((act >> l) & 1ull)) continue;
            mi = max(mi, (uint32_t)__builtin_amdgcn_readlane((int)n_inner, l));
            mo = max(mo, (uint32_t)__builtin_amdgcn_readlane((int)n_outer, l));
        }
        if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)act) - 1)) {
            RT_STAT(so + 7, 1); RT_STAT(so + 8, mi); RT_STAT(so + 9, mo); RT_STAT(so + 10, __popcll(act));
        }
    }
#endif
}

// Per-lane traversal of a BVH that holds curves: spheres are tested on the
// spot, curves are queued and tested wave-wide (BezWave).  One BVH step per
// loop iteration, so the wave checks the queue between steps.  A curve
// reports t as a distance along unit(d) (Q10), i.e. raw ray parameter
// t/|d|: for |d| < 1 the box range must reach closest/|d|.
__device__ __forceinline__ void bvh_closest_curves(const DevScene& sc, const v3 o, const v3 d, const double time,
                                                double& closest, int32_t& best, uint32_t* lstk, const int lmax,
                                                BezWave& W) {
    const double a = dot(d, d), ia = 1.0 / a;
    const BoxRayW br = box_ray_w(o, d);              // rays from anywhere (BoxRayW)
    const int32_t bs = sc.leaf_base[LEAF_SPHERE], bm = sc.leaf_base[LEAF_MSPHERE], bz = sc.leaf_base[LEAF_BEZIER];
    const double tscale = fmax(1.0, 1.0 / sqrt(a));
    const uint32_t lane = threadIdx.x & 63u;
    bez_ray(o, d, W.ray[lane]);
    const uint32_t stride = blockDim.x;
    int sp = 0;
    int32_t node = sc.bvh2_root;
    bool trav = true;
    int pb = 0, pe = 0;                         // this lane's curves still to queue
    uint32_t qn = 0, svn = 0;                   // queued candidates, survivors awaiting subdivision
#ifdef RT_STATS
    uint32_t n_node = 0, n_leaf = 0, n_cand = 0, n_flush = 0, n_iter = 0;
#endif
    // a lane visits each node and leaf at most once and queues each curve at most once, two per step
    const uint32_t cap = 2u * (uint32_t)(sc.n_bvh2 + sc.n_bleaf) + (uint32_t)sc.n_bez + 1024u;
    for (uint32_t it = 0;; ++it) {          // wave-uniform
        if (it > cap) { raise_fault(RT_FAULT_CURVE); break; }
#ifdef RT_STATS
        ++n_iter;
#endif
        if (pb >= pe && trav) {                 // lanes with curves pending only queue them below
            if (node >= 0) {
#ifdef RT_STATS
                ++n_node;
#endif
                const BvhNode2 N = sc.bvh2[node];
                const float tcap = f32_up(closest * tscale);
                float tl, tr;
                bool hl, hr;
                node_hit(N, br, tcap, hl, hr, tl, tr);
                if (hl && hr) {
                    const bool lfirst = tl <= tr;
                    if (sp < lmax) { lstk[sp * stride] = (uint32_t)(lfirst ? N.r : N.l); ++sp; }
                    node = lfirst ? N.l : N.r;
                } else if (hl) {
                    node = N.l;
                } else if (hr) {
                    node = N.r;
                } else if (sp == 0) {
                    trav = false;
                } else {
                    --sp;
                    node = (int32_t)lstk[sp * stride];
                }
            } else if (~node >= kDirectCurve) {               // a leaf holding one curve
                pb = ~node - kDirectCurve; pe = pb + 1;
#ifdef RT_STATS
                ++n_leaf; ++n_cand;
#endif
                if (sp == 0) {
                    trav = false;
                } else {
                    --sp;
                    node = (int32_t)lstk[sp * stride];
                }
            } else {
                const BvhLeaf L = sc.bleaf[~node];
                for (int s = L.sb; s < L.sb + L.sn; ++s) {
                    const SphereRec S = sc.sph[s];
                    sphere_test(o, d, a, ia, mk(S.cx, S.cy, S.cz), S.rr, bs + s, closest, best);
                }
                for (int s = L.mb; s < L.mb + L.mn; ++s) {
                    const MSphereRec S = sc.msph[s];
                    const double frac = (time - S.t0) / S.den;
                    const v3 cen = mk(S.c0x, S.c0y, S.c0z) + mk(S.dcx, S.dcy, S.dcz) * frac;
                    sphere_test(o, d, a, ia, cen, S.rr, bm + s, closest, best);
                }
                pb = L.bb; pe = L.bb + L.bn;
#ifdef RT_STATS
                ++n_leaf; n_cand += (uint32_t)L.bn;
#endif
                if (sp == 0) {
                    trav = false;
                } else {
                    --sp;
                    node = (int32_t)lstk[sp * stride];
                }
            }
        }
        // append one of this lane's curve candidates (kBezQ: at most one per lane per step)
        {
            const bool has = pb < pe;
            const unsigned long long m = __ballot(has);
            if (has) { W.q[qn + lanes_below(m)] = ((uint32_t)pb << 6) | lane; ++pb; }
            qn += (uint32_t)__popcll(m);
        }
        const bool more = __ballot(trav || pb < pe) != 0ull;
        if (qn >= 64u || (!more && (qn > 0u || svn > 0u))) {
#ifdef RT_STATS
            ++n_flush;
#endif
            W.cl[lane] = closest;
            wave_sync();
            svn = bez_stage_a(sc, W, qn, svn);
            qn = 0;
            const uint32_t nact = (uint32_t)__popcll(__ballot(1));
            const uint32_t nb = more ? svn - svn % nact : svn;
            if (nb > 0u) {
                W.hz[lane] = INFINITY;
                W.hkey[lane] = 0ull;
                wave_sync();
                bez_stage_b(sc, W, nb, svn);
                svn -= nb;
                bez_take_batch(sc, W, lane, bz, closest, best);
                wave_sync();
            }
        }
        if (!more) break;
    }
#ifdef RT_STATS
    RT_STAT(11, 1); RT_STAT(12, n_node); RT_STAT(13, n_leaf); RT_STAT(14, n_cand);
    if (lane == (uint32_t)__ffsll((long long)__ballot(1)) - 1u) {
        RT_STAT(27, n_flush); RT_STAT(28, n_iter); RT_STAT(29, 1); RT_STAT(30, __popcll(__ballot(1)));
    }
#endif
}

// ---------------------------------------------------------- closest hit
// hit-obj-list semantics (geometry.scm:33-50): shrinking t-max, strict
// (tmin, closest) for spheres, non-strict for rects.  Every lane of a wave
// walks the same group / primitive sequence, so the primitive records are
// fetched once per wave through the scalar unit.
// --------------------------------------------- Kleinian limit set (f4)
// geometry.scm:596-673: six inversion spheres, at most 10 inversions per
// distance estimate, sphere tracing (at most 100 steps) along the raw ray.
__device__ __forceinline__ v3 klein_sphere(const int i) {
    return (i == 0) ? mk(300.0, 300.0, 0.0) : (i == 1) ? mk(300.0, -300.0, 0.0)
         : (i == 2) ? mk(-300.0, 300.0, 0.0) : (i == 3) ? mk(-300.0, -300.0, 0.0)
         : (i == 4) ? mk(0.0, 0.0, 424.26) : mk(0.0, 0.0, -424.26);
}
__device__ __forceinline__ double klein_dist(const v3 center, const v3 p) {         // dist-func :609-635
    v3 pos = p - center;
    double dr = 1.0;
    for (int iter = 0; iter < 10; ++iter) {
        int idx = 0;
        v3 sp = klein_sphere(0);
        for (; idx < 6; ++idx) {
            sp = klein_sphere(idx);
            if (length(pos - sp) < 300.0) break;
        }
        if (idx == 6) break;
        const v3 diff = pos - sp;
        dr = dr * (90000.0 / dot(diff, diff));
        const double l = length(diff);
        pos = (diff * 90000.0) * (1.0 / (l * l)) + sp;
    }
    return 0.7 * ((length(pos) - 125.0) / fabs(dr));
}
__device__ __noinline__ v3 klein_normal(const v3 center, const v3 p) {               // get-normal :637-643
    return unit(mk(klein_dist(center, p + mk(0.01, 0.0, 0.0)) - klein_dist(center, p - mk(0.01, 0.0, 0.0)),
                   klein_dist(center, p + mk(0.0, 0.01, 0.0)) - klein_dist(center, p - mk(0.0, 0.01, 0.0)),
                   klein_dist(center, p + mk(0.0, 0.0, 0.01)) - klein_dist(center, p - mk(0.0, 0.0, 0.01))));
}
__device__ __forceinline__ bool klein_test(const KleinRec& K, const v3 o, const v3 d, const double tmax,
                                           double& tout) {                             // make-klein :655-670
    const v3 c = mk(K.cx, K.cy, K.cz);
    double len = 0.0;
    v3 pos = o;
    for (int iter = 0; iter < 100; ++iter) {
        const double dist = klein_dist(c, pos);
        len = len + dist;
        pos = o + d * len;
        if (dist < 0.001 && kTmin < len && len < tmax) { tout = len; return true; }
    }
    return false;
}

// ------------------------------------------------------- constant medium
// Closest boundary hit in (tmin, tmax) over a medium's boundary groups, with
// the reference's hit semantics (spheres strict, rects non-strict).
__device__ __forceinline__ bool boundary_hit(const DevScene& sc, const MediumRec& M, const v3 o0, const v3 d0,
                                             const double time, const double tmin, const double tmax,
                                             double& tout) {
    double closest = tmax;
    bool hit = false;
    for (int g = M.bg_begin; g < M.bg_end; ++g) {
        const Group G = sc.bgroups[g];
        v3 o = o0, d = d0;
        if (G.chain >= 0) chain_ray(sc.chains[G.chain], o, d);
        if (G.type == LEAF_SPHERE || G.type == LEAF_MSPHERE) {
            const double a = dot(d, d);
            for (int s = G.begin; s < G.end; ++s) {
                v3 c;
                double rr;
                if (G.type == LEAF_SPHERE) {
                    const SphereRec S = sc.sph[s];
                    c = mk(S.cx, S.cy, S.cz); rr = S.rr;
                } else {
                    const MSphereRec S = sc.msph[s];
                    c = mk(S.c0x, S.c0y, S.c0z) + mk(S.dcx, S.dcy, S.dcz) * ((time - S.t0) / S.den);
                    rr = S.rr;
                }
                const v3 oc = o - c;
                const double b = dot(oc, d);
                const double cc = dot(oc, oc) - rr;
                const double disc = b * b - a * cc;
                if (disc > 0.0) {
                    const double sq = sqrt(disc);
                    double t = (-b - sq) / a;
                    if (!(tmin < t && t < closest)) t = (-b + sq) / a;
                    if (tmin < t && t < closest) { closest = t; hit = true; }
                }
            }
        } else {
            double ok, dk, oa, da, ob, db;
            if (G.type == LEAF_RECT_XY) { ok = o.z; dk = d.z; oa = o.x; da = d.x; ob = o.y; db = d.y; }
            else if (G.type == LEAF_RECT_XZ) { ok = o.y; dk = d.y; oa = o.x; da = d.x; ob = o.z; db = d.z; }
            else { ok = o.x; dk = d.x; oa = o.y; da = d.y; ob = o.z; db = d.z; }
            for (int s = G.begin; s < G.end; ++s) {
                const RectRec R = sc.rect[s];
                const double t = (R.k - ok) / dk;
                if (t < tmin || t > closest) continue;
                const double A = oa + t * da, Bv = ob + t * db;
                if (A < R.a0 || A > R.a1 || Bv < R.b0 || Bv > R.b1) continue;
                closest = t; hit = true;
            }
        }
    }
    tout = closest;
    return hit;
}
// make-constant-medium's hit (geometry.scm:547-575).  o0, d0 are the world
// ray (boundary groups carry their full instance chain); d is the ray in the
// medium's own space.  Draws one random number when the ray's span inside
// the boundary overlaps (tmin, tmax), like the reference.
__device__ __forceinline__ bool medium_test(const DevScene& sc, const MediumRec& M, const v3 o0, const v3 d0,
                                            const v3 d, const double time, const double tmax, Rng& g,
                                            double& tout) {
    double t1r, t2r;
    if (!boundary_hit(sc, M, o0, d0, time, -kTmax, kTmax, t1r)) return false;
    if (!boundary_hit(sc, M, o0, d0, time, t1r + 0.0001, kTmax, t2r)) return false;
    double t1 = (t1r < kTmin) ? kTmin : t1r;
    const double t2 = (t2r > tmax) ? tmax : t2r;
    if (t1 >= t2) return false;
    if (t1 < 0.0) t1 = 0.0;
    const double len = length(d);
    const double inside = (t2 - t1) * len;
    const double hd = M.neg_inv_density * log(g.next());
    if (!(hd < inside)) return false;
    tout = t1 + hd / len;
    return true;
}

// The time-0 tree a kernel traverses (k_extend_lds stages it in LDS).
struct Tree0 { const BvhNode2* nodes; const BvhLeaf* leaves; const SphereRec* sph; const int32_t* fid; };
__device__ __forceinline__ Tree0 tree0_hbm(const DevScene& sc) { return Tree0{sc.fbvh2, sc.fbleaf, sc.fsph, sc.fid}; }
// The all-times tree (k_camera stages it in LDS when the scene has moving spheres).
struct TreeA { const BvhNode2* nodes; const BvhLeaf* leaves; const SphereRec* sph; const MSphereRec* msph; };
__device__ __forceinline__ TreeA treeA_hbm(const DevScene& sc) { return TreeA{sc.bvh2, sc.bleaf, sc.sph, sc.msph}; }

// One non-BVH group of hit-obj-list (geometry.scm:33-50): its primitives in
// list order against the shrinking closest.
template <int F>
__device__ __forceinline__ void group_closest(const DevScene& sc, const Group& G, const v3 o0, const v3 d0,
                                              const double time, double& closest, int32_t& best, Rng* rng) {
    constexpr bool BEZ = (F & kFeatCurves) != 0;
    constexpr bool MED = (F & kFeatExtra) != 0;
    v3 o = o0, d = d0;
    if (G.chain >= 0) chain_ray(sc.chains[G.chain], o, d);
    const int32_t base = sc.leaf_base[G.type];
    if (G.type == LEAF_SPHERE) {                       // geometry.scm:146-171
        const double a = dot(d, d), ia = 1.0 / a;
        for (int s = G.begin; s < G.end; ++s) {
            const SphereRec S = sc.sph[s];
            sphere_test(o, d, a, ia, mk(S.cx, S.cy, S.cz), S.rr, base + s, closest, best);
        }
    } else if (G.type == LEAF_MSPHERE) {               // geometry.scm:177-208
        const double a = dot(d, d), ia = 1.0 / a;
        double last_t0 = 0.0, last_den = 0.0, frac = 0.0;
        bool have = false;
        for (int s = G.begin; s < G.end; ++s) {
            const MSphereRec S = sc.msph[s];
            if (!have || S.t0 != last_t0 || S.den != last_den) {   // uniform branch
                frac = (time - S.t0) / S.den;
                last_t0 = S.t0; last_den = S.den; have = true;
            }
            const v3 cen = mk(S.c0x, S.c0y, S.c0z) + mk(S.dcx, S.dcy, S.dcz) * frac;
            sphere_test(o, d, a, ia, cen, S.rr, base + s, closest, best);
        }
    } else if (G.type == LEAF_KLEIN) {                 // geometry.scm:645-673
        if (MED) {
            for (int s = G.begin; s < G.end; ++s) {
                double t;
                if (klein_test(sc.klein[s], o, d, closest, t)) { closest = t; best = base + s; }
            }
        }
    } else if (G.type == LEAF_MEDIUM) {                // geometry.scm:545-578
        if (MED) {
            for (int s = G.begin; s < G.end; ++s) {
                double t;
                if (medium_test(sc, sc.med[s], o0, d0, d, time, closest, *rng, t)) { closest = t; best = base + s; }
            }
        }
    } else if (G.type == LEAF_BEZIER) {                // bezier.scm:176-214
        if (BEZ) {
            BezRay R;
            bez_ray(o, d, R);
            for (int s = G.begin; s < G.end; ++s) {
                double t;
                if (bezier_test(sc.bez[s], R, closest, t)) { closest = t; best = base + s; }
            }
        }
    } else {                                            // geometry.scm:376-431
        // XY: k on z, (a,b) = (x,y); XZ: k on y, (x,z); YZ: k on x, (y,z)
        double ok, dk, oa, da, ob, db;
        if (G.type == LEAF_RECT_XY) { ok = o.z; dk = d.z; oa = o.x; da = d.x; ob = o.y; db = d.y; }
        else if (G.type == LEAF_RECT_XZ) { ok = o.y; dk = d.y; oa = o.x; da = d.x; ob = o.z; db = d.z; }
        else { ok = o.x; dk = d.x; oa = o.y; da = d.y; ob = o.z; db = d.z; }
        for (int s = G.begin; s < G.end; ++s) {
            const RectRec R = sc.rect[s];
            const double t = (R.k - ok) / dk;
            if (t < kTmin || t > closest) continue;
            const double A = oa + t * da, Bv = ob + t * db;
            if (A < R.a0 || A > R.a1 || Bv < R.b0 || Bv > R.b1) continue;
            closest = t; best = base + s;
        }
    }
}

template <int F, class SE = uint32_t>
__device__ __forceinline__ int32_t closest_hit(const DevScene& sc, const v3 o0, const v3 d0,
                                               const double time, double& closest, SE* lstk,
                                               const int lmax, BezWave* bw, Rng* rng, const Tree0 t0,
                                               const TreeA ta) {
    constexpr bool BEZ = (F & kFeatCurves) != 0;
    int32_t best = -1;
    closest = kTmax;
    for (int g = 0; g < sc.n_groups; ++g) {
        const Group G = sc.groups[g];
        if (G.type == GROUP_BVH) {
            if (BEZ && sc.bvh_has_bez)
                bvh_closest_curves(sc, o0, d0, time, closest, best, reinterpret_cast<uint32_t*>(lstk), lmax, *bw);
            else if (sc.fbvh2 && (sc.tree0_any_time || __double_as_longlong(time) == 0ll))   // the time-0 tree
                bvh_closest_lane<true, SE, false, BEZ>(sc, o0, d0, time, closest, best, lstk, lmax, t0.nodes, t0.leaves,
                                                       t0.sph, nullptr, nullptr, t0.fid);
            else bvh_closest_lane<false, SE, false, BEZ>(sc, o0, d0, time, closest, best, lstk, lmax, ta.nodes, ta.leaves,
                                                     nullptr, ta.sph, ta.msph);
            continue;
        }
        group_closest<F>(sc, G, o0, d0, time, closest, best, rng);
    }
    return best;
}

// The LDS kernels' closest hit.  SOLO: the world is exactly one BVH group
// (the cover scene: every object is a world-level sphere), so the kernel holds
// only the tree walk — no code or registers for the other group types.
// ALL_ONLY (k_camera over the all-times tree): a camera ray whose time is
// +0.0 also walks the all-times tree, whose boxes bound every time and whose
// moving-sphere test at time 0 computes the frozen centre with the same
// operations — the same closest hit, so one walk is compiled instead of two.
template <bool SOLO, bool ALL_ONLY = false>
__device__ __forceinline__ int32_t closest_hit_lds(const DevScene& sc, const v3 o, const v3 d, const double time,
                                                   double& closest, uint16_t* lstk, const int lmax, const Tree0 t0,
                                                   const TreeA ta) {
    if (!SOLO) return closest_hit<0, uint16_t>(sc, o, d, time, closest, lstk, lmax, nullptr, nullptr, t0, ta);
    int32_t best = -1;
    closest = kTmax;
    if (!ALL_ONLY && (sc.tree0_any_time || __double_as_longlong(time) == 0ll))
        bvh_closest_lane<true, uint16_t, true>(sc, o, d, time, closest, best, lstk, lmax, t0.nodes, nullptr, t0.sph,
                                               nullptr, nullptr, t0.fid);
    else
        bvh_closest_lane<false, uint16_t>(sc, o, d, time, closest, best, lstk, lmax, ta.nodes, ta.leaves, nullptr,
                                          ta.sph, ta.msph);
    return best;
}

// ------------------------------------------------------------ path state
struct PathRegs {
    v3 o, d;
    double time;
    v3 T;
    uint32_t pix, smp, wid, rng, depth;
};
// pixel and absolute sample of work id wid (RNG keys, see PathState)
__device__ __forceinline__ void wid_key(const RenderParams& rp, const uint32_t wid, uint32_t& pix, uint32_t& smp) {
    const uint32_t s_rel = wid / rp.npix;
    pix = rp.pixlist[wid - s_rel * rp.npix];
    smp = rp.spp0 + s_rel;
}
// depth 0: slot i of the raygen output (wid = i, throughput 1); deeper: the
// path record (its depth is the iteration's, passed in)
__device__ __forceinline__ void load_path(const PathState& st, uint32_t i, PathRegs& p, const RenderParams& rp,
                                          const uint32_t depth) {
    const bool depth0 = depth == 0u;
    const RayRec R = st.ray[i];
    p.o = mk(R.ox, R.oy, R.oz);
    p.d = mk(R.dx, R.dy, R.dz);
    if (depth0) {
        p.time = st.tm[i];
        p.T = mk(1.0, 1.0, 1.0);
        p.wid = i; p.depth = 0u; p.rng = st.rng0[i];
    } else {
        const PathRec P = st.path[i];
        p.time = 0.0;                                    // every scattered ray (Q4)
        p.T = mk(P.tr, P.tg, P.tb);
        p.wid = P.wid; p.depth = depth; p.rng = P.rng;
    }
    wid_key(rp, p.wid, p.pix, p.smp);
}
// a scattered path (depth >= 1: no time)
__device__ __forceinline__ void store_path(const PathState& st, uint32_t k, const PathRegs& p) {
    st.ray[k] = ray_rec(p.o, p.d);
    st.path[k] = path_rec(p.T, p.wid, p.rng);
}
// a finished sample's colour: one 24-B record per work id (rgb together, so a
// scattered sample write touches one 32-B sector instead of three lines)
__device__ __forceinline__ void put_sample(const RenderParams& rp, const uint32_t w, const double r, const double g,
                                           const double b) {
    double* o = rp.sb + 3u * (size_t)w;
    o[0] = r; o[1] = g; o[2] = b;
}
// path done: sample colour = T (*) L into the chunk's sample buffer
__device__ __forceinline__ void write_sample(const RenderParams& rp, const PathRegs& p, const v3 L) {
    put_sample(rp, p.wid, p.T.x * L.x, p.T.y * L.y, p.T.z * L.z);
}
__device__ __forceinline__ v3 sky_radiance(const DevScene& sc, const v3 d) {
    if (sc.sky != 0) return mk(0.0, 0.0, 0.0);            // black main.scm:97-98
    const v3 ud = unit(d);                                 // sky-color main.scm:91-95
    const double s = 0.5 * (1.0 + ud.y);
    return mk(1.0, 1.0, 1.0) * (1.0 - s) + mk(0.5, 0.7, 1.0) * s;
}

// ------------------------------------------------------ stream compaction
// Virtual index -> physical slot of a sharded queue (QView).  The 8 shard
// counts are wave-uniform (scalar loads); the select chain avoids dynamic
// register indexing.
struct QMap { uint32_t off[kShards]; uint32_t cap; bool contiguous; };
__device__ __forceinline__ QMap qmap(const QView v) {
    QMap m;
    m.cap = v.cap;
    m.contiguous = v.counts == nullptr;
    uint32_t acc = 0;
#pragma unroll
    // a shard's counter can pass its capacity (the append then dropped the item and
    // raised RT_FAULT_SHARD): consumers index only what was written
    for (int x = 0; x < kShards; ++x) { m.off[x] = acc; if (!m.contiguous) acc += min(v.counts[x * kCntStride], v.cap); }
    return m;
}
__device__ __forceinline__ uint32_t qphys(const QMap& m, uint32_t k) {
    if (m.contiguous) return k;
    uint32_t base = 0, x = 0;
#pragma unroll
    for (int j = 1; j < kShards; ++j)
        if (k >= m.off[j]) { base = m.off[j]; x = (uint32_t)j; }
    return x * m.cap + (k - base);
}

// Block-aggregated, shard-spread stream compaction (all threads of the block
// must call it: it holds barriers).  cls in [0, NC) selects the queue, -1 =
// nothing to append.  Per class: wave64 ballot + mbcnt inside each wave, an
// exclusive scan of the wave counts in LDS, ONE atomicAdd per block on the
// counter of shard blockIdx % kShards.  Returns the item's physical slot
// (within its class queue).
template <int NC>
__device__ __forceinline__ uint32_t block_append(const int cls, uint32_t* __restrict__ counts,
                                                 const uint32_t shard_cap, uint32_t* s_cnt) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t shard = blockIdx.x & (kShards - 1);
    uint32_t below = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const unsigned long long mask = __ballot(cls == c);
        if (cls == c)
            below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        if (lane == 0) s_cnt[c * 16 + wave] = (uint32_t)__popcll(mask);
    }
    __syncthreads();
    if (threadIdx.x < (uint32_t)NC) {
        const int c = threadIdx.x;
        uint32_t tot = 0;
        for (uint32_t w = 0; w < nw; ++w) { const uint32_t v = s_cnt[c * 16 + w]; s_cnt[c * 16 + w] = tot; tot += v; }
        s_cnt[NC * 16 + c] = tot ? atomicAdd(counts + (c * kShards + shard) * kCntStride, tot) : 0u;
    }
    __syncthreads();
    uint32_t slot = 0;
    if (cls >= 0) {
        const uint32_t local = s_cnt[NC * 16 + cls] + s_cnt[cls * 16 + wave] + below;
        if (local < shard_cap) slot = shard * shard_cap + local;
        else { raise_fault(RT_FAULT_SHARD); slot = kNoSlot; }     // never write past the shard
    }
    __syncthreads();                       // s_cnt is reused by the next call
    return slot;
}

// =====================================================================
// k_extend — one closest-hit query per live path.  Misses are finished on
// the spot (sky); hits are appended to the queue of their material type so
// each shade kernel runs one material's code (wavefront material queues).
// =====================================================================
template <int F>
__global__ __launch_bounds__(256) void k_extend(const DevScene sc, const RenderParams rp,
                                                const PathState st, const QView in, uint32_t n, HitBuf hit,
                                                uint32_t shard_cap, uint32_t* __restrict__ counts,
                                                const bool depth0) {
    extern __shared__ uint32_t s_lstack[];          // per-lane BVH stack, 256 x sc.lane_stack (dynamic LDS)
    const int LS = sc.lane_stack;
    __shared__ uint32_t s_cnt[4 * 16 + 4];
    constexpr bool BEZ = (F & kFeatCurves) != 0;
    constexpr bool MED = (F & kFeatExtra) != 0;
    __shared__ BezWave s_bw[BEZ ? 4 : 1];
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    int cls = -1;
    uint32_t i = 0;
    HitRec hr{};
    if (k < n) {
        i = qphys(qmap(in), k);
        const RayRec R = st.ray[i];
        const v3 o = mk(R.ox, R.oy, R.oz);
        const v3 d = mk(R.dx, R.dy, R.dz);
        double t;
        Rng g;
        if (MED) {
            uint32_t pix, smp;
            wid_key(rp, depth0 ? i : st.path[i].wid, pix, smp);
            g.init(rp.k0, rp.k1, pix, smp, depth0 ? st.rng0[i] : st.path[i].rng);
        }
        const int32_t leaf = closest_hit<F>(sc, o, d, depth0 ? st.tm[i] : 0.0, t, s_lstack + threadIdx.x, LS,
                                            &s_bw[BEZ ? (threadIdx.x >> 6) : 0], &g, tree0_hbm(sc), treeA_hbm(sc));
        if (MED) {                                   // draws taken inside media
            if (depth0) st.rng0[i] = g.ctr; else st.path[i].rng = g.ctr;
        }
        if (leaf < 0) {
            const v3 L = sky_radiance(sc, d);
            if (depth0) {                                // throughput 1: (* 1 x) = x
                put_sample(rp, i, 1.0 * L.x, 1.0 * L.y, 1.0 * L.z);
            } else {
                const PathRec P = st.path[i];
                put_sample(rp, P.wid, P.tr * L.x, P.tg * L.y, P.tb * L.z);
            }
        } else {
            hr = HitRec{t, leaf, i};
            cls = sc.leaves[leaf].mtype;
        }
    }
    const uint32_t slot = block_append<4>(cls, counts, shard_cap, s_cnt);
    if (cls >= 0 && slot != kNoSlot) hit.h[(size_t)cls * hit.stride + slot] = hr;
}

// =====================================================================
// k_hit_rays — the world's closest hit for a caller's batch of rays
// (rt_hit_rays; hit-obj-list geometry.scm:33-50 over the scene list, as the
// integrator calls it at main.scm:104): t and the leaf's material, or -1.
// The same closest_hit<F> the extend kernels run; a diagnostic / test probe,
// not on the render path.  Scenes with media are refused by the host (the
// medium's hit test draws from the path's random stream).
// =====================================================================
template <int F>
__global__ __launch_bounds__(256) void k_hit_rays(const DevScene sc, const double* __restrict__ rays, uint32_t n,
                                                  double* __restrict__ out_t, int32_t* __restrict__ out_mat) {
    extern __shared__ uint32_t s_lstack[];
    constexpr bool BEZ = (F & kFeatCurves) != 0;
    __shared__ BezWave s_bw[BEZ ? 4 : 1];
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n) return;
    const double* r = rays + 7 * (size_t)k;
    double t = 0.0;
    const int32_t leaf = closest_hit<F>(sc, mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6], t,
                                        s_lstack + threadIdx.x, sc.lane_stack, &s_bw[BEZ ? (threadIdx.x >> 6) : 0],
                                        nullptr, tree0_hbm(sc), treeA_hbm(sc));
    out_t[k] = leaf < 0 ? 0.0 : t;
    out_mat[k] = leaf < 0 ? -1 : sc.leaves[leaf].mat;
}

// Wave-level append into the sharded material queues (block_append's layout:
// class c, shard x -> counter (c * kShards + x), slot x * shard_cap + rank)
// for kernels whose lanes finish at different loop iterations.  One atomic
// per distinct (class, shard) among the wave's finishing lanes.
// SPILL: the shard is the caller's choice and not bounded by it (k_extend_curves picks one per wave, and
// its waves claim rays dynamically), so an item that finds its shard full moves on to the next shard, up
// to all kShards of them (together they hold every item of the launch).  The full shard's entries below
// its capacity were all written (the lanes that got them), so the consumers' clamped counts stay exact.
template <bool SPILL = false>
__device__ __forceinline__ uint32_t wave_append(const int cls, const uint32_t shard, uint32_t* __restrict__ counts,
                                                const uint32_t shard_cap) {
    const uint32_t lane = threadIdx.x & 63u;
    bool pending = cls >= 0;
    uint32_t key = pending ? (uint32_t)cls * kShards + shard : 0u;
    uint32_t tries = 0;
    uint32_t slot = 0;
    unsigned long long m = __ballot(pending);
    while (m) {
        const int leader = __ffsll((long long)m) - 1;
        const uint32_t K = (uint32_t)__shfl((int)key, leader, 64);
        const bool mine = pending && key == K;
        const unsigned long long mk = __ballot(mine);
        uint32_t base = 0;
        if ((int)lane == leader) base = atomicAdd(counts + K * kCntStride, (uint32_t)__popcll(mk));
        base = (uint32_t)__shfl((int)base, leader, 64);
        if (mine) {
            const uint32_t local = base + lanes_below(mk);
            if (local < shard_cap) {
                slot = (K % kShards) * shard_cap + local;
                pending = false;
            } else if (SPILL && ++tries < (uint32_t)kShards) {
                key = (K / kShards) * kShards + ((K + 1u) % kShards);     // the same class, the next shard
            } else {
                raise_fault(RT_FAULT_SHARD);                              // never write past the shard
                slot = kNoSlot;
                pending = false;
            }
        }
        m = __ballot(pending);
    }
    return slot;
}

// =====================================================================
// k_extend_curves — closest hit for scenes whose world BVH holds curves
// (bezier.scm), persistent: a lane whose ray is resolved takes the next one
// (one claim atomic per wave), so a wave is not held by its longest ray
// (stats build: a wave looped 417 times for 77 steps per ray on average).
// Same traversal, candidate batching and group order as closest_hit /
// bvh_closest_curves; a ray finishes once its traversal has ended and every
// curve candidate it queued has been resolved by a batch (W.done).
// =====================================================================
static_assert(4 * sizeof(BezWave) + 256 * sizeof(uint32_t) * RT_CURVE_LDS_STACK <= 160 * 1024 / RT_CURVE_WAVES,
              "k_extend_curves: RT_CURVE_WAVES blocks of BezWave state and LDS stack columns must fit a CU's LDS");
#ifndef RT_CURVE_PREFETCH
#define RT_CURVE_PREFETCH 1            // load the lane's next BVH4 node one iteration ahead (32 VGPRs)
#endif
// FUSE (1: device libm, 2: the exact libm): every depth from fz.depth on in one launch, so the launch
// drains once per chunk instead of once per depth (C5: ~1.1 ms per depth launch).  A lane whose ray is
// resolved parks its hit in the wave's hand-off ring (FuseHit) and takes the next ray at once; when 64
// hits are parked, every lane of the wave shades one (shade_hit, the wavefront shade's own code: any
// material, no Perlin tables, no light mixture — launch_extend checks the scene), whatever its own walk
// is doing, so shading runs on whole waves (round 5 shaded on the ~20 lanes of a finishing batch).  A
// scattered path is stored in place (same slot) and listed as ready (FuseReady); free lanes take ready
// paths before new rays.  Paths that end write their sample; continuation segments are counted into
// *fz.segs.
template <bool EX>
__device__ __forceinline__ bool fused_shade(const DevScene& sc, const RenderParams& rp, PathRegs& p, const double t,
                                            const int32_t leaf, v3& L);   // below shade_hit
template <int FUSE = 0>
__global__ __launch_bounds__(256, RT_CURVE_WAVES) void k_extend_curves(const DevScene sc, const RenderParams rp,
                                                       const PathState st, const QView in, uint32_t n, HitBuf hit,
                                                       uint32_t shard_cap, uint32_t* __restrict__ counts,
                                                       const bool depth0, unsigned int* __restrict__ claim,
                                                       const CurveFuse fz) {
    extern __shared__ uint32_t s_lstack[];          // per-lane BVH4 stack column, 256 x sc.lds4 (dynamic LDS)
    __shared__ BezWave s_bw[4];
    BezWave& W = s_bw[threadIdx.x >> 6];
    uint32_t* lstk = s_lstack + threadIdx.x;
    const uint32_t stride = blockDim.x;
    const uint32_t lane = threadIdx.x & 63u;
    const QMap qm = qmap(in);
    const int32_t bs = sc.leaf_base[LEAF_SPHERE], bm = sc.leaf_base[LEAF_MSPHERE], bz = sc.leaf_base[LEAF_BEZIER];
    int gb = 0;                                     // the world BVH group (commit_scene builds at most one)
    while (gb < sc.n_groups && sc.groups[gb].type != GROUP_BVH) ++gb;
    bool active = false, exhausted = false, trav = false;
    uint32_t i = 0, queued = 0;
    uint32_t dep = FUSE ? fz.depth : 0u, fsegs = 0;  // FUSE: the lane's path depth, continuation segments
    // The ray itself (o, d, time) is not kept in registers across iterations: the BVH step needs only
    // its box-test form and t scale, the sphere leaves and the finish reload it (ray_of below), so stage
    // B's walk state fits beside the loop's (registers cap the waves per SIMD, RT_CURVE_WAVES)
    double tscale = 1.0, closest = kTmax;
    int32_t best = -1, node = 0;
    // best's material class (leaf_cls), loaded whenever best changes: the load is in flight while the
    // traversal goes on, not a round trip of the finish
    int32_t bcls = -1;
    BoxRayW br{};                                   // rays from anywhere (BoxRayW)
#if RT_CURVE_PREFETCH
    BvhNode4 N{};                                   // the lane's next node, loaded one iteration ahead
#endif
    auto ray_of = [&](v3& o, v3& d, double& tm) {
        const RayRec R = st.ray[i];
        o = mk(R.ox, R.oy, R.oz);
        d = mk(R.dx, R.dy, R.dz);
        tm = depth0 ? st.tm[i] : 0.0;
    };
    int sp = 0, pb = 0, pe = 0;
    // the walk's stack: LDS column for the first lds4 entries, the global overflow area past them
    const int lds4 = sc.lds4;                       // <= kCurveLdsStack (rt_api.cpp): the column's allocated depth
    const uint32_t ovf_lane = blockIdx.x * 256u + threadIdx.x;
    const int scap = max(lds4, sc.stack4);          // commit_scene's bound on the walk's stack
    auto push = [&](const int32_t e) {
        if (sp >= scap) { raise_fault(RT_FAULT_PATH); return; }
        if (sp < lds4) lstk[sp * stride] = (uint32_t)e;
        else sc.stk_ovf[(size_t)(sp - lds4) * sc.ovf_lanes + ovf_lane] = (uint32_t)e;
        ++sp;
    };
    auto pop = [&]() -> int32_t {
        --sp;
        return (int32_t)(sp < lds4 ? lstk[sp * stride] : sc.stk_ovf[(size_t)(sp - lds4) * sc.ovf_lanes + ovf_lane]);
    };
    // a lane takes ray i (its closest hit from scratch): the groups before the BVH, then the BVH4 walk
    auto start_ray = [&]() {
        v3 o, d;
        double tm;
        ray_of(o, d, tm);
        closest = kTmax;
        best = -1;
        for (int g = 0; g < gb; ++g) group_closest<0>(sc, sc.groups[g], o, d, tm, closest, best, nullptr);
        bcls = best >= 0 ? (int32_t)sc.leaf_cls[best] : -1;
        br = box_ray_w(o, d);
        tscale = fmax(1.0, 1.0 / sqrt(dot(d, d)));
        bez_ray(o, d, W.ray[lane]);
        sp = 0; node = sc.bvh4_root; trav = gb < sc.n_groups;
#if RT_CURVE_PREFETCH
        if (trav && node >= 0) N = sc.bvh4[node];
#endif
    };
    uint32_t qn = 0, svn = 0;                       // wave-uniform: queued candidates, survivors
    // the wave's survivor ring (launch_extend_curves keeps the grid within sc.ring_waves) and the ring
    // slot of survivor 0: survivors are taken oldest first, so slot = rtail + position
    BezRoot* const ring = reinterpret_cast<BezRoot*>(sc.bez_ring) +
                          (size_t)(blockIdx.x * 4u + (threadIdx.x >> 6)) * (size_t)kBezRing;
    uint32_t rtail = 0;
    // FUSE: the wave's hand-off rings (parked hits, ready paths; wave-uniform heads and tails)
    FuseHit* const pk = FUSE ? reinterpret_cast<FuseHit*>(sc.fuse_ring + (size_t)(blockIdx.x * 4u + (threadIdx.x >> 6)) *
                                                          kFuseWaveBytes) : nullptr;
    FuseReady* const rd = reinterpret_cast<FuseReady*>(pk + kFuseRing);
    uint32_t pk_head = 0, pk_tail = 0, rd_head = 0, rd_tail = 0;
    // a ray takes at most one step per node / leaf and one queue step per two curves: bound its
    // working iterations (a valid walk stays far below)
    const uint32_t ray_cap = g_curve_ray_cap ? g_curve_ray_cap : 4u * (uint32_t)(sc.n_bvh2 + sc.n_bleaf + sc.n_bez) + 4096u;
    uint32_t ray_it = 0;
    // a lane whose ray hit the cap stays out of the refill for good: candidates it queued may still sit
    // in W.q / W.sv, and a new ray in the lane would take their results (W.done, hz / hkey)
    bool dead = false;
#ifdef RT_STATS
    uint32_t st_iter = 0, st_steps = 0, st_busy = 0, st_wait = 0, st_flush = 0;
    const unsigned long long st_clk0 = __builtin_amdgcn_s_memtime();
    unsigned long long st_clk_a = 0, st_clk1 = 0, st_clk2 = 0, st_clk3 = 0, st_t = 0;
#endif
    for (;;) {
        // only iterations in which the lane itself works count: one waiting for a batch
        // other lanes trigger is bounded by their work (the last batch runs once no lane can add)
        if (active && (trav || pb < pe) && ++ray_it > ray_cap) {
            raise_fault(RT_FAULT_PATH); active = false; trav = false; pb = pe; dead = true;
        }
#ifdef RT_STATS
        ++st_iter;
        if (active && trav && pb >= pe) ++st_steps;
        if (active) ++st_busy;
        if (active && !trav && pb >= pe) ++st_wait;
#endif
#ifdef RT_STATS
        st_t = __builtin_amdgcn_s_memtime();
#endif
        // 1. rays whose traversal ended and whose curves are all resolved: the
        //    groups after the BVH, then miss (sky) or hit + material queue
        int cls = -1;
        HitRec hr{};
        // Finished lanes are written out (and refilled in step 2) together, once RT_CURVE_FINISH_BATCH of
        // them are ready, every active lane is, or the ray list is exhausted: a miss's path-record gather,
        // the queue append's returning atomics and the refill's claim and ray loads are dependent
        // round trips, which cost the wave the same whether one lane or sixteen take them.
        const bool fin = active && !trav && pb >= pe && W.done[lane] == queued;
        const unsigned long long fin_m = __ballot(fin);
        const bool flush = fin_m != 0ull && (exhausted || __popcll(fin_m) >= RT_CURVE_FINISH_BATCH ||
                                             fin_m == __ballot(active));
        if constexpr (FUSE != 0) {
            // park every resolved ray at once (its lane takes the next one in step 2)
            if (fin) {
                pk[(pk_tail + lanes_below(fin_m)) & (uint32_t)(kFuseRing - 1)] =
                    FuseHit{i, (uint32_t)(best + 1) | (dep << kFuseLeafBits), closest};
                active = false;
            }
            pk_tail += (uint32_t)__popcll(fin_m);
            // a shading round: 64 parked hits, or — once no new rays are left and no ready path waits — the
            // ones there are, when the finishing batch's share of the wave is idle or the wave is drained
            const uint32_t npk = pk_tail - pk_head;
            bool round = npk >= 64u;  // a whole wave (48 / 32: -0.1 / -1.1 % at 1 spp, -0.9 / -2.9 % at 8)
            if (!round && npk > 0u && exhausted && rd_head == rd_tail) {
                const unsigned long long am = __ballot(active);
                round = am == 0ull || __popcll(__ballot(!active && !dead)) >= RT_CURVE_FINISH_BATCH;
            }
            if (round) {
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // the parked hits other lanes wrote
                wave_sync();
                const uint32_t take = npk < 64u ? npk : 64u;
                bool go = false;
                uint32_t gslot = 0, gdep = 0;
                if (lane < take) {
                    const FuseHit h = pk[(pk_head + lane) & (uint32_t)(kFuseRing - 1)];
                    double t = h.t;
                    int32_t leaf = (int32_t)(h.leaf_dep & ((1u << kFuseLeafBits) - 1u)) - 1;
                    PathRegs p;
                    load_path(st, h.slot, p, rp, h.leaf_dep >> kFuseLeafBits);
                    for (int g = gb + 1; g < sc.n_groups; ++g) group_closest<0>(sc, sc.groups[g], p.o, p.d, p.time, t, leaf, nullptr);
                    v3 L;
                    if (leaf < 0) L = sky_radiance(sc, p.d);
                    else go = fused_shade<FUSE == 2>(sc, rp, p, t, leaf, L);
                    if (go) {
                        store_path(st, h.slot, p);
                        gslot = h.slot;
                        gdep = p.depth;
                        ++fsegs;
                    } else {
                        write_sample(rp, p, L);
                    }
                }
                pk_head += take;
                const unsigned long long gm = __ballot(go);
                if (go) rd[(rd_tail + lanes_below(gm)) & (uint32_t)(kFuseRing - 1)] = FuseReady{gslot, gdep};
                rd_tail += (uint32_t)__popcll(gm);
                if (rd_tail - rd_head > (uint32_t)kFuseRing || pk_tail - pk_head > (uint32_t)kFuseRing)
                    raise_fault(RT_FAULT_PATH);                  // cannot happen (FuseHit, rt_device.h)
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // the paths and ready entries just stored
                wave_sync();
            }
        } else if (fin && flush) {
            if (gb + 1 < sc.n_groups || best < 0) {          // the groups after the BVH or the sky: the ray again
                v3 o, d;
                double tm;
                ray_of(o, d, tm);
                for (int g = gb + 1; g < sc.n_groups; ++g) group_closest<0>(sc, sc.groups[g], o, d, tm, closest, best, nullptr);
                if (gb + 1 < sc.n_groups && best >= 0) bcls = sc.leaf_cls[best];
                if (best < 0) {
                    const v3 L = sky_radiance(sc, d);
                    if (depth0) {                            // throughput 1: (* 1 x) = x
                        put_sample(rp, i, 1.0 * L.x, 1.0 * L.y, 1.0 * L.z);
                    } else {
                        const PathRec P = st.path[i];
                        put_sample(rp, P.wid, P.tr * L.x, P.tg * L.y, P.tb * L.z);
                    }
                }
            }
            if (best >= 0) {
                hr = HitRec{closest, best, i};
                cls = bcls;                                  // a byte per leaf (1 MB at C5), not the 128-B record
            }
            active = false;
        }
        // one shard per wave: the finishing lanes' appends take one returning atomic per class (a per-ray
        // shard, k / 256, spread a batch over several shards, one dependent atomic each: -0.8 % at C5).
        // Waves claim rays dynamically, so a shard's share is not bounded by n / kShards: a full shard
        // spills into the next (wave_append<true>)
        if constexpr (FUSE == 0) {
            const uint32_t slot = wave_append<true>(cls, (blockIdx.x * 4u + (threadIdx.x >> 6)) & (uint32_t)(kShards - 1),
                                                    counts, shard_cap);
            if (cls >= 0 && slot != kNoSlot) hit.h[(size_t)cls * hit.stride + slot] = hr;
        }
#ifdef RT_STATS
        { const unsigned long long t = __builtin_amdgcn_s_memtime(); st_clk1 += t - st_t; st_t = t; }
#endif
        // 2. free lanes take the next rays: FUSE, the wave's ready paths first; then claimed positions in the
        //    input queue
        unsigned long long need = __ballot(!active && !dead);
        if constexpr (FUSE != 0) {
            const uint32_t nrd = rd_tail - rd_head;
            if (need && nrd) {
                const uint32_t cnt = (uint32_t)__popcll(need), take = cnt < nrd ? cnt : nrd;
                const uint32_t r = lanes_below(need);
                if (!active && !dead && r < take) {
                    const FuseReady e = rd[(rd_head + r) & (uint32_t)(kFuseRing - 1)];
                    i = e.slot;
                    dep = e.depth;
                    start_ray();
                    W.done[lane] = 0u;
                    queued = 0u;
                    pb = pe = 0;
                    active = true;
                    ray_it = 0;
                }
                rd_head += take;
                need = __ballot(!active && !dead);
            }
        }
        if (need && !exhausted) {
            const uint32_t cnt = (uint32_t)__popcll(need);
            const int leader = __ffsll((long long)need) - 1;
            uint32_t base = 0;
            if ((int)lane == leader) base = atomicAdd(claim, cnt);
            base = (uint32_t)__shfl((int)base, leader, 64);
            if (base + cnt >= n) exhausted = true;
            if (!active && !dead) {
                const uint32_t kk = base + lanes_below(need);
                if (kk < n) {
                    {
                        i = qphys(qm, kk);
                        dep = FUSE ? fz.depth : 0u;
                        start_ray();
                    }
                    W.done[lane] = 0u;
                    queued = 0u;
                    pb = pe = 0;
                    active = true;
                    ray_it = 0;
                }
            }
        }
        if (__ballot(active) == 0ull) {              // every queued candidate has been resolved
            if constexpr (FUSE == 0) break;
            // FUSE: done once nothing is parked or ready (or no lane is left to take a path: a fault)
            if ((exhausted && pk_head == pk_tail && rd_head == rd_tail) || __ballot(!dead) == 0ull) break;
        }
#ifdef RT_STATS
        { const unsigned long long t = __builtin_amdgcn_s_memtime(); st_clk2 += t - st_t; st_t = t; }
#endif
        // 3. one BVH4 step (bvh_closest_curves over the collapsed tree): the node's hit children
        //    nearest first, the nearest entered, the others pushed
        if (active && trav && pb >= pe) {
            if (node >= 0) {
#if !RT_CURVE_PREFETCH
                const BvhNode4 N = sc.bvh4[node];
#endif
                const float tcap = f32_up(closest * tscale);
                float key[4];
                int32_t ref[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float tx0 = fmaf(N.lo[0][j], br.ix, -br.lx), tx1 = fmaf(N.hi[0][j], br.ix, -br.hx);
                    const float ty0 = fmaf(N.lo[1][j], br.iy, -br.ly), ty1 = fmaf(N.hi[1][j], br.iy, -br.hy);
                    const float tz0 = fmaf(N.lo[2][j], br.iz, -br.lz), tz1 = fmaf(N.hi[2][j], br.iz, -br.hz);
                    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
                    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tcap));
                    key[j] = (tn <= tf && j < N.n) ? tn : INFINITY;   // slab ends are finite: INFINITY = missed
                    ref[j] = N.ref[j];
                }
                auto cswap = [&](const int x, const int y) {
                    const bool sw = key[y] < key[x];
                    const float kx = key[x];
                    const int32_t rx = ref[x];
                    key[x] = sw ? key[y] : kx; key[y] = sw ? kx : key[y];
                    ref[x] = sw ? ref[y] : rx; ref[y] = sw ? rx : ref[y];
                };
                // a full sort: with only the nearest found (the rest pushed in slot order) C5 loses 4 %
                cswap(0, 1); cswap(2, 3); cswap(0, 2); cswap(1, 3); cswap(1, 2);
                if (key[0] == INFINITY) {
                    if (sp == 0) trav = false;
                    else node = pop();
                } else {
                    // the hit children beyond the nearest, farthest first (the keys are sorted, misses last)
                    const int np = (key[1] != INFINITY) + (key[2] != INFINITY) + (key[3] != INFINITY);
                    if (sp + np <= lds4) {                      // all in the LDS column: no per-push branches
                        uint32_t* top = lstk + sp * stride;
                        if (np >= 3) { top[0] = (uint32_t)ref[3]; top += stride; }
                        if (np >= 2) { top[0] = (uint32_t)ref[2]; top += stride; }
                        if (np >= 1) top[0] = (uint32_t)ref[1];
                        sp += np;
                    } else {
                        if (key[3] != INFINITY) push(ref[3]);
                        if (key[2] != INFINITY) push(ref[2]);
                        if (key[1] != INFINITY) push(ref[1]);
                    }
                    node = ref[0];
                }
                // a leaf holding one curve: queued from its ref in this step (no leaf record, no extra step)
                if (trav && ~node >= kDirectCurve) {
                    pb = ~node - kDirectCurve; pe = pb + 1;
                    if (sp == 0) trav = false;
                    else node = pop();
                }
            } else if (~node >= kDirectCurve) {                   // the root, or a popped direct leaf
                pb = ~node - kDirectCurve; pe = pb + 1;
                if (sp == 0) trav = false;
                else node = pop();
            } else {
                const BvhLeaf L = sc.bleaf[~node];
                if (L.sn + L.mn > 0) {                              // spheres in the curve tree: the ray again
                    v3 o, d;
                    double tm;
                    ray_of(o, d, tm);
                    const double a = dot(d, d), ia = 1.0 / a;
                    for (int s = L.sb; s < L.sb + L.sn; ++s) {
                        const SphereRec S = sc.sph[s];
                        sphere_test(o, d, a, ia, mk(S.cx, S.cy, S.cz), S.rr, bs + s, closest, best);
                    }
                    for (int s = L.mb; s < L.mb + L.mn; ++s) {
                        const MSphereRec S = sc.msph[s];
                        const double frac = (tm - S.t0) / S.den;
                        const v3 cen = mk(S.c0x, S.c0y, S.c0z) + mk(S.dcx, S.dcy, S.dcz) * frac;
                        sphere_test(o, d, a, ia, cen, S.rr, bm + s, closest, best);
                    }
                    bcls = best >= 0 ? (int32_t)sc.leaf_cls[best] : -1;
                }
                pb = L.bb; pe = L.bb + L.bn;
                if (sp == 0) trav = false;
                else node = pop();
            }
        }
#if RT_CURVE_PREFETCH
        // the next node's record, in flight while the batches below run (+5 % at C5 with 2 waves per SIMD)
        if (active && trav && node >= 0) N = sc.bvh4[node];
#endif
#ifdef RT_STATS
        { const unsigned long long t = __builtin_amdgcn_s_memtime(); st_clk3 += t - st_t; st_t = t; }
#endif
        // 4. queue one of the lane's curve candidates (kBezQ: at most one per lane per step; a leaf with
        //    several curves queues them over the next iterations, its traversal paused meanwhile)
        {
            const bool has = active && pb < pe;
            const unsigned long long m = __ballot(has);
            if (has) { W.q[qn + lanes_below(m)] = ((uint32_t)pb << 6) | lane; ++pb; ++queued; }
            qn += (uint32_t)__popcll(m);
        }
        // 5. batches: root culls at 64 queued candidates, subdivisions in
        //    multiples of 64 (everything once no lane can add candidates)
        const bool more = __ballot(active && (trav || pb < pe)) != 0ull;
#if RT_BEZ_WAIT_FLUSH
        const bool press = __popcll(__ballot(active && !trav && pb >= pe && W.done[lane] != queued)) >= RT_BEZ_WAIT_FLUSH;
#else
        constexpr bool press = false;
#endif
        if (qn >= (uint32_t)RT_BEZ_QFLUSH || ((!more || press) && (qn > 0u || svn > 0u))) {
#ifdef RT_STATS
            ++st_flush;
#endif
            W.cl[lane] = closest;
            wave_sync();
#ifdef RT_STATS
            const unsigned long long ca = __builtin_amdgcn_s_memtime();
#endif
            svn = bez_stage_a<true>(sc, W, qn, svn, ring, rtail);
#ifdef RT_STATS
            st_clk_a += __builtin_amdgcn_s_memtime() - ca;
#endif
            qn = 0;
            const uint32_t nb = (more && !press) ? (svn >= (uint32_t)RT_BEZ_HOLD ? svn - svn % 64u : 0u) : svn;
            if (nb > 0u) {
                W.hz[lane] = INFINITY;
                W.hkey[lane] = 0ull;
                wave_sync();
                // the ring entries other lanes wrote: stores complete and visible to the wave's loads
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
                bez_stage_b<true>(sc, W, nb, svn, ring, rtail);
                svn -= nb;
                rtail += nb;
                if (active) {
                    const int32_t b0 = best;
                    bez_take_batch(sc, W, lane, bz, closest, best);
                    if (best != b0) bcls = sc.leaf_cls[best];
                }
                wave_sync();
            }
        }
    }
    if constexpr (FUSE != 0) {                       // continuation segments: wave sum, one atomic per wave
        for (int off = 32; off > 0; off >>= 1) fsegs += __shfl_xor(fsegs, off, 64);
        if (lane == 0u && fsegs) atomicAdd(fz.segs, (unsigned long long)fsegs);
    }
#ifdef RT_STATS
    RT_STAT(20, st_steps); RT_STAT(21, st_busy); RT_STAT(22, st_wait);
    if (lane == 0u) {
        RT_STAT(23, st_iter); RT_STAT(24, 1); RT_STAT(25, st_flush);
        RT_STAT(40, __builtin_amdgcn_s_memtime() - st_clk0); RT_STAT(41, st_clk_a);
        RT_STAT(42, st_clk1); RT_STAT(43, st_clk2); RT_STAT(44, st_clk3);   // kernel / stage A clocks per wave
    }
#endif
}

#ifndef RT_EXTLDS_BLOCK
#define RT_EXTLDS_BLOCK 512
#endif
// Waves per SIMD the LDS kernels are compiled for (VGPR cap 512 / waves).
// k_extend_lds at 8 (64 VGPRs, spilling per-ray state outside the node loop)
// measured +5 % on the overlapped two-lane frame against 6 (80 VGPRs), -1 %
// with one lane; k_camera stays at 6 (8 made no difference and spills more).
#ifndef RT_EXTLDS_WAVES
#define RT_EXTLDS_WAVES 8
#endif
#ifndef RT_CAMERA_WAVES
#define RT_CAMERA_WAVES 6
#endif
constexpr int kExtLdsBlock = RT_EXTLDS_BLOCK;
// Copy n records of T from HBM into LDS, 16-B words, all threads of the block.
template <class T>
__device__ __forceinline__ void stage_lds(T* dst, const T* src, const int n, const int nthreads) {
    static_assert(sizeof(T) % 16 == 0, "records are whole 16-B words");
    const uint4* g = reinterpret_cast<const uint4*>(src);
    uint4* l = reinterpret_cast<uint4*>(dst);
    const int words = n * (int)(sizeof(T) / 16);
    for (int k = threadIdx.x; k < words; k += nthreads) l[k] = g[k];
}

// Work distribution and hit-queue append of the persistent LDS kernels: a
// block takes kExtLdsBlock consecutive items per grid-stride step, each wave
// its own 64 of them, appended with wave_append (one atomic per wave and
// class, no barrier), so a wave is never held by a slower wave of its block
// (against block_append's one atomic per block and three barriers: +3 %).
// Items keep their shard (blockIdx % kShards); queue order does not change
// images (a path's result does not depend on its queue position).
__device__ __forceinline__ uint32_t ext_first() { return blockIdx.x * kExtLdsBlock + (threadIdx.x & ~63u); }
__device__ __forceinline__ uint32_t ext_lid() { return threadIdx.x & 63u; }
__device__ __forceinline__ uint32_t ext_append(const int cls, uint32_t* __restrict__ counts, const uint32_t shard_cap,
                                               uint32_t*) {
    return wave_append(cls, blockIdx.x & (uint32_t)(kShards - 1), counts, shard_cap);
}

// Dynamic LDS the persistent kernels carve (host and device use the same
// formula: the kernels check it against the allocation they were given).
// Layout: tree nodes | leaves | sphere records [| moving spheres] | 16-bit
// lane stacks | fsph -> leaf id (time-0 tree) | leaf -> material class (bytes).
__host__ __device__ __forceinline__ size_t lds_tail_bytes(const DevScene& sc) {
    return ((size_t)sc.n_fsph * 4 + 15) / 16 * 16 + ((size_t)sc.n_leaves + 15) / 16 * 16;
}
// time-0 leaf records the LDS kernels stage: none for SOLO scenes (direct leaves)
__host__ __device__ __forceinline__ int tree0_lds_leaves(const DevScene& sc) { return sc.bvh_solo ? 0 : sc.n_fbleaf; }
__host__ __device__ __forceinline__ size_t extend_lds_need(const DevScene& sc) {
    return (size_t)sc.n_fbvh2 * sizeof(BvhNode2) + (size_t)tree0_lds_leaves(sc) * sizeof(BvhLeaf) +
           (size_t)sc.n_fsph * sizeof(SphereRec) +
           (size_t)RT_EXTLDS_BLOCK * (size_t)(sc.lane_stack > 0 ? sc.lane_stack : 1) * sizeof(uint16_t) +
           lds_tail_bytes(sc);
}
__host__ __device__ __forceinline__ size_t camera_lds_need(const DevScene& sc) {     // all-times tree
    return (size_t)sc.n_bvh2 * sizeof(BvhNode2) + (size_t)sc.n_bleaf * sizeof(BvhLeaf) +
           (size_t)sc.n_sph * sizeof(SphereRec) + (size_t)sc.n_msph * sizeof(MSphereRec) +
           (size_t)RT_EXTLDS_BLOCK * (size_t)(sc.lane_stack > 0 ? sc.lane_stack : 1) * sizeof(uint16_t) +
           lds_tail_bytes(sc);
}
// stage n 32-bit words (fid, packed class bytes)
__device__ __forceinline__ void stage_words(uint32_t* dst, const uint32_t* src, const int n, const int nthreads) {
    for (int k = threadIdx.x; k < n; k += nthreads) dst[k] = src[k];
}

// =====================================================================
// k_extend_lds — k_extend for launches whose rays all carry time +0.0 (every
// depth >= 1 launch) in scenes whose time-0 tree fits in LDS: persistent
// blocks stage the tree (nodes, leaves, sphere records) into LDS once and
// grid-stride over the queue, so node fetches cost LDS latency instead of
// L1/L2 latency.  Sphere scenes only (no curves, media or Klein: F = 0).
// =====================================================================

template <bool SOLO>
__global__ __launch_bounds__(kExtLdsBlock, RT_EXTLDS_WAVES) void k_extend_lds(const DevScene sc, const RenderParams rp,
                                                             const PathState st, const QView in, uint32_t n,
                                                             HitBuf hit, uint32_t shard_cap,
                                                             uint32_t* __restrict__ counts, const uint32_t lds_bytes,
                                                             unsigned long long* __restrict__ err) {
    extern __shared__ uint4 s_dyn[];
    __shared__ uint32_t s_cnt[4 * 16 + 4];
    const int nn = sc.n_fbvh2, nl = SOLO ? 0 : sc.n_fbleaf, ns = sc.n_fsph;
    if (extend_lds_need(sc) > lds_bytes || (SOLO && !sc.bvh_solo)) {            // the carve below would leave the allocation
        if (threadIdx.x == 0) { atomicOr(err, 1ull); raise_fault(RT_FAULT_LDS); }
        return;
    }
    BvhNode2* s_nodes = reinterpret_cast<BvhNode2*>(s_dyn);
    BvhLeaf* s_leaves = reinterpret_cast<BvhLeaf*>(s_nodes + nn);
    SphereRec* s_sph = reinterpret_cast<SphereRec*>(s_leaves + nl);
    uint16_t* s_lstack = reinterpret_cast<uint16_t*>(s_sph + ns);
    int32_t* s_fid = reinterpret_cast<int32_t*>(s_lstack + (size_t)kExtLdsBlock * (sc.lane_stack > 0 ? sc.lane_stack : 1));
    uint8_t* s_cls = reinterpret_cast<uint8_t*>(s_fid) + ((size_t)ns * 4 + 15) / 16 * 16;
    stage_lds(s_nodes, sc.fbvh2, nn, kExtLdsBlock);      // the time-0 tree
    if (!SOLO) stage_lds(s_leaves, sc.fbleaf, nl, kExtLdsBlock);
    stage_lds(s_sph, sc.fsph, ns, kExtLdsBlock);
    stage_words(reinterpret_cast<uint32_t*>(s_fid), reinterpret_cast<const uint32_t*>(sc.fid), ns, kExtLdsBlock);
    stage_words(reinterpret_cast<uint32_t*>(s_cls), reinterpret_cast<const uint32_t*>(sc.leaf_cls),
                (sc.n_leaves + 3) / 4, kExtLdsBlock);
    __syncthreads();
    const Tree0 t0{s_nodes, s_leaves, s_sph, s_fid};
    const int LS = sc.lane_stack;
    const QMap qm = qmap(in);
    for (uint32_t base = ext_first(); base < n; base += gridDim.x * kExtLdsBlock) {
        const uint32_t k = base + ext_lid();
        int cls = -1;
        HitRec hr{};
        if (k < n) {
            const uint32_t i = qphys(qm, k);
            const RayRec R = st.ray[i];
            const v3 o = mk(R.ox, R.oy, R.oz);
            const v3 d = mk(R.dx, R.dy, R.dz);
            double t;
            const int32_t leaf = closest_hit_lds<SOLO>(sc, o, d, 0.0, t, s_lstack + threadIdx.x, LS, t0, treeA_hbm(sc));
            if (leaf < 0) {
                const v3 L = sky_radiance(sc, d);
                const PathRec P = st.path[i];
                put_sample(rp, P.wid, P.tr * L.x, P.tg * L.y, P.tb * L.z);
            } else {
                hr = HitRec{t, leaf, i};
                cls = s_cls[leaf];
            }
        }
        const uint32_t slot = ext_append(cls, counts, shard_cap, s_cnt);
        if (cls >= 0 && slot != kNoSlot) hit.h[(size_t)cls * hit.stride + slot] = hr;
    }
}

// =====================================================================
// k_camera — raygen and the first closest-hit query in one persistent kernel
// (depth 0, sphere scenes): each work item's camera ray is traced where it is
// made, against a tree staged in LDS once per block — the all-times tree
// (ALL: the scene has moving spheres, camera rays carry shutter times) or the
// time-0 tree (no moving spheres: it serves every time).  Only rays that hit
// something store their depth-0 state for the shade kernels.
// =====================================================================
template <bool ALL, bool SOLO>
__global__ __launch_bounds__(kExtLdsBlock, RT_CAMERA_WAVES) void k_camera(const DevScene sc, const RenderParams rp,
                                                                          const PathState st, const uint32_t n,
                                                                          HitBuf hit, uint32_t shard_cap,
                                                                          uint32_t* __restrict__ counts,
                                                                          const uint32_t lds_bytes,
                                                                          unsigned long long* __restrict__ err) {
    extern __shared__ uint4 s_dyn[];
    __shared__ uint32_t s_cnt[4 * 16 + 4];
    if ((ALL ? camera_lds_need(sc) : extend_lds_need(sc)) > lds_bytes || (SOLO && !sc.bvh_solo)) {
        if (threadIdx.x == 0) { atomicOr(err, 2ull); raise_fault(RT_FAULT_LDS); }
        return;
    }
    const int nn = ALL ? sc.n_bvh2 : sc.n_fbvh2, nl = ALL ? sc.n_bleaf : (SOLO ? 0 : sc.n_fbleaf);
    const int ns = ALL ? sc.n_sph : sc.n_fsph, nm = ALL ? sc.n_msph : 0;
    BvhNode2* s_nodes = reinterpret_cast<BvhNode2*>(s_dyn);
    BvhLeaf* s_leaves = reinterpret_cast<BvhLeaf*>(s_nodes + nn);
    SphereRec* s_sph = reinterpret_cast<SphereRec*>(s_leaves + nl);
    MSphereRec* s_msph = reinterpret_cast<MSphereRec*>(s_sph + ns);
    uint16_t* s_lstack = reinterpret_cast<uint16_t*>(s_msph + nm);
    int32_t* s_fid = reinterpret_cast<int32_t*>(s_lstack + (size_t)kExtLdsBlock * (sc.lane_stack > 0 ? sc.lane_stack : 1));
    uint8_t* s_cls = reinterpret_cast<uint8_t*>(s_fid) + ((size_t)sc.n_fsph * 4 + 15) / 16 * 16;
    stage_lds(s_nodes, ALL ? sc.bvh2 : sc.fbvh2, nn, kExtLdsBlock);
    if (nl) stage_lds(s_leaves, ALL ? sc.bleaf : sc.fbleaf, nl, kExtLdsBlock);
    stage_lds(s_sph, ALL ? sc.sph : sc.fsph, ns, kExtLdsBlock);
    if (ALL) stage_lds(s_msph, sc.msph, nm, kExtLdsBlock);
    stage_words(reinterpret_cast<uint32_t*>(s_fid), reinterpret_cast<const uint32_t*>(sc.fid), sc.n_fsph, kExtLdsBlock);
    stage_words(reinterpret_cast<uint32_t*>(s_cls), reinterpret_cast<const uint32_t*>(sc.leaf_cls),
                (sc.n_leaves + 3) / 4, kExtLdsBlock);
    __syncthreads();
    const Tree0 t0 = ALL ? tree0_hbm(sc) : Tree0{s_nodes, s_leaves, s_sph, s_fid};
    const TreeA ta = ALL ? TreeA{s_nodes, s_leaves, s_sph, s_msph} : treeA_hbm(sc);
    const int LS = sc.lane_stack;
    for (uint32_t base = ext_first(); base < n; base += gridDim.x * kExtLdsBlock) {
        const uint32_t w = base + ext_lid();
        int cls = -1;
        HitRec hr{};
        if (w < n) {
            v3 o, d;
            double time, t;
            Rng g;
            camera_ray(sc, rp, w, o, d, time, g);
            // ALL: a camera ray whose time is +0.0 (shutter t0 = t1 = 0) takes the time-0 tree from HBM
            const int32_t leaf = closest_hit_lds<SOLO, ALL>(sc, o, d, time, t, s_lstack + threadIdx.x, LS, t0, ta);
            if (leaf < 0) {
                const v3 L = sky_radiance(sc, d);            // throughput 1: (* 1 x) = x
                put_sample(rp, w, 1.0 * L.x, 1.0 * L.y, 1.0 * L.z);
            } else {
                st.ray[w] = ray_rec(o, d);                          // depth-0 state for the shade kernels
                st.tm[w] = time;
                st.rng0[w] = g.ctr;
                hr = HitRec{t, leaf, w};
                cls = s_cls[leaf];
            }
        }
        const uint32_t slot = ext_append(cls, counts, shard_cap, s_cnt);
        if (cls >= 0 && slot != kNoSlot) hit.h[(size_t)cls * hit.stride + slot] = hr;
    }
}

// ------------------------------------------------------------- textures
struct PerlinLds { double ranvec[768]; int32_t perm[768]; };

__device__ __forceinline__ double perlin_noise(const PerlinLds& P, v3 p) {           // perlin.scm:69-90
    const double fx = floor(p.x), fy = floor(p.y), fz = floor(p.z);
    const double u = p.x - fx, v = p.y - fy, w = p.z - fz;
    const long long i = (long long)fx, j = (long long)fy, k = (long long)fz;
    // aliasing quirk (perlin.scm:76, Q2): only the di = dj = 1 corners survive
    v3 c[2];
#pragma unroll
    for (int dk = 0; dk < 2; ++dk) {
        const int h = P.perm[(i + 1) & 255] ^ P.perm[256 + ((j + 1) & 255)] ^ P.perm[512 + ((k + dk) & 255)];
        c[dk] = mk(P.ranvec[3 * h], P.ranvec[3 * h + 1], P.ranvec[3 * h + 2]);
    }
    const double uu = u * u * (3.0 - 2.0 * u);
    const double vv = v * v * (3.0 - 2.0 * v);
    const double ww = w * w * (3.0 - 2.0 * w);
    double acc = 0.0;
#pragma unroll
    for (int di = 0; di < 2; ++di)
#pragma unroll
        for (int dj = 0; dj < 2; ++dj)
#pragma unroll
            for (int dk = 0; dk < 2; ++dk) {
                const double wi = di ? uu : (1.0 - uu);
                const double wj = dj ? vv : (1.0 - vv);
                const double wk = dk ? ww : (1.0 - ww);
                acc += wi * wj * wk * dot(mk(u - di, v - dj, w - dk), c[dk]);
            }
    return acc;
}
__device__ __forceinline__ double perlin_turb(const PerlinLds& P, v3 p) {            // perlin.scm:92-103
    double acc = 0.0, weight = 1.0;
#pragma nounroll
    for (int depth = 0; depth < 7; ++depth) {
        acc = acc + weight * perlin_noise(P, p);
        p = p * 2.0;
        weight = weight * 0.5;
    }
    return fabs(acc);
}
// checker-texture's test (texture.scm:16-23): (< (* (sin 10x) (sin 10y)
// (sin 10z)) 0).  Only the product's sign matters, so each factor's sign is
// found by reducing y = 10x to r = y - k*pi (k = rint(y/pi), three-part pi,
// fma: |error| < 1e-14 for |y| < 2^20): sin y = (-1)^k sin r.  When every |r|
// exceeds 1e-12 the signs are certain, no factor is 0 and the product (above
// 1e-37) cannot underflow, so the test equals the one on libm / OCML sines;
// otherwise (near a zero, huge or NaN arguments) the sines are evaluated.
__device__ __forceinline__ bool sin_sign_neg(const double y, bool& sure) {
    constexpr double kInvPi = 0.31830988618379067154;
    constexpr double kPiA = 3.1415926218032836914;               // pi split in three (Cody-Waite)
    constexpr double kPiB = 3.1786509424591713469e-08;
    constexpr double kPiC = 1.2246467864107188502e-16;
    const double k = rint(y * kInvPi);
    const double r = fma(-k, kPiC, fma(-k, kPiB, fma(-k, kPiA, y)));
    sure = sure && fabs(y) < 1048576.0 && fabs(r) > 1e-12;
    const bool odd = ((long long)k & 1ll) != 0;
    return odd != (r < 0.0);
}
__device__ __forceinline__ bool checker_odd(const v3 p) {
    const double x = 10.0 * p.x, y = 10.0 * p.y, z = 10.0 * p.z;
    bool sure = true;
    const bool nx = sin_sign_neg(x, sure), ny = sin_sign_neg(y, sure), nz = sin_sign_neg(z, sure);
    if (sure) return (nx != ny) != nz;
    // the rare case (an argument within 1e-12 of a multiple of pi): the product itself.  Only its sign is
    // used, and any faithful sine (OCML's as libm's) has the exact sine's sign for a double argument (no
    // nonzero double is a multiple of pi), so the product's sign is libm's
    const double sines = sin(x) * sin(y) * sin(z);
    return sines < 0.0;
}

// PN = false compiles the noise / marble cases out (scenes without them)
template <bool PN>
__device__ __forceinline__ v3 tex_value(const DevScene& sc, const PerlinLds& P, int id, v3 p) {   // texture.scm
    for (int guard = 0; guard < 64; ++guard) {
        const DevTexture t = sc.texs[id];
        if (t.type == TEX_CONSTANT) return mk(t.r, t.g, t.bl);
        if (t.type == TEX_CHECKER) {                                 // :16-23
            id = checker_odd(p) ? t.b : t.a;
            continue;
        }
        if (!PN) return mk(0.0, 0.0, 0.0);
        if (t.type == TEX_NOISE) {                                   // :25-28
            const double nz = perlin_noise(P, p * t.scale);
            return mk(1.0, 1.0, 1.0) * nz;
        }
        // TEX_MARBLE :30-34
        const double m = 0.5 * (1.0 + rt_sin(t.scale * p.z + 10.0 * perlin_turb(P, p)));
        return mk(1.0, 1.0, 1.0) * m;
    }
    return mk(0.0, 0.0, 0.0);
}

// (expt x 5) (material.scm:73) as libm's correctly rounded pow(x, 5.0): x^5
// in double-double (error-free products via fma, relative error < 2^-100
// before the one final rounding), so it rounds like a correctly rounded pow
// except within 2^-100 of a rounding boundary; ~15 instructions instead of
// OCML's log/exp-based pow (which is itself only faithful, <= 1 ulp).
__device__ __forceinline__ double pow5(const double x) {
    const double x2 = x * x, x2l = fma(x, x, -x2);
    double h = x2 * x2;
    double l = fma(x2, x2, -h) + 2.0 * (x2 * x2l);
    const double s = h + l;                                  // renormalise x^4
    l = l - (s - h);
    h = s;
    const double h5 = h * x;
    const double l5 = fma(h, x, -h5) + l * x;
    return h5 + l5;
}
// a hit's texture value from its leaf record: constant and checker-of-constants
// colours are inline (texture.scm:12-23); anything else goes through tex_value
template <bool PN>
__device__ __forceinline__ v3 leaf_tex(const DevScene& sc, const PerlinLds& P, const LeafInfo& li, const v3 p) {
    if (li.tex_kind == TK_CONSTANT) return mk(li.albedo[0], li.albedo[1], li.albedo[2]);
    if (li.tex_kind == TK_CHECKER_CONST)
        return checker_odd(p) ? mk(li.albedo2[0], li.albedo2[1], li.albedo2[2]) : mk(li.albedo[0], li.albedo[1], li.albedo[2]);
    return tex_value<PN>(sc, P, li.tex, p);
}
__device__ __forceinline__ v3 reflect(v3 v, v3 n) { return v - n * (2.0 * dot(v, n)); }  // material.scm:41-43

// --------------------------------------------- light sampling (f2 extension)
// g:pdf-value / g:random for the light, "Rest of Your Life" style (see
// rt_oracle.c light_pdf_value / light_random for the restatement they match).
__device__ __forceinline__ double light_pdf_value(const DevLight& L, const v3 o, const v3 v) {
    if (L.type == LIGHT_RECT) {
        double ok, dk, oa, da, ob, db;
        v3 n;
        if (L.axis == 0) { ok = o.z; dk = v.z; oa = o.x; da = v.x; ob = o.y; db = v.y; n = mk(0.0, 0.0, 1.0); }
        else if (L.axis == 1) { ok = o.y; dk = v.y; oa = o.x; da = v.x; ob = o.z; db = v.z; n = mk(0.0, 1.0, 0.0); }
        else { ok = o.x; dk = v.x; oa = o.y; da = v.y; ob = o.z; db = v.z; n = mk(1.0, 0.0, 0.0); }
        const double t = (L.k - ok) / dk;
        if (t < kTmin || t > kTmax) return 0.0;
        const double A = oa + t * da, Bv = ob + t * db;
        if (A < L.a0 || A > L.a1 || Bv < L.b0 || Bv > L.b1) return 0.0;
        const double area = (L.a1 - L.a0) * (L.b1 - L.b0);
        const double distance_squared = t * t * dot(v, v);
        const double cosine = fabs(dot(v, n) / length(v));
        return distance_squared / (cosine * area);
    }
    // sphere: hit test as geometry.scm:146-171, then 1 / solid angle of the cone
    const v3 c = mk(L.cx, L.cy, L.cz);
    const v3 oc = o - c;
    const double a = dot(v, v), b = dot(oc, v), cc = dot(oc, oc) - L.r * L.r;
    const double disc = b * b - a * cc;
    if (disc <= 0.0) return 0.0;
    double t = (-b - sqrt(disc)) / a;
    if (!(kTmin < t && t < kTmax)) {
        t = (-b + sqrt(disc)) / a;
        if (!(kTmin < t && t < kTmax)) return 0.0;
    }
    const v3 co = c - o;
    const double cos_theta_max = sqrt(1.0 - L.r * L.r / dot(co, co));
    const double solid_angle = 2.0 * kPi * (1.0 - cos_theta_max);
    return 1.0 / solid_angle;
}
template <bool EX>
__device__ __forceinline__ v3 random_to_sphere(const double radius, const double distance_squared, Rng& g) {
    const double r1 = g.next();
    const double r2 = g.next();
    const double z = 1.0 + r2 * (sqrt(1.0 - radius * radius / distance_squared) - 1.0);
    const double phi = 2.0 * kPi * r1;                       // in (0, 2 pi): rt_libm.h's range, no fallback
    return mk((EX ? rtlibm::cos_(phi) : cos(phi)) * sqrt(1.0 - z * z), (EX ? rtlibm::sin_(phi) : sin(phi)) * sqrt(1.0 - z * z), z);
}
template <bool EX>
__device__ __forceinline__ v3 light_random(const DevLight& L, const v3 o, Rng& g) {
    if (L.type == LIGHT_RECT) {
        const double a = L.a0 + g.next() * (L.a1 - L.a0);
        const double b = L.b0 + g.next() * (L.b1 - L.b0);
        const v3 pnt = (L.axis == 0) ? mk(a, b, L.k) : (L.axis == 1) ? mk(a, L.k, b) : mk(L.k, a, b);
        return pnt - o;
    }
    const v3 direction = mk(L.cx, L.cy, L.cz) - o;
    const double distance_squared = dot(direction, direction);
    const v3 w = unit(direction);
    const v3 aa = (fabs(w.x) > 0.9) ? mk(0.0, 1.0, 0.0) : mk(1.0, 0.0, 0.0);
    const v3 vv = unit(cross(w, aa));
    const v3 uu = cross(w, vv);
    const double x = random_to_sphere<EX>(L.r, distance_squared, g).x;  // local: three evaluations (Q29)
    const double y = random_to_sphere<EX>(L.r, distance_squared, g).y;
    const double z = random_to_sphere<EX>(L.r, distance_squared, g).z;
    return (uu * x + vv * y) + w * z;
}

// ------------------------------------------------------------- shading
// Hit record + material (material.scm:15-111).  MATF = the material type a
// queue holds (compile-time; -1 = any, used by the tail kernel).  Returns true
// if the path continues (p holds the scattered ray, new throughput, depth+1);
// otherwise L is the terminal radiance (emission or 0).
// LS = false compiles the light-sampling mixture (f2) out: scenes without a
// light target never take it, and its constants cost scalar registers.
// leaves: the leaf records (LDS in k_shade when the table is small, else HBM)
// trig: rt_libm.h's sin / cos table for the lambertian bounce (an LDS copy in k_shade)
template <int MATF, bool PN = true, bool LS = true, bool EX = true>
__device__ __forceinline__ bool shade_hit(const DevScene& sc, const PerlinLds& P, const RenderParams& rp,
                                          PathRegs& p, const double t, const int32_t leaf, v3& L,
                                          const LeafInfo* __restrict__ leaves,
                                          const double* __restrict__ trig = rtlibm::kSinCosTab) {
    L = mk(0.0, 0.0, 0.0);
    const LeafInfo& li = leaves[leaf];                       // one record: geometry, material, texture (fields read where used)
    v3 o = p.o, d = p.d;
    if (li.chain >= 0) chain_ray(sc.chains[li.chain], o, d);
    v3 pt = o + d * t;                         // point-at-parameter on the (local) ray
    v3 nrm;
    if (li.type == LEAF_SPHERE) {
        nrm = (pt - mk(li.c[0], li.c[1], li.c[2])) * li.inv_r;
    } else if (li.type == LEAF_MSPHERE) {
        v3 cen;
        if (__double_as_longlong(p.time) == 0ll) {          // center(0), computed as below on the host
            cen = mk(li.c[0], li.c[1], li.c[2]);
        } else {
            const MSphereRec S = sc.msph[li.local];
            cen = mk(S.c0x, S.c0y, S.c0z) + mk(S.dcx, S.dcy, S.dcz) * ((p.time - S.t0) / S.den);
        }
        nrm = (pt - cen) * li.inv_r;
    } else if (li.type == LEAF_RECT_XY) {
        nrm = mk(0.0, 0.0, 1.0);
    } else if (li.type == LEAF_RECT_XZ) {
        nrm = mk(0.0, 1.0, 0.0);
    } else if (li.type == LEAF_RECT_YZ || li.type == LEAF_MEDIUM) {
        nrm = mk(1.0, 0.0, 0.0);                             // medium: (v:vec3 1 0 0), geometry.scm:569
    } else if (li.type == LEAF_KLEIN) {
        const KleinRec K = sc.klein[li.local];
        nrm = klein_normal(mk(K.cx, K.cy, K.cz), pt);        // at ray-pos = point-at-parameter, :664
    } else {
        nrm = d * -1.0;                                      // curve: (v:scale (dir r) -1), bezier.scm:204
    }
    if (li.flip) nrm = nrm * -1.0;                          // flip-normals :438
    if (li.chain >= 0) chain_hit(sc.chains[li.chain], pt, nrm);
    const int mt = (MATF >= 0) ? MATF : li.mtype;
    const v3 rdir = p.d;
    const bool can_continue = p.depth < (uint32_t)kMaxDepth;
    if (mt == MAT_DIFFUSE_LIGHT) {                           // material.scm:103-111
        if (dot(nrm, rdir) < 0.0) L = leaf_tex<PN>(sc, P, li, pt);
        return false;
    }
    if (!can_continue) return false;                         // depth cap (main.scm:112,119)
    Rng g;
    g.init(rp.k0, rp.k1, p.pix, p.smp, p.rng);
    if (LS && mt == MAT_LAMBERTIAN && sc.light.type != LIGHT_OFF) {
        // pdf.scm mixture of (hitable-pdf light p) and (cosine-pdf normal)
        // (extension f2; oracle: rt_oracle.c light_pdf_value / light_random)
        const v3 axis2 = unit(nrm);
        const v3 a = (fabs(axis2.x) > 0.9) ? mk(0.0, 1.0, 0.0) : mk(1.0, 0.0, 0.0);
        const v3 axis1 = unit(cross(axis2, a));
        const v3 axis0 = cross(axis2, axis1);
        const DevLight& Lt = sc.light;
        v3 dir;
        if (g.next() < 0.5) {
            dir = light_random<EX>(Lt, pt, g);
        } else {
            const double r1 = g.next(), r2 = g.next();
            const double r3 = g.next(), r4 = g.next();
            (void)g.next();
            const double r6 = g.next();
            double c1, s3;
            bounce_cos_sin<EX>(2.0 * kPi * r1, 2.0 * kPi * r3, c1, s3, trig);
            const double x = c1 * 2.0 * sqrt(r2);
            const double y = s3 * 2.0 * sqrt(r4);
            const double z = sqrt(1.0 - r6);
            dir = (axis0 * x + axis1 * y) + axis2 * z;
        }
        double cz = dot(unit(dir), axis2);
        const double cos_val = (cz > 0.0) ? div_ia(cz, kPi, kInvPi) : 0.0;
        const double pdf_val = 0.5 * light_pdf_value(Lt, pt, dir) + 0.5 * cos_val;
        if (!(pdf_val > 0.0)) return false;                 // no 0 * inf: the path ends (L = 0)
        double cosine = dot(nrm, unit(dir));
        if (cosine < 0.0) cosine = 0.0;
        const double spdf = div_ia(cosine, kPi, kInvPi);
        const double ipdf = 1.0 / pdf_val;
        const v3 att = leaf_tex<PN>(sc, P, li, pt);
        p.T = mk((p.T.x * (att.x * spdf)) * ipdf, (p.T.y * (att.y * spdf)) * ipdf,
                 (p.T.z * (att.z * spdf)) * ipdf);
        p.d = dir;
    } else if (mt == MAT_LAMBERTIAN) {                       // material.scm:24-39
        // onb.scm:8-16
        const v3 axis2 = unit(nrm);
        const v3 a = (fabs(axis2.x) > 0.9) ? mk(0.0, 1.0, 0.0) : mk(1.0, 0.0, 0.0);
        const v3 axis1 = unit(cross(axis2, a));
        const v3 axis0 = cross(axis2, axis1);
        // (local uvw (random-cosine-direction)): `local` is a syntax-rules
        // macro (onb.scm:27-36), so random-cosine-direction (util.scm:37-44,
        // x2 quirk on x and y) runs three times, left to right, and call k
        // supplies component k only (Q29): 6 draws, the 5th unused.
        const double r1 = g.next(), r2 = g.next();
        const double r3 = g.next(), r4 = g.next();
        (void)g.next();
        const double r6 = g.next();
        double c1, s3;
        bounce_cos_sin<EX>(2.0 * kPi * r1, 2.0 * kPi * r3, c1, s3, trig);
        const double x = c1 * 2.0 * sqrt(r2);
        const double y = s3 * 2.0 * sqrt(r4);
        const double z = sqrt(1.0 - r6);
        const v3 target = (axis0 * x + axis1 * y) + axis2 * z;   // onb `local`
        const v3 sd = unit(target);
        const double pdf = div_ia(dot(axis2, sd), kPi, kInvPi);
        double cosine = dot(nrm, unit(sd));
        if (cosine < 0.0) cosine = 0.0;
        const double spdf = div_ia(cosine, kPi, kInvPi);     // scattering-pdf
        const double ipdf = 1.0 / pdf;
        const v3 att = leaf_tex<PN>(sc, P, li, pt);
        // forward form of  e + ((att*spdf) (*) L_next) * (1/pdf)  (main.scm:113-118)
        p.T = mk((p.T.x * (att.x * spdf)) * ipdf, (p.T.y * (att.y * spdf)) * ipdf,
                 (p.T.z * (att.z * spdf)) * ipdf);
        p.d = sd;
    } else if (mt == MAT_METAL) {                            // material.scm:45-57 (R2)
        const v3 reflected = reflect(unit(rdir), nrm);
        v3 s;
        for (int it = 0;; ++it) {                            // util.scm:9-15
            const double a = g.next(), b = g.next(), c = g.next();
            s = mk(a * 2.0 - 1.0, b * 2.0 - 1.0, c * 2.0 - 1.0);
            if (dot(s, s) < 1.0) break;
            if (it >= g_reject_cap) { raise_fault(RT_FAULT_REJECT); s = mk(0.0, 0.0, 0.0); break; }
        }
        const v3 sd = reflected + s * li.mparam;
        if (!(dot(sd, nrm) > 0.0)) return false;             // absorbed: emitted 0
        const v3 att = leaf_tex<PN>(sc, P, li, pt);
        p.T = p.T * att;
        p.d = sd;
    } else {                                                 // dielectric material.scm:76-101 (R2)
        const double ref_idx = li.mparam;
        const v3 reflected = reflect(rdir, nrm);
        const double dd = dot(rdir, nrm);
        const v3 outward = (dd > 0.0) ? nrm * -1.0 : nrm;
        const double ni = (dd > 0.0) ? ref_idx : 1.0 / ref_idx;
        const double cosine = (dd > 0.0) ? (dd * ref_idx) / length(rdir) : (-dd) / length(rdir);
        // refract :59-67 (raw v in the tangential term, Q5)
        const v3 uv = unit(rdir);
        const double dt = dot(uv, outward);
        const double disc = 1.0 - ni * ni * (1.0 - dt * dt);
        double prob = 1.0;
        v3 refracted = mk(0, 0, 0);
        if (disc > 0.0) {
            refracted = (rdir - outward * dt) * ni - outward * sqrt(disc);
            const double r0a = (1.0 - ref_idx) / (1.0 + ref_idx);   // schlick :69-74
            const double r0 = r0a * r0a;
            prob = r0 + (1.0 - r0) * pow5(1.0 - cosine);
        }
        p.d = (g.next() < prob) ? reflected : refracted;   // attenuation (1,1,1)
    }
    p.o = pt;
    p.time = 0.0;                                            // make-ray: time 0 (Q4)
    p.rng = g.ctr;
    p.depth += 1u;
    return true;
}

// the fused curve extend's shading (k_extend_curves<FUSE>): any material, no Perlin tables (PN false: the
// table reference is never read), no light mixture
template <bool EX>
__device__ __forceinline__ bool fused_shade(const DevScene& sc, const RenderParams& rp, PathRegs& p, const double t,
                                            const int32_t leaf, v3& L) {
    return shade_hit<-1, false, false, EX>(sc, *reinterpret_cast<const PerlinLds*>(sc.leaves), rp, p, t, leaf, L, sc.leaves);
}

template <bool PN = true>
__device__ __forceinline__ void stage_perlin(const DevScene& sc, PerlinLds& P) {
    if (PN && sc.has_perlin) {   // the Perlin tables (perlin.scm:32-36 data) into LDS
        for (int k = threadIdx.x; k < 768; k += blockDim.x) { P.ranvec[k] = sc.ranvec[k]; P.perm[k] = sc.perm[k]; }
        __syncthreads();
    }
}

// =====================================================================
// k_shade<MAT> — one material's hit queue; survivors compacted into `out`.
// (One kernel for all materials, sorting each block's hits by material in
// LDS so the ray / path reads stay within one slot range, was measured and
// not kept: its occupancy is the lambertian code's, and the memory-bound
// metal / dielectric hits lost more than the shared lines saved — DESIGN §4.)
// =====================================================================
#ifndef RT_SHADE_WAVES
#define RT_SHADE_WAVES 1               // lambertian / light: the compiler's choice (127 VGPRs, 4 waves)
#endif
#ifndef RT_SHADE_WAVES_MD
#define RT_SHADE_WAVES_MD 1            // metal / dielectric (memory-bound gathers)
#endif
// the exact libm's lambertian kernels without Perlin tables or the light mixture (EX) at 4 waves: with the
// bounce angles' in-range sin / cos (rt_cos_sin) they need 137 VGPRs left alone and fit 128 with no spill
template <int MAT, bool PN, bool LS, bool EX>
constexpr int shade_waves() {
    return (MAT == MAT_METAL || MAT == MAT_DIELECTRIC) ? RT_SHADE_WAVES_MD
         : (MAT == MAT_LAMBERTIAN && EX && !PN && !LS) ? 4 : RT_SHADE_WAVES;
}
template <int MAT, bool PN, bool LS, bool LL, bool EX>
__global__ __launch_bounds__(256, (shade_waves<MAT, PN, LS, EX>())) void k_shade(const DevScene* __restrict__ scp, const RenderParams rp,
                                                                const PathState in, const HitRec* __restrict__ hq,
                                                                const QView qv, PathState out,
                                                                uint32_t* __restrict__ out_counts, uint32_t shard_cap,
                                                                const uint32_t depth) {
    const DevScene& sc = *scp;                       // scene in device memory: fields load on demand
    __shared__ uint32_t s_cnt[16 + 1];
    // the lambertian bounce's sin / cos table (rt_libm.h) in LDS: its lookups are gathers
    constexpr bool kTrig = MAT == MAT_LAMBERTIAN && EX;
    __shared__ double s_trig[kTrig ? 4 * 112 : 2];
    if (kTrig)
        for (int k = threadIdx.x; k < 4 * 112; k += 256) s_trig[k] = rtlibm::kSinCosTab[k];
    // dynamic LDS: the leaf records (LL), then the Perlin tables (PN) — only
    // what the scene uses, so the block's LDS does not cap the occupancy
    extern __shared__ uint4 s_leafdyn[];
    LeafInfo* s_leaves = reinterpret_cast<LeafInfo*>(s_leafdyn);
    PerlinLds& P = *reinterpret_cast<PerlinLds*>(s_leafdyn + (LL ? (size_t)sc.n_leaves * sizeof(LeafInfo) / 16 : 0));
    if (LL) stage_lds(s_leaves, sc.leaves, sc.n_leaves, 256);
    stage_perlin<PN>(sc, P);                         // (its barrier also covers the leaf and table staging)
    if ((LL || kTrig) && !(PN && sc.has_perlin)) __syncthreads();
    const LeafInfo* leaves = LL ? s_leaves : sc.leaves;
    const QMap qm = qmap(qv);
    uint32_t n = 0;
#pragma unroll
    for (int x = 0; x < kShards; ++x) n += min(qv.counts[x * kCntStride], qv.cap);   // written entries only
    const uint32_t gstride = gridDim.x * 256u;
    for (uint32_t base = blockIdx.x * 256u; base < n; base += gstride) {
        const uint32_t k = base + threadIdx.x;
        bool alive = false;
        PathRegs p;
        if (k < n) {
            const HitRec H = hq[qphys(qm, k)];
            load_path(in, H.slot, p, rp, depth);
            v3 L;
            alive = shade_hit<MAT, PN, LS, EX>(sc, P, rp, p, H.t, H.leaf, L, leaves, kTrig ? s_trig : rtlibm::kSinCosTab);
            if (!alive) write_sample(rp, p, L);
        }
        const uint32_t slot = block_append<1>(alive ? 0 : -1, out_counts, shard_cap, s_cnt);
        if (alive && slot != kNoSlot) store_path(out, slot, p);
    }
}

// =====================================================================
// k_finish — the long tail (a few dielectric / metal paths bouncing up to
// depth 100): one thread per remaining path runs extend + shade in a loop
// instead of ~100 more wavefront launches with a host sync each.
// =====================================================================
#ifndef RT_FINISH_WAVES
#define RT_FINISH_WAVES 4             // plain-sphere tails without Perlin / light mixture: 128 VGPRs, 4 waves per SIMD
#endif                                // (the compiler's choice is 143: 3 waves; the other variants would spill at 128)
template <int F, bool PN, bool LSM>
constexpr int finish_waves() { return (F == 0 && !PN && !LSM) ? RT_FINISH_WAVES : 1; }
template <int F, bool PN, bool LSM, bool SOLO = false, bool EX = false>
__global__ __launch_bounds__(256, (finish_waves<F, PN, LSM>())) void k_finish(const DevScene* __restrict__ scp, const RenderParams rp, const PathState st,
                                                const QView in, uint32_t n,
                                                unsigned long long* __restrict__ tail_ctl, int tree0_lds,
                                                const uint32_t depth) {
    const DevScene& sc = *scp;                       // scene in device memory: fields load on demand
    // dynamic LDS: per-lane BVH stack (256 x sc.lane_stack; 16-bit entries
    // for SOLO), then, if tree0_lds, the time-0 tree (nodes, leaves, sphere
    // records) as in k_extend_lds, then, for scenes with Perlin tables, the
    // tables.  SOLO (the world is one sphere BVH, DevScene::bvh_solo, with the
    // tree in LDS): the closest hit is k_extend_lds's — direct leaves, no leaf
    // records, 16-bit stack — so the tail carries no group loop.
    extern __shared__ uint4 s_fdyn[];
    uint32_t* s_lstack = reinterpret_cast<uint32_t*>(s_fdyn);
    uint16_t* s_lstack16 = reinterpret_cast<uint16_t*>(s_fdyn);
    const int LS = sc.lane_stack;
    constexpr bool BEZ = (F & kFeatCurves) != 0;
    constexpr bool MED = (F & kFeatExtra) != 0;
    static_assert(!SOLO || F == 0, "SOLO tails are plain-sphere scenes");
    __shared__ BezWave s_bw[BEZ ? 4 : 1];
    const int words = SOLO ? (256 * (LS > 0 ? LS : 1) * 2 + 15) / 16            // stack size in uint4
                           : (256 * (LS > 0 ? LS : 1) + 3) / 4;
    const int tl_leaves = SOLO ? 0 : sc.n_fbleaf;
    const size_t tree_words = tree0_lds ? ((size_t)sc.n_fbvh2 * sizeof(BvhNode2) + (size_t)tl_leaves * sizeof(BvhLeaf) +
                                           (size_t)sc.n_fsph * sizeof(SphereRec)) / 16 : 0;
    PerlinLds& P = *reinterpret_cast<PerlinLds*>(s_fdyn + words + tree_words);
    Tree0 t0 = tree0_hbm(sc);
    if (tree0_lds) {
        const int nn = sc.n_fbvh2, nl = tl_leaves, ns = sc.n_fsph;
        BvhNode2* s_nodes = reinterpret_cast<BvhNode2*>(s_fdyn + words);
        BvhLeaf* s_leaves = reinterpret_cast<BvhLeaf*>(s_nodes + nn);
        SphereRec* s_sph = reinterpret_cast<SphereRec*>(s_leaves + nl);
        stage_lds(s_nodes, sc.fbvh2, nn, 256);
        if (!SOLO) stage_lds(s_leaves, sc.fbleaf, nl, 256);
        stage_lds(s_sph, sc.fsph, ns, 256);
        t0 = Tree0{s_nodes, s_leaves, s_sph, sc.fid};
        __syncthreads();
    }
    stage_perlin<PN>(sc, P);
    // Persistent lanes: a lane whose path ended takes the next unstarted one
    // (one atomic per wave per refill), so a wave is not held by its longest
    // path while its other lanes idle.  tail_ctl[0] counts segments,
    // tail_ctl[1] is the next path index.
    unsigned int* next = reinterpret_cast<unsigned int*>(tail_ctl + 1);
    const QMap qm = qmap(in);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t segs = 0, pseg = 0;                    // pseg: segments of the lane's current path
    bool active = false, exhausted = false;
    PathRegs p;
    for (;;) {
        const unsigned long long need = __ballot(!active);
        if (need && !exhausted) {
            uint32_t base = 0;
            const uint32_t cnt = (uint32_t)__popcll(need);
            const uint32_t leader = (uint32_t)__ffsll((long long)need) - 1u;
            if (lane == leader) base = atomicAdd(next, cnt);
            base = __shfl(base, (int)leader, 64);
            if (base + cnt >= n) exhausted = true;
            if (!active) {
                const uint32_t k = base + lanes_below(need);
                if (k < n) { load_path(st, qphys(qm, k), p, rp, depth); active = true; pseg = 0; }
            }
        }
        if (__ballot(active) == 0ull) break;
        if (active && ++pseg > (uint32_t)kMaxDepth + 2u) {   // depth is capped at kMaxDepth (main.scm:26)
            raise_fault(RT_FAULT_PATH);
            active = false;
        }
        if (active) {
            double t;
            ++segs;
            Rng g;
            if (MED) g.init(rp.k0, rp.k1, p.pix, p.smp, p.rng);
            int32_t leaf;
            if constexpr (SOLO)
                leaf = closest_hit_lds<true>(sc, p.o, p.d, p.time, t, s_lstack16 + threadIdx.x, LS, t0, treeA_hbm(sc));
            else
                leaf = closest_hit<F>(sc, p.o, p.d, p.time, t, s_lstack + threadIdx.x, LS,
                                      &s_bw[BEZ ? (threadIdx.x >> 6) : 0], &g, t0, treeA_hbm(sc));
            if (MED) p.rng = g.ctr;
            v3 L;
            bool cont = false;
            if (leaf < 0) L = sky_radiance(sc, p.d);
            else cont = shade_hit<-1, PN, LSM, EX>(sc, P, rp, p, t, leaf, L, sc.leaves);
            if (!cont) { write_sample(rp, p, L); active = false; }
        }
    }
    // segment statistics: wave sum, one atomic per wave
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off, 64);
    if (lane == 0u && segs) atomicAdd(tail_ctl, (unsigned long long)segs);
}

// =====================================================================
// k_accumulate — *raw-data* running sum, samples added in order
// =====================================================================
__global__ __launch_bounds__(256) void k_accumulate(const RenderParams rp, uint32_t S,
                                                    double* __restrict__ accum) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= rp.npix) return;
    const uint32_t j = rp.compact ? q : rp.pixlist[q];
    double a0 = accum[3u * j], a1 = accum[3u * j + 1], a2 = accum[3u * j + 2];
    for (uint32_t s = 0; s < S; ++s) {                   // sample order per channel, as before
        const double* r = rp.sb + 3u * ((size_t)s * rp.npix + q);
        a0 = a0 + r[0]; a1 = a1 + r[1]; a2 = a2 + r[2];
    }
    accum[3u * j] = a0; accum[3u * j + 1] = a1; accum[3u * j + 2] = a2;
}

// main.scm:481-491 — sqrt(sum/count), floor(255.99*min(1,c))
__global__ __launch_bounds__(256) void k_resolve_u8(const double* __restrict__ accum, uint32_t n,
                                                    double count, uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const double c = sqrt(accum[i] / count);
    const double m = (1.0 < c) ? 1.0 : c;
    out[i] = (uint8_t)floor(255.99 * m);
}

// ------------------------------------------------------------ launchers
#define HIP_RETURN_IF(x) do { const hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)
hipError_t launch_raygen(const DevScene& sc, const RenderParams& rp, const PathState& st,
                         hipStream_t s) {
    const uint32_t blocks = (rp.B + 255u) / 256u;
    hipLaunchKernelGGL(k_raygen, dim3(blocks), dim3(256), 0, s, sc, rp, st);
    return hipGetLastError();
}
static uint32_t finish_blocks() { return 512u; }    // persistent tail grid (1024: +2 % single-lane, -1 % with the two render lanes: profiles/r03/ab/ab_tail_grid.log)
static bool finish_generic() {               // RTAMD_FINISH_GENERIC: the group-loop tail for SOLO scenes too (A/B, tests)
    const char* e = std::getenv("RTAMD_FINISH_GENERIC");  // read per launch: tests switch it inside one process
    return e != nullptr && e[0] != '0';
}
static int scene_features(const DevScene& sc) {
    return (sc.n_bez > 0 ? kFeatCurves : 0) | (sc.n_med > 0 || sc.n_klein > 0 ? kFeatExtra : 0);
}
static uint32_t curve_blocks() {            // cap on the persistent curve grid (RTAMD_CURVE_BLOCKS; 0 = per-ray k_extend)
    const char* e = std::getenv("RTAMD_CURVE_BLOCKS");  // read per launch: tests switch it inside one process
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 1u << 20;
}
bool curve_persistent() { return curve_blocks() > 0u; }   // the host's check before a fused launch
// resident blocks of a curve kernel instance for its dynamic LDS, cached per (kernel, device, LDS bytes)
static hipError_t curve_occupancy(const void* f, const size_t lds, uint32_t* out) {
    static const void* occ_f[3] = {nullptr, nullptr, nullptr};
    static int occ_dev[3] = {-1, -1, -1};
    static size_t occ_lds[3] = {~(size_t)0, ~(size_t)0, ~(size_t)0};
    static uint32_t occ_blocks[3] = {0, 0, 0};
    int dev = 0;
    HIP_RETURN_IF(hipGetDevice(&dev));
    const int slot = f == reinterpret_cast<const void*>(&k_extend_curves<1>) ? 1
                   : f == reinterpret_cast<const void*>(&k_extend_curves<2>) ? 2 : 0;
    if (occ_f[slot] != f || occ_lds[slot] != lds || occ_dev[slot] != dev) {
        int per_cu = 0, cus = 0;
        HIP_RETURN_IF(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 256, lds));
        HIP_RETURN_IF(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        occ_blocks[slot] = (uint32_t)(per_cu > 0 ? per_cu : 1) * (uint32_t)(cus > 0 ? cus : 1);
        occ_lds[slot] = lds;
        occ_dev[slot] = dev;
        occ_f[slot] = f;
    }
    *out = occ_blocks[slot];
    return hipSuccess;
}
hipError_t launch_extend(const DevScene& sc, const DevScene*, const RenderParams& rp, const PathState& st, const QView& in,
                         uint32_t n, const HitBuf& hit, uint32_t shard_cap,
                         uint32_t* counts, bool depth0, unsigned int* claim, const CurveFuse* fuse, hipStream_t s) {
    const uint32_t blocks = (n + 255u) / 256u;
    const size_t lds = (size_t)256 * (size_t)(sc.lane_stack > 0 ? sc.lane_stack : 1) * sizeof(uint32_t);
    // the persistent curve kernel: every curve in the world BVH (its groups outside the BVH are spheres and
    // rects only: group_closest<0>, so the per-lane curve walk is not compiled into it)
    if (scene_features(sc) == kFeatCurves && sc.bvh_has_bez && sc.bez_groups == 0 && claim && curve_blocks() > 0) {
        // resident blocks only: later blocks would find the rays claimed.  The BVH4 walk's LDS stack column
        // holds lds4 entries per lane (the rest in the overflow area).  Occupancy per (device, LDS bytes)
        const size_t clds = (size_t)256 * (size_t)(sc.lds4 > 0 ? sc.lds4 : 1) * sizeof(uint32_t);
        uint32_t occ_blocks = 0;
        const void* kf = !fuse ? reinterpret_cast<const void*>(&k_extend_curves<0>)
                       : rp.exact_libm ? reinterpret_cast<const void*>(&k_extend_curves<2>)
                                       : reinterpret_cast<const void*>(&k_extend_curves<1>);
        HIP_RETURN_IF(curve_occupancy(kf, clds, &occ_blocks));
        uint32_t pb = blocks < occ_blocks ? blocks : occ_blocks;
        if (pb > curve_blocks()) pb = curve_blocks();
        // the overflow area holds sc.ovf_lanes lanes per render lane: never launch more (ovf_lane indexes it)
        if (sc.stk_ovf && pb > sc.ovf_lanes / 256u) pb = sc.ovf_lanes / 256u;
        if (pb > sc.ring_waves / 4u) pb = sc.ring_waves / 4u;   // one survivor ring per wave
        if (pb == 0u) pb = 1u;
        HIP_RETURN_IF(hipMemsetAsync(claim, 0, sizeof(unsigned int), s));
        if (!fuse) {
            hipLaunchKernelGGL((k_extend_curves<0>), dim3(pb), dim3(256), clds, s, sc, rp, st, in, n, hit,
                               shard_cap, counts, depth0, claim, CurveFuse{});
        } else if (rp.exact_libm) {
            hipLaunchKernelGGL((k_extend_curves<2>), dim3(pb), dim3(256), clds, s, sc, rp, st, in, n, hit,
                               shard_cap, counts, false, claim, *fuse);
        } else {
            hipLaunchKernelGGL((k_extend_curves<1>), dim3(pb), dim3(256), clds, s, sc, rp, st, in, n, hit,
                               shard_cap, counts, false, claim, *fuse);
        }
        return hipGetLastError();
    }
    if (fuse) return hipErrorNotSupported;           // only the persistent curve kernel shades its own hits
#define RT_EXTEND_F(F)                                                                                      \
    hipLaunchKernelGGL((k_extend<F>), dim3(blocks), dim3(256), lds, s, sc, rp, st, in, n, hit,             \
                       shard_cap, counts, depth0)
    switch (scene_features(sc)) {
    case 0: RT_EXTEND_F(0); break;
    case 1: RT_EXTEND_F(1); break;
    case 2: RT_EXTEND_F(2); break;
    default: RT_EXTEND_F(3); break;
    }
#undef RT_EXTEND_F
    return hipGetLastError();
}
hipError_t launch_hit_rays(const DevScene& sc, const double* rays, uint32_t n, double* out_t, int32_t* out_mat,
                           hipStream_t s) {
    const uint32_t blocks = (n + 255u) / 256u;
    const size_t lds = (size_t)256 * (size_t)(sc.lane_stack > 0 ? sc.lane_stack : 1) * sizeof(uint32_t);
    if (!blocks) return hipSuccess;
    switch (scene_features(sc)) {
    case 0: hipLaunchKernelGGL((k_hit_rays<0>), dim3(blocks), dim3(256), lds, s, sc, rays, n, out_t, out_mat); break;
    default:
        hipLaunchKernelGGL((k_hit_rays<kFeatCurves | kFeatExtra>), dim3(blocks), dim3(256), lds, s, sc, rays, n, out_t,
                           out_mat);
        break;
    }
    return hipGetLastError();
}
// bytes of LDS k_extend_lds needs for the scene's time-0 tree (0 = cannot run)
size_t extend_lds_bytes(const DevScene& sc) {
    if (!sc.fbvh2 || sc.n_bez || sc.n_med || sc.n_klein) return 0;
    if (sc.n_fbvh2 >= 32768 || sc.n_fbleaf >= 32768) return 0;        // 16-bit stack entries
    return extend_lds_need(sc);
}
// the kernel instance a scene's LDS launches use (SOLO: the world is one BVH group)
static const void* extend_lds_fn(const DevScene& sc) {
    return sc.bvh_solo ? reinterpret_cast<const void*>(&k_extend_lds<true>)
                       : reinterpret_cast<const void*>(&k_extend_lds<false>);
}
static const void* camera_fn(const DevScene& sc) {
    if (sc.tree0_any_time)
        return sc.bvh_solo ? reinterpret_cast<const void*>(&k_camera<false, true>)
                           : reinterpret_cast<const void*>(&k_camera<false, false>);
    return sc.bvh_solo ? reinterpret_cast<const void*>(&k_camera<true, true>)
                       : reinterpret_cast<const void*>(&k_camera<true, false>);
}
hipError_t launch_extend_lds(const DevScene& sc, const RenderParams& rp, const PathState& st, const QView& in,
                             uint32_t n, const HitBuf& hit,
                             uint32_t shard_cap, uint32_t* counts, uint32_t max_blocks, unsigned long long* err,
                             hipStream_t s) {
    const size_t lds = extend_lds_bytes(sc);
    uint32_t blocks = (n + kExtLdsBlock - 1) / kExtLdsBlock;
    if (blocks > max_blocks) blocks = max_blocks;
    blocks = (blocks + kShards - 1) / kShards * kShards;      // every shard gets the same number of blocks
    if (sc.bvh_solo)
        hipLaunchKernelGGL(k_extend_lds<true>, dim3(blocks), dim3(kExtLdsBlock), lds, s, sc, rp, st, in, n, hit,
                           shard_cap, counts, (uint32_t)lds, err);
    else
        hipLaunchKernelGGL(k_extend_lds<false>, dim3(blocks), dim3(kExtLdsBlock), lds, s, sc, rp, st, in, n, hit,
                           shard_cap, counts, (uint32_t)lds, err);
    return hipGetLastError();
}
// resident blocks of a persistent LDS kernel: every block it can keep on the device at once
static hipError_t resident_blocks(const void* f, size_t lds, uint32_t* max_blocks) {
    HIP_RETURN_IF(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int dev = 0, cus = 0, per_cu = 0;
    HIP_RETURN_IF(hipGetDevice(&dev));
    HIP_RETURN_IF(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_RETURN_IF(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, kExtLdsBlock, lds));
    *max_blocks = (uint32_t)(cus * (per_cu > 0 ? per_cu : 0));
    return hipSuccess;
}
hipError_t extend_lds_prepare(const DevScene& sc, size_t lds, uint32_t* max_blocks) {
    return resident_blocks(extend_lds_fn(sc), lds, max_blocks);
}
// LDS bytes k_camera needs (0 = cannot run): the all-times tree when the scene
// has moving spheres, else the time-0 tree
size_t camera_lds_bytes(const DevScene& sc) {
    if (!sc.fbvh2 || sc.n_bez || sc.n_med || sc.n_klein) return 0;
    if (sc.tree0_any_time) return extend_lds_bytes(sc);
    if (sc.n_bvh2 >= 32768 || sc.n_bleaf >= 32768) return 0;          // 16-bit stack entries
    return camera_lds_need(sc);
}
hipError_t camera_prepare(const DevScene& sc, size_t lds, uint32_t* max_blocks) {
    return resident_blocks(camera_fn(sc), lds, max_blocks);
}
hipError_t launch_camera(const DevScene& sc, const RenderParams& rp, const PathState& st, uint32_t n,
                         const HitBuf& hit, uint32_t shard_cap, uint32_t* counts,
                         size_t lds, uint32_t max_blocks, unsigned long long* err, hipStream_t s) {
    uint32_t blocks = (n + kExtLdsBlock - 1) / kExtLdsBlock;
    if (blocks > max_blocks) blocks = max_blocks;
    blocks = (blocks + kShards - 1) / kShards * kShards;
#define RT_CAMERA(A, S)                                                                                       \
    hipLaunchKernelGGL((k_camera<A, S>), dim3(blocks), dim3(kExtLdsBlock), lds, s, sc, rp, st, n, hit,          \
                       shard_cap, counts, (uint32_t)lds, err)
    if (sc.tree0_any_time) { if (sc.bvh_solo) RT_CAMERA(false, true); else RT_CAMERA(false, false); }
    else { if (sc.bvh_solo) RT_CAMERA(true, true); else RT_CAMERA(true, false); }
#undef RT_CAMERA
    return hipGetLastError();
}
constexpr size_t kShadeLeafLds = 32768;      // stage the leaf records when they fit (256 leaves)
hipError_t launch_shade(int mat, const DevScene& sc, const DevScene* scd, const RenderParams& rp, const PathState& in,
                        const HitBuf& hit, const QView& qv, uint32_t n_upper,
                        const PathState& out, uint32_t* out_counts, uint32_t shard_cap, uint32_t depth, hipStream_t s) {
    // grid-stride cap: each block stages the leaf records once, so fewer,
    // longer-lived blocks (2048 was best of 1024..8192 with 96M-path pools;
    // 1024 with the 288M-path pools: +1.5 % C2, 512 -14 %: profiles/r02/shadeb/)
    // (rt_api's shard slack assumes <= 4096, a multiple of 8).  2048 / 4096 blocks for the sparse metal /
    // dielectric queues measured the same as 1024 (profiles/r03/ab/ab_sparse_grid.log)
    constexpr uint32_t max_blocks = 1024;
    uint32_t blocks = (n_upper + 255u) / 256u;
    blocks = (blocks + kShards - 1) / kShards * kShards;     // every shard gets the same number of blocks
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks == 0u) blocks = kShards;
    const HitRec* hq = hit.h + (size_t)mat * hit.stride;
#define RT_SHADE_EX(M, PN, LS, EX)                                                                           \
    do {                                                                                                     \
        if (ll)                                                                                              \
            hipLaunchKernelGGL((k_shade<M, PN, LS, true, EX>), dim3(blocks), dim3(256), lds, s, scd, rp, in,   \
                               hq, qv, out, out_counts, shard_cap, depth);                                   \
        else                                                                                                 \
            hipLaunchKernelGGL((k_shade<M, PN, LS, false, EX>), dim3(blocks), dim3(256), lds, s, scd, rp, in,  \
                               hq, qv, out, out_counts, shard_cap, depth);                                   \
    } while (0)
    // libm's own sin / cos for the bounce directions (bounce_cos_sin: RT_OPT_EXACT_LIBM, by default in
    // scenes with curves); only the lambertian kernels draw directions with them
#define RT_SHADE(M, PN, LS)                                                                                  \
    do {                                                                                                     \
        if (M == MAT_LAMBERTIAN && rp.exact_libm) RT_SHADE_EX(M, PN, LS, true);                             \
        else RT_SHADE_EX(M, PN, LS, false);                                                                  \
    } while (0)
    const bool pn = sc.has_noise_tex != 0;
    const bool ls = sc.light.type != LIGHT_OFF;       // only lambertian scatter uses the light mixture
    const size_t leaf_lds = (size_t)sc.n_leaves * sizeof(LeafInfo);
    const bool ll = leaf_lds <= kShadeLeafLds;
    // PN kernels of every material carry the Perlin tables (metal albedo may be a noise texture)
    const size_t lds = (ll ? leaf_lds : 0) + ((pn && mat != MAT_DIELECTRIC && sc.has_perlin) ? sizeof(PerlinLds) : 0);
    switch (mat) {
    case MAT_LAMBERTIAN:
        if (ls) { if (pn) RT_SHADE(MAT_LAMBERTIAN, true, true); else RT_SHADE(MAT_LAMBERTIAN, false, true); }
        else { if (pn) RT_SHADE(MAT_LAMBERTIAN, true, false); else RT_SHADE(MAT_LAMBERTIAN, false, false); }
        break;
    case MAT_METAL: if (pn) RT_SHADE(MAT_METAL, true, false); else RT_SHADE(MAT_METAL, false, false); break;
    case MAT_DIELECTRIC: RT_SHADE(MAT_DIELECTRIC, false, false); break;          // attenuation is constant 1
    default: if (pn) RT_SHADE(MAT_DIFFUSE_LIGHT, true, false); else RT_SHADE(MAT_DIFFUSE_LIGHT, false, false); break;
    }
#undef RT_SHADE
#undef RT_SHADE_EX
    return hipGetLastError();
}
hipError_t launch_finish(const DevScene& sc, const DevScene* scd, const RenderParams& rp, const PathState& st, const QView& in,
                         uint32_t n, unsigned long long* seg_count, size_t tree0_budget, uint32_t depth,
                         hipStream_t s) {
    uint32_t blocks = (n + 255u) / 256u;
    if (blocks > finish_blocks()) blocks = finish_blocks();   // persistent lanes refill from the path list
    const size_t tree = (size_t)sc.n_fbvh2 * sizeof(BvhNode2) + (size_t)sc.n_fbleaf * sizeof(BvhLeaf) +
                        (size_t)sc.n_fsph * sizeof(SphereRec);
    const int tree0_lds = (sc.fbvh2 && tree0_budget > 0 && tree <= tree0_budget) ? 1 : 0;
    // SOLO tail: plain-sphere world in one BVH, its time-0 tree in LDS, child refs within int16
    const bool solo = tree0_lds && sc.bvh_solo && scene_features(sc) == 0 && extend_lds_bytes(sc) > 0 &&
                      sc.n_bvh2 < 32768 && sc.n_bleaf < 32768 && !finish_generic();
    const size_t stack_entry = solo ? sizeof(uint16_t) : sizeof(uint32_t);
    size_t lds = ((size_t)256 * (size_t)(sc.lane_stack > 0 ? sc.lane_stack : 1) * stack_entry + 15) / 16 * 16;
    if (tree0_lds) lds += solo ? tree - (size_t)sc.n_fbleaf * sizeof(BvhLeaf) : tree;
    // the Perlin tables ride at the end of the dynamic LDS, only where they are staged (PN and tables given)
    const size_t perlin = sc.has_perlin ? sizeof(PerlinLds) : 0;
    // the bounce directions' sin / cos (RT_OPT_EXACT_LIBM): rt_libm.h's or the device library's
    const bool ex = rp.exact_libm != 0;
#define RT_FINISH_F(F) RT_FINISH(F, true, true)
#define RT_FINISH_SOLO_EX(PN, LS, EX) \
    hipLaunchKernelGGL((k_finish<0, PN, LS, true, EX>), dim3(blocks), dim3(256), lds + (PN ? perlin : 0), s, scd, rp, st, \
                       in, n, seg_count, tree0_lds, depth)
#define RT_FINISH_EX(F, PN, LS, EX) \
    hipLaunchKernelGGL((k_finish<F, PN, LS, false, EX>), dim3(blocks), dim3(256), lds + (PN ? perlin : 0), s, scd, rp, st, \
                       in, n, seg_count, tree0_lds, depth)
#define RT_FINISH_SOLO(PN, LS) do { if (ex) RT_FINISH_SOLO_EX(PN, LS, true); else RT_FINISH_SOLO_EX(PN, LS, false); } while (0)
#define RT_FINISH(F, PN, LS) do { if (ex) RT_FINISH_EX(F, PN, LS, true); else RT_FINISH_EX(F, PN, LS, false); } while (0)
    // the plain-sphere feature set also gets Perlin / light-mixture specialisations:
    // the tail kernel carries every material's code, so dropping the unused ones
    // trims its register file
    const bool pn = sc.has_noise_tex != 0;
    const bool ls = sc.light.type != LIGHT_OFF;
    switch (scene_features(sc)) {
    case 0:
        if (solo) {
            if (pn) { if (ls) RT_FINISH_SOLO(true, true); else RT_FINISH_SOLO(true, false); }
            else { if (ls) RT_FINISH_SOLO(false, true); else RT_FINISH_SOLO(false, false); }
        } else if (pn) { if (ls) RT_FINISH(0, true, true); else RT_FINISH(0, true, false); }
        else { if (ls) RT_FINISH(0, false, true); else RT_FINISH(0, false, false); }
        break;
    case 1: RT_FINISH_F(1); break;
    case 2: RT_FINISH_F(2); break;
    default: RT_FINISH_F(3); break;
    }
#undef RT_FINISH_F
#undef RT_FINISH_SOLO
#undef RT_FINISH
#undef RT_FINISH_SOLO_EX
#undef RT_FINISH_EX
    return hipGetLastError();
}
// test hooks (render_impl: RTAMD_REJECT_CAP / RTAMD_CURVE_RAY_CAP, tests only): the samplers' attempt
// cap (default kRejectCap) and the persistent curve kernel's per-ray iteration cap (0 = the scene's bound)
hipError_t set_test_caps(int reject_cap, uint32_t curve_ray_cap) {
    static int applied[64];                     // per device; 0 = not written yet (the defaults)
    static uint32_t applied_ray[64];
    int dev = 0;
    HIP_RETURN_IF(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    const int have = applied[dev] ? applied[dev] - 1 : kRejectCap;
    if (reject_cap != have) {
        HIP_RETURN_IF(hipMemcpyToSymbol(HIP_SYMBOL(g_reject_cap), &reject_cap, sizeof reject_cap));
        applied[dev] = reject_cap + 1;
    }
    if (curve_ray_cap != applied_ray[dev]) {
        HIP_RETURN_IF(hipMemcpyToSymbol(HIP_SYMBOL(g_curve_ray_cap), &curve_ray_cap, sizeof curve_ray_cap));
        applied_ray[dev] = curve_ray_cap;
    }
    return hipSuccess;
}
// the device fault word: read and clear (render_impl, after the render's streams are synchronised)
hipError_t take_fault(uint32_t* out) {
    uint32_t f = 0;
    HIP_RETURN_IF(hipMemcpyFromSymbol(&f, HIP_SYMBOL(g_fault), sizeof f));
    if (f) {
        const uint32_t z = 0;
        HIP_RETURN_IF(hipMemcpyToSymbol(HIP_SYMBOL(g_fault), &z, sizeof z));
    }
    *out = f;
    return hipSuccess;
}
// the batched-curve counters: read and clear (render_impl, at the start and end of a render)
hipError_t take_curve_stats(unsigned long long out[2]) {
    HIP_RETURN_IF(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_curve_stats), 2 * sizeof(unsigned long long)));
    if (out[0] || out[1]) {
        const unsigned long long z[2] = {0ull, 0ull};
        HIP_RETURN_IF(hipMemcpyToSymbol(HIP_SYMBOL(g_curve_stats), z, sizeof z));
    }
    return hipSuccess;
}
#ifdef RT_STATS
extern "C" int rt_debug_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stats), sizeof g_stats) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[48] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof z) != hipSuccess) return 1;
    }
    return 0;
}
#endif
hipError_t launch_accumulate(const RenderParams& rp, uint32_t S, double* accum, hipStream_t s) {
    const uint32_t blocks = (rp.npix + 255u) / 256u;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(256), 0, s, rp, S, accum);
    return hipGetLastError();
}
// rt_curve_depth_probe: bez_maxd — the depth estimate every curve kernel runs (stage A, the per-lane
// walk) — on caller-given ray-space control points (12 doubles per curve) and 8 eps
__global__ __launch_bounds__(256) void k_curve_depth(const double* __restrict__ cps, const double* __restrict__ eps8,
                                                     uint32_t n, int32_t* __restrict__ out) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n) return;
    const double* p = cps + 12 * (size_t)k;
    Bez4 c;
    c.p0 = mk(p[0], p[1], p[2]); c.p1 = mk(p[3], p[4], p[5]); c.p2 = mk(p[6], p[7], p[8]); c.p3 = mk(p[9], p[10], p[11]);
    out[k] = bez_maxd(c, eps8[k]);
}
hipError_t launch_curve_depth(const double* cps, const double* eps8, uint32_t n, int32_t* out, hipStream_t s) {
    if (n == 0u) return hipSuccess;
    hipLaunchKernelGGL(k_curve_depth, dim3((n + 255u) / 256u), dim3(256), 0, s, cps, eps8, n, out);
    return hipGetLastError();
}
// the frame-end gather's placement (rt_gather_shards): shard pixel q's three sums to image pixel pix[q]
__global__ __launch_bounds__(256) void k_scatter_pixels(const double* __restrict__ src, const uint32_t* __restrict__ pix,
                                                        uint32_t n, double* __restrict__ frame) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= n) return;
    const size_t j = pix[q];
    frame[3 * j] = src[3 * (size_t)q];
    frame[3 * j + 1] = src[3 * (size_t)q + 1];
    frame[3 * j + 2] = src[3 * (size_t)q + 2];
}
hipError_t launch_scatter_pixels(const double* src, const uint32_t* pix, uint32_t n, double* frame, hipStream_t s) {
    if (n == 0u) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_pixels, dim3((n + 255u) / 256u), dim3(256), 0, s, src, pix, n, frame);
    return hipGetLastError();
}
hipError_t launch_resolve_u8(const double* accum, uint32_t n, int count, uint8_t* out, hipStream_t s) {
    const uint32_t blocks = (n + 255u) / 256u;
    hipLaunchKernelGGL(k_resolve_u8, dim3(blocks), dim3(256), 0, s, accum, n, (double)count, out);
    return hipGetLastError();
}

}  // namespace rtamd
