// rt_kernels.hip — CDNA4 (gfx950) wavefront path-tracing kernels.
//
// The reference's recursive `color` (main.scm:100-121) becomes an iterative
// wavefront over a pool of paths kept SoA in HBM:
//
//   k_raygen    trace-all jitter + cam:get-ray      main.scm:476-478, camera.scm:80-92
//   k_extend    closest hit over the flattened       geometry.scm:14-56,146-215,376-543
//               object tree (one segment per path)
//   k_shade     hit record + material scatter +      material.scm:15-111, texture.scm,
//               sky / emission; survivors compacted  perlin.scm, main.scm:91-121
//               with a wave64 ballot + mbcnt prefix
//               and one atomic per wave
//   k_accumulate per-pixel running sum in sample     main.scm:480,488
//               order (deterministic, no atomics)
//   k_resolve_u8 correct-gamma + quantise            main.scm:481-491
//
// All arithmetic is f64 like the reference's flonums.  Random numbers come
// from a Philox4x32-10 stream keyed by (seed, pixel, sample) with a per-path
// draw counter, consumed in the reference's order.
#include <hip/hip_runtime.h>
#include "rt_device.h"

namespace rtamd {

// ------------------------------------------------------------------ RNG
__device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                         uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
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

// ------------------------------------------------------------ vec.scm
struct v3 { double x, y, z; };
__device__ __forceinline__ v3 mk(double x, double y, double z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 operator*(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 operator*(v3 a, double k) { return mk(a.x * k, a.y * k, a.z * k); }
__device__ __forceinline__ double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double length(v3 a) { return sqrt(dot(a, a)); }
__device__ __forceinline__ v3 unit(v3 a) { const double k = 1.0 / length(a); return a * k; }
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
__global__ __launch_bounds__(256) void k_raygen(const DevScene sc, const RenderParams rp,
                                                PathState st) {
    const uint32_t w = blockIdx.x * 256u + threadIdx.x;
    if (w >= rp.B) return;
    const uint32_t s_rel = w / rp.npix;
    const uint32_t q = w - s_rel * rp.npix;
    const uint32_t j = rp.pixlist[q];
    const uint32_t y = j / rp.nx, x = j - y * rp.nx;
    const uint32_t smp = rp.spp0 + s_rel;
    Rng g;
    g.init(rp.k0, rp.k1, j, smp, 0u);
    // main.scm:476-477 (let* order: u then v)
    const double u = ((double)x + g.next()) / (double)rp.nx;
    const double v = ((double)y + g.next()) / (double)rp.ny;
    // camera.scm:80-92
    const DevCamera& c = sc.cam;
    v3 p;
    for (;;) {   // util.scm:17-23 random-in-unit-disk
        const double a = g.next(), b = g.next();
        p = mk(a * 2.0 - 1.0, b * 2.0 - 1.0, 0.0 * 2.0 - 0.0);
        if (dot(p, p) < 1.0) break;
    }
    const v3 rd = p * c.lens;
    const v3 cu = mk(c.u[0], c.u[1], c.u[2]), cv = mk(c.v[0], c.v[1], c.v[2]);
    const v3 offset = cu * rd.x + cv * rd.y;
    const double time = c.t0 + g.next() * (c.t1 - c.t0);
    const v3 origin = mk(c.origin[0], c.origin[1], c.origin[2]);
    const v3 o = origin + offset;
    const v3 d = ((mk(c.llc[0], c.llc[1], c.llc[2]) + mk(c.hor[0], c.hor[1], c.hor[2]) * u) +
                  mk(c.ver[0], c.ver[1], c.ver[2]) * v) - origin - offset;
    st.ox[w] = o.x; st.oy[w] = o.y; st.oz[w] = o.z;
    st.dx[w] = d.x; st.dy[w] = d.y; st.dz[w] = d.z;
    st.tm[w] = time;
    st.tr[w] = 1.0; st.tg[w] = 1.0; st.tb[w] = 1.0;
    st.pix[w] = j; st.smp[w] = smp; st.wid[w] = w; st.rng[w] = g.ctr; st.depth[w] = 0u;
}

// =====================================================================
// k_extend — closest hit (hit-obj-list semantics: shrinking t-max,
// strict (tmin, closest) for spheres, non-strict for rects)
// =====================================================================
__global__ __launch_bounds__(256) void k_extend(const DevScene sc, const PathState st, uint32_t n,
                                                HitBuf hit) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const v3 o0 = mk(st.ox[i], st.oy[i], st.oz[i]);
    const v3 d0 = mk(st.dx[i], st.dy[i], st.dz[i]);
    const double time = st.tm[i];
    double closest = kTmax;
    int32_t best = -1;
    for (int g = 0; g < sc.n_groups; ++g) {
        const Group G = sc.groups[g];
        v3 o = o0, d = d0;
        if (G.chain >= 0) chain_ray(sc.chains[G.chain], o, d);
        const int32_t base = sc.leaf_base[G.type];
        if (G.type == LEAF_SPHERE) {                       // geometry.scm:146-171
            const double a = dot(d, d);
            for (int s = G.begin; s < G.end; ++s) {
                const SphereRec S = sc.sph[s];
                const v3 oc = o - mk(S.cx, S.cy, S.cz);
                const double b = dot(oc, d);
                const double c = dot(oc, oc) - S.rr;
                const double disc = b * b - a * c;
                if (disc > 0.0) {
                    const double sq = sqrt(disc);
                    double t = (-b - sq) / a;
                    if (!(kTmin < t && t < closest)) t = (-b + sq) / a;
                    if (kTmin < t && t < closest) { closest = t; best = base + s; }
                }
            }
        } else if (G.type == LEAF_MSPHERE) {               // geometry.scm:177-208
            const double a = dot(d, d);
            double last_t0 = 0.0, last_den = 0.0, frac = 0.0;
            bool have = false;
            for (int s = G.begin; s < G.end; ++s) {
                const MSphereRec S = sc.msph[s];
                if (!have || S.t0 != last_t0 || S.den != last_den) {   // uniform branch
                    frac = (time - S.t0) / S.den;
                    last_t0 = S.t0; last_den = S.den; have = true;
                }
                const v3 cen = mk(S.c0x, S.c0y, S.c0z) + mk(S.dcx, S.dcy, S.dcz) * frac;
                const v3 oc = o - cen;
                const double b = dot(oc, d);
                const double c = dot(oc, oc) - S.rr;
                const double disc = b * b - a * c;
                if (disc > 0.0) {
                    const double sq = sqrt(disc);
                    double t = (-b - sq) / a;
                    if (!(kTmin < t && t < closest)) t = (-b + sq) / a;
                    if (kTmin < t && t < closest) { closest = t; best = base + s; }
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
    hit.t[i] = closest;
    hit.leaf[i] = best;
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
__device__ __forceinline__ v3 tex_value(const DevScene& sc, const PerlinLds& P, int id, v3 p) {   // texture.scm
    for (int guard = 0; guard < 64; ++guard) {
        const DevTexture t = sc.texs[id];
        if (t.type == TEX_CONSTANT) return mk(t.r, t.g, t.bl);
        if (t.type == TEX_CHECKER) {                                 // :16-23
            const double sines = sin(10.0 * p.x) * sin(10.0 * p.y) * sin(10.0 * p.z);
            id = (sines < 0.0) ? t.b : t.a;
            continue;
        }
        if (t.type == TEX_NOISE) {                                   // :25-28
            const double nz = perlin_noise(P, p * t.scale);
            return mk(1.0, 1.0, 1.0) * nz;
        }
        // TEX_MARBLE :30-34
        const double m = 0.5 * (1.0 + sin(t.scale * p.z + 10.0 * perlin_turb(P, p)));
        return mk(1.0, 1.0, 1.0) * m;
    }
    return mk(0.0, 0.0, 0.0);
}

__device__ __forceinline__ v3 reflect(v3 v, v3 n) { return v - n * (2.0 * dot(v, n)); }  // material.scm:41-43

// =====================================================================
// k_shade — hit record, scatter, emission, sky; compaction of survivors
// =====================================================================
__global__ __launch_bounds__(256) void k_shade(const DevScene sc, const RenderParams rp,
                                               const PathState in, const HitBuf hit, uint32_t n,
                                               PathState out, uint32_t* __restrict__ out_count) {
    __shared__ PerlinLds P;
    if (sc.has_perlin) {   // stage the Perlin tables in LDS (perlin.scm:32-36 data)
        for (int k = threadIdx.x; k < 768; k += 256) { P.ranvec[k] = sc.ranvec[k]; P.perm[k] = sc.perm[k]; }
        __syncthreads();
    }
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    bool alive = false;
    v3 no = mk(0, 0, 0), nd = mk(0, 0, 0), nT = mk(0, 0, 0);
    uint32_t pix = 0, smp = 0, wid = 0, rctr = 0, depth = 0;
    if (i < n) {
        const v3 ro = mk(in.ox[i], in.oy[i], in.oz[i]);
        const v3 rdir = mk(in.dx[i], in.dy[i], in.dz[i]);
        const double time = in.tm[i];
        const v3 T = mk(in.tr[i], in.tg[i], in.tb[i]);
        pix = in.pix[i]; smp = in.smp[i]; wid = in.wid[i]; rctr = in.rng[i]; depth = in.depth[i];
        const double t = hit.t[i];
        const int32_t leaf = hit.leaf[i];
        v3 L = mk(0, 0, 0);          // terminal radiance (sky / emission / 0)
        if (leaf < 0) {
            if (sc.sky == 0) {       // sky-color main.scm:91-95
                const v3 ud = unit(rdir);
                const double s = 0.5 * (1.0 + ud.y);
                L = mk(1.0, 1.0, 1.0) * (1.0 - s) + mk(0.5, 0.7, 1.0) * s;
            }
        } else {
            const LeafInfo li = sc.leaves[leaf];
            const Group G = sc.groups[li.group];
            v3 o = ro, d = rdir;
            if (G.chain >= 0) chain_ray(sc.chains[G.chain], o, d);
            v3 p = o + d * t;        // point-at-parameter on the (local) ray
            v3 nrm;
            if (li.type == LEAF_SPHERE) {
                const SphereRec S = sc.sph[li.local];
                nrm = (p - mk(S.cx, S.cy, S.cz)) * li.inv_r;
            } else if (li.type == LEAF_MSPHERE) {
                const MSphereRec S = sc.msph[li.local];
                const v3 cen = mk(S.c0x, S.c0y, S.c0z) + mk(S.dcx, S.dcy, S.dcz) * ((time - S.t0) / S.den);
                nrm = (p - cen) * li.inv_r;
            } else if (li.type == LEAF_RECT_XY) {
                nrm = mk(0.0, 0.0, 1.0);
            } else if (li.type == LEAF_RECT_XZ) {
                nrm = mk(0.0, 1.0, 0.0);
            } else {
                nrm = mk(1.0, 0.0, 0.0);
            }
            if (li.flip) nrm = nrm * -1.0;                          // flip-normals :438
            if (G.chain >= 0) chain_hit(sc.chains[G.chain], p, nrm);
            const DevMaterial m = sc.mats[li.mat];
            Rng g;
            g.init(rp.k0, rp.k1, pix, smp, rctr);
            const bool can_continue = depth < (uint32_t)kMaxDepth;
            // phase 1: scatter direction (all RNG draws, in the reference's order)
            bool need_tex = false;
            double wscale = 1.0, ipdf = 1.0;   // lambertian weight: (att*spdf) * (1/pdf)
            if (m.type == MAT_LAMBERTIAN) {                          // material.scm:24-39
                if (can_continue) {
                    // onb.scm:8-16
                    const v3 axis2 = unit(nrm);
                    const v3 a = (fabs(axis2.x) > 0.9) ? mk(0.0, 1.0, 0.0) : mk(1.0, 0.0, 0.0);
                    const v3 axis1 = unit(cross(axis2, a));
                    const v3 axis0 = cross(axis2, axis1);
                    // util.scm:37-44 (x2 quirk on x and y)
                    const double r1 = g.next();
                    const double r2 = g.next();
                    const double z = sqrt(1.0 - r2);
                    const double phi = 2.0 * kPi * r1;
                    double sphi, cphi;
                    sincos(phi, &sphi, &cphi);
                    const double x = cphi * 2.0 * sqrt(r2);
                    const double y = sphi * 2.0 * sqrt(r2);
                    const v3 target = (axis0 * x + axis1 * y) + axis2 * z;   // onb `local`
                    const v3 sd = unit(target);
                    const double pdf = dot(axis2, sd) / kPi;
                    double cosine = dot(nrm, unit(sd));
                    if (cosine < 0.0) cosine = 0.0;
                    wscale = cosine / kPi;                           // scattering-pdf
                    ipdf = 1.0 / pdf;
                    no = p; nd = sd; alive = true; need_tex = true;
                }
            } else if (m.type == MAT_METAL) {                        // material.scm:45-57 (R2)
                if (can_continue) {
                    const v3 reflected = reflect(unit(rdir), nrm);
                    v3 s;
                    for (;;) {                                       // util.scm:9-15
                        const double a = g.next(), b = g.next(), c = g.next();
                        s = mk(a * 2.0 - 1.0, b * 2.0 - 1.0, c * 2.0 - 1.0);
                        if (dot(s, s) < 1.0) break;
                    }
                    const v3 sd = reflected + s * m.fuzz;
                    if (dot(sd, nrm) > 0.0) { no = p; nd = sd; alive = true; need_tex = true; }
                }
            } else if (m.type == MAT_DIELECTRIC) {                   // material.scm:76-101 (R2)
                if (can_continue) {
                    const double ref_idx = m.ref_idx;
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
                        prob = r0 + (1.0 - r0) * pow(1.0 - cosine, 5.0);
                    }
                    nd = (g.next() < prob) ? reflected : refracted;
                    no = p; alive = true;                            // attenuation (1,1,1)
                }
            } else {                                                 // diffuse light :103-111
                need_tex = dot(nrm, rdir) < 0.0;
            }
            // phase 2: one texture evaluation site (albedo / emission at p)
            v3 tv = mk(1.0, 1.0, 1.0);
            if (need_tex) tv = tex_value(sc, P, m.tex, p);
            // phase 3: throughput (forward form of e + W (*) L_next)
            if (m.type == MAT_LAMBERTIAN) {
                nT = mk((T.x * (tv.x * wscale)) * ipdf, (T.y * (tv.y * wscale)) * ipdf,
                        (T.z * (tv.z * wscale)) * ipdf);
            } else if (m.type == MAT_METAL) {
                nT = T * tv;
            } else if (m.type == MAT_DIELECTRIC) {
                nT = T;
            } else if (need_tex) {
                L = tv;
            }
            rctr = g.ctr;
        }
        if (!alive) {                // path done: sample colour = T (*) L
            rp.sb[wid] = T.x * L.x;
            rp.sb[rp.B + wid] = T.y * L.y;
            rp.sb[2u * rp.B + wid] = T.z * L.z;
        }
    }
    // stream compaction of survivors: wave64 ballot, mbcnt prefix, one atomic per wave
    const unsigned long long mask = __ballot(alive);
    if (mask) {
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        const uint32_t leader = (uint32_t)__ffsll((long long)mask) - 1u;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(out_count, (uint32_t)__popcll(mask));
        base = __shfl(base, (int)leader, 64);
        if (alive) {
            const uint32_t k = base + below;
            out.ox[k] = no.x; out.oy[k] = no.y; out.oz[k] = no.z;
            out.dx[k] = nd.x; out.dy[k] = nd.y; out.dz[k] = nd.z;
            out.tm[k] = 0.0;                                         // make-ray: time 0 (Q4)
            out.tr[k] = nT.x; out.tg[k] = nT.y; out.tb[k] = nT.z;
            out.pix[k] = pix; out.smp[k] = smp; out.wid[k] = wid; out.rng[k] = rctr;
            out.depth[k] = depth + 1u;
        }
    }
}

// =====================================================================
// k_accumulate — *raw-data* running sum, samples added in order
// =====================================================================
__global__ __launch_bounds__(256) void k_accumulate(const RenderParams rp, uint32_t S,
                                                    double* __restrict__ accum) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= rp.npix) return;
    const uint32_t j = rp.pixlist[q];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double acc = accum[3u * j + c];
        const double* sbc = rp.sb + (size_t)c * rp.B;
        for (uint32_t s = 0; s < S; ++s) acc = acc + sbc[(size_t)s * rp.npix + q];
        accum[3u * j + c] = acc;
    }
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
hipError_t launch_raygen(const DevScene& sc, const RenderParams& rp, const PathState& st,
                         hipStream_t s) {
    const uint32_t blocks = (rp.B + 255u) / 256u;
    hipLaunchKernelGGL(k_raygen, dim3(blocks), dim3(256), 0, s, sc, rp, st);
    return hipGetLastError();
}
hipError_t launch_extend(const DevScene& sc, const PathState& st, uint32_t n, const HitBuf& hit,
                         hipStream_t s) {
    const uint32_t blocks = (n + 255u) / 256u;
    hipLaunchKernelGGL(k_extend, dim3(blocks), dim3(256), 0, s, sc, st, n, hit);
    return hipGetLastError();
}
hipError_t launch_shade(const DevScene& sc, const RenderParams& rp, const PathState& in,
                        const HitBuf& hit, uint32_t n, const PathState& out, uint32_t* out_count,
                        hipStream_t s) {
    const uint32_t blocks = (n + 255u) / 256u;
    hipLaunchKernelGGL(k_shade, dim3(blocks), dim3(256), 0, s, sc, rp, in, hit, n, out, out_count);
    return hipGetLastError();
}
hipError_t launch_accumulate(const RenderParams& rp, uint32_t S, double* accum, hipStream_t s) {
    const uint32_t blocks = (rp.npix + 255u) / 256u;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(256), 0, s, rp, S, accum);
    return hipGetLastError();
}
hipError_t launch_resolve_u8(const double* accum, uint32_t n, int count, uint8_t* out, hipStream_t s) {
    const uint32_t blocks = (n + 255u) / 256u;
    hipLaunchKernelGGL(k_resolve_u8, dim3(blocks), dim3(256), 0, s, accum, n, (double)count, out);
    return hipGetLastError();
}

}  // namespace rtamd
