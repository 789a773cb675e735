/*
 * rt_oracle.c — CPU f64 restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline) — never as part of the product path.
 *
 * It restates, in the reference's own evaluation order, the Gauche Scheme code
 * of soma-arc/scheme-raytrace (reference @ /root/reference):
 *   vec.scm:7-70           vector algebra (left folds; unit = v * (1/|v|))
 *   ray.scm:8-54           ray #(o d time), make-ray forces time 0 (Q4)
 *   util.scm:9-23,37-44    rejection samplers, cosine direction (x2 quirk, Q1)
 *   onb.scm:8-36           ONB from w, `local`
 *   camera.scm:63-92       make-camera, get-ray (direction not normalised)
 *   geometry.scm:14-56     hit dispatch, hit-obj-list (closest, strict <)
 *   geometry.scm:146-215   sphere / moving sphere
 *   geometry.scm:376-543   rects, flip-normals, box, translate, rotate-y
 *   material.scm:15-111    lambertian / metal / dielectric / diffuse light
 *   texture.scm:12-34      constant / checker / noise / marble
 *   perlin.scm:51-103      perlin-interp, noise (aliasing quirk Q2), turb
 *   main.scm:91-124        sky-color, black, color (recursive), correct-gamma
 *   main.scm:471-491       trace-all (jitter, running sum, resolve)
 * with the repairs R1-R3 of SURVEY.md Appendix A (metal / dielectric are
 * specular: L = e + att*L_next).  The reference's global srfi-27 stream is
 * replaced by the counter-based Philox4x32-10 stream keyed by
 * (seed, pixel, sample) that the GPU uses too, with
 * draws consumed in the order the Scheme code consumes them (arguments
 * evaluated left to right).
 *
 * Build: see oracle/Makefile (-O2 -ffp-contract=off: no FMA contraction, so
 * every f64 operation rounds exactly as the reference's flonum ops do).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#define ORC_MAX_DEPTH 100              /* main.scm:26 */
#define ORC_TMIN 0.001                 /* main.scm:104 */
#define ORC_TMAX 999999999999.0        /* constant.scm:6 */
#define ORC_PI 3.141592653589793       /* math.const pi = 4*atan(1) */

/* ------------------------------------------------------------------ RNG */
/* Philox4x32-10 (Salmon et al., SC'11; Random123 reference constants). */
static void philox4x32_10(uint32_t ctr[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ ctr[1] ^ k0, n2 = hi0 ^ ctr[3] ^ k1;
        ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
    }
}

void orc_philox(const uint32_t ctr_in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
    uint32_t c[4] = {ctr_in[0], ctr_in[1], ctr_in[2], ctr_in[3]};
    philox4x32_10(c, k0, k1);
    memcpy(out, c, sizeof c);
}

/* two u32 -> double in (0,1): 52 random bits, u = (2k+1) * 2^-53 */
static double u32pair_to_unit(uint32_t hi, uint32_t lo) {
    uint64_t k = ((uint64_t)(hi >> 12) << 32) | lo;
    return (double)(2 * k + 1) * (1.0 / 9007199254740992.0);
}

typedef struct {
    uint32_t k0, k1, pix, smp, ctr;
} orc_rng;

/* draw d of the stream: block d>>1, ctr = {block, sample, pixel, 0} */
static double orc_random_real(orc_rng* g) {
    uint32_t d = g->ctr++;
    uint32_t c[4] = {d >> 1, g->smp, g->pix, 0u};
    philox4x32_10(c, g->k0, g->k1);
    return (d & 1u) ? u32pair_to_unit(c[2], c[3]) : u32pair_to_unit(c[0], c[1]);
}

/* exported for tests: draw `n` values of stream (seed, pix, smp) from draw index `first` */
void orc_stream(uint64_t seed, uint32_t pix, uint32_t smp, uint32_t first, int n, double* out) {
    orc_rng g = {(uint32_t)seed, (uint32_t)(seed >> 32), pix, smp, first};
    for (int i = 0; i < n; ++i) out[i] = orc_random_real(&g);
}

/* --------------------------------------------------------------- vec.scm */
typedef struct { double x, y, z; } v3;
static inline v3 V(double x, double y, double z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
/* sum / diff are left folds of f64vector-add / -sub (vec.scm:20-33) */
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, double k) { return V(a.x * k, a.y * k, a.z * k); }
/* f64vector-dot: r = 0; r += a_i*b_i (i = 0..2) */
static inline double vdot(v3 a, v3 b) {
    double r = 0.0;
    r += a.x * b.x; r += a.y * b.y; r += a.z * b.z;
    return r;
}
static inline double vlength(v3 a) { return sqrt(vdot(a, a)); }          /* vec.scm:54 */
static inline v3 vunit(v3 a) { double k = 1.0 / vlength(a); return vscale(a, k); } /* :60-62 */
static inline v3 vcross(v3 a, v3 b) {                                       /* :64-70 */
    return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}

typedef struct { v3 o, d; double time; } ray_t;
static inline v3 point_at(ray_t r, double t) { return vadd(r.o, vscale(r.d, t)); } /* ray.scm:23-25 */

/* ------------------------------------------------------------- scene data */
enum { TEX_CONSTANT = 0, TEX_CHECKER = 1, TEX_NOISE = 2, TEX_MARBLE = 3 };
enum { MAT_LAMBERTIAN = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2, MAT_DIFFUSE_LIGHT = 3 };
enum { OBJ_SPHERE = 0, OBJ_MOVING_SPHERE, OBJ_RECT, OBJ_FLIP, OBJ_BOX, OBJ_TRANSLATE,
       OBJ_ROTATE_Y, OBJ_LIST, OBJ_BVH, OBJ_BEZIER, OBJ_MEDIUM, OBJ_KLEIN };

typedef struct { int type, a, b; v3 rgb; double scale; } orc_tex;
typedef struct { int type, tex; double fuzz, ref_idx; } orc_mat;
typedef struct {
    int type, mat, child, axis;
    int first, count;                   /* OBJ_LIST / OBJ_BVH children in kids[] */
    v3 c0, c1;                          /* sphere centre / moving centres / box p0,p1 / offset */
    double r, t0, t1;
    double a0, a1, b0, b1, k;           /* rect */
    double sin_t, cos_t;                /* rotate-y */
    int box_list;                       /* OBJ_BOX: its 6-rect list object */
    v3 cp[4];                           /* OBJ_BEZIER control points */
    double width;
    double density;                     /* OBJ_MEDIUM (child = boundary, mat = phase lambertian) */
} orc_obj;

/* A conservative f64 bounding-volume tree over one OBJ_BVH's primitives (see
 * "BVH" below).  Leaves hold up to 4 primitives of prim[]; node boxes are
 * padded outward, so culling never removes a primitive that could win. */
typedef struct { double lo[3], hi[3]; int left, right, first, count; } orc_bnode;
typedef struct {
    int nprim;
    int* prim;                          /* object ids, in leaf order */
    int* order;                         /* each one's index in the flattened list (tie-breaks) */
    unsigned char* nonstrict;           /* 1: hits at t == t-max (curves), 0: only t < t-max (spheres) */
    orc_bnode* node; int nnode, cnode;
} orc_bvh;

typedef struct {
    orc_tex* tex; int ntex, ctex;
    orc_mat* mat; int nmat, cmat;
    orc_obj* obj; int nobj, cobj;
    int* kids; int nkids, ckids;
    double cam[24];
    int sky, world;
    int light;                          /* light-sampling target object (-1: off), pdf.scm extension */
    v3 ranvec[256];
    int perm_x[256], perm_y[256], perm_z[256];
    int have_perlin;
    /* OBJ_BVH acceleration (built lazily by scene_prepare; bvh_of[obj] = -1: flat list) */
    orc_bvh* bvh; int nbvh;
    int* bvh_of; int nbvh_of;
    int bvh_ready, bvh_flat;
} orc_scene;

#define GROW(ptr, n, cap)                                                    \
    do {                                                                     \
        if ((n) >= (cap)) {                                                  \
            (cap) = (cap) ? 2 * (cap) : 16;                                  \
            (ptr) = realloc((ptr), (size_t)(cap) * sizeof(*(ptr)));          \
        }                                                                    \
    } while (0)

orc_scene* orc_scene_new(void) {
    orc_scene* s = calloc(1, sizeof *s);
    s->world = -1;
    s->light = -1;
    return s;
}
static void bvh_clear(orc_scene* s) {
    for (int i = 0; i < s->nbvh; ++i) {
        free(s->bvh[i].prim); free(s->bvh[i].order); free(s->bvh[i].nonstrict); free(s->bvh[i].node);
    }
    free(s->bvh); free(s->bvh_of);
    s->bvh = 0; s->nbvh = 0; s->bvh_of = 0; s->nbvh_of = 0; s->bvh_ready = 0;
}
void orc_scene_free(orc_scene* s) {
    if (!s) return;
    bvh_clear(s);
    free(s->tex); free(s->mat); free(s->obj); free(s->kids); free(s);
}

int orc_add_texture_constant(orc_scene* s, const double rgb[3]) {
    GROW(s->tex, s->ntex, s->ctex);
    orc_tex t; memset(&t, 0, sizeof t); t.type = TEX_CONSTANT; t.rgb = V(rgb[0], rgb[1], rgb[2]);
    s->tex[s->ntex] = t; return s->ntex++;
}
int orc_add_texture_checker(orc_scene* s, int even, int odd) {
    GROW(s->tex, s->ntex, s->ctex);
    orc_tex t; memset(&t, 0, sizeof t); t.type = TEX_CHECKER; t.a = even; t.b = odd;
    s->tex[s->ntex] = t; return s->ntex++;
}
int orc_add_texture_noise(orc_scene* s, double sc) {
    GROW(s->tex, s->ntex, s->ctex);
    orc_tex t; memset(&t, 0, sizeof t); t.type = TEX_NOISE; t.scale = sc;
    s->tex[s->ntex] = t; return s->ntex++;
}
int orc_add_texture_marble(orc_scene* s, double sc) {
    GROW(s->tex, s->ntex, s->ctex);
    orc_tex t; memset(&t, 0, sizeof t); t.type = TEX_MARBLE; t.scale = sc;
    s->tex[s->ntex] = t; return s->ntex++;
}
static int add_mat(orc_scene* s, int type, int tex, double fuzz, double ref) {
    GROW(s->mat, s->nmat, s->cmat);
    orc_mat m; m.type = type; m.tex = tex; m.fuzz = fuzz; m.ref_idx = ref;
    s->mat[s->nmat] = m; return s->nmat++;
}
int orc_add_material_lambertian(orc_scene* s, int tex) { return add_mat(s, MAT_LAMBERTIAN, tex, 0, 0); }
int orc_add_material_metal(orc_scene* s, int tex, double fuzz) { return add_mat(s, MAT_METAL, tex, fuzz, 0); }
int orc_add_material_dielectric(orc_scene* s, double ref) { return add_mat(s, MAT_DIELECTRIC, -1, 0, ref); }
int orc_add_material_diffuse_light(orc_scene* s, int tex) { return add_mat(s, MAT_DIFFUSE_LIGHT, tex, 0, 0); }

static int new_obj(orc_scene* s, int type) {
    s->bvh_ready = 0;
    GROW(s->obj, s->nobj, s->cobj);
    memset(&s->obj[s->nobj], 0, sizeof(orc_obj));
    s->obj[s->nobj].type = type;
    s->obj[s->nobj].child = -1;
    s->obj[s->nobj].mat = -1;
    return s->nobj++;
}
int orc_add_sphere(orc_scene* s, const double c[3], double r, int mat) {
    int i = new_obj(s, OBJ_SPHERE);
    s->obj[i].c0 = V(c[0], c[1], c[2]); s->obj[i].r = r; s->obj[i].mat = mat;
    return i;
}
int orc_add_moving_sphere(orc_scene* s, const double c0[3], const double c1[3], double t0, double t1,
                          double r, int mat) {
    int i = new_obj(s, OBJ_MOVING_SPHERE);
    orc_obj* o = &s->obj[i];
    o->c0 = V(c0[0], c0[1], c0[2]); o->c1 = V(c1[0], c1[1], c1[2]);
    o->t0 = t0; o->t1 = t1; o->r = r; o->mat = mat;
    return i;
}
int orc_add_rect(orc_scene* s, int axis, double a0, double a1, double b0, double b1, double k, int mat) {
    int i = new_obj(s, OBJ_RECT);
    orc_obj* o = &s->obj[i];
    o->axis = axis; o->a0 = a0; o->a1 = a1; o->b0 = b0; o->b1 = b1; o->k = k; o->mat = mat;
    return i;
}
int orc_add_flip_normals(orc_scene* s, int child) {
    int i = new_obj(s, OBJ_FLIP);
    s->obj[i].child = child; s->obj[i].mat = s->obj[child].mat;
    return i;
}
int orc_add_list(orc_scene* s, const int* objs, int n) {
    int i = new_obj(s, OBJ_LIST);
    s->obj[i].first = s->nkids; s->obj[i].count = n;
    for (int j = 0; j < n; ++j) { GROW(s->kids, s->nkids, s->ckids); s->kids[s->nkids++] = objs[j]; }
    return i;
}
int orc_add_bvh(orc_scene* s, const int* objs, int n, double t0, double t1, int sah) {
    (void)t0; (void)t1; (void)sah;
    int i = orc_add_list(s, objs, n);
    s->obj[i].type = OBJ_BVH;
    return i;
}
/* geometry.scm:444-463: the box is a scene of 6 rects (in this order) */
int orc_add_box(orc_scene* s, const double p0[3], const double p1[3], int mat) {
    int r[6];
    r[0] = orc_add_rect(s, 0, p0[0], p1[0], p0[1], p1[1], p1[2], mat);
    r[1] = orc_add_flip_normals(s, orc_add_rect(s, 0, p0[0], p1[0], p0[1], p1[1], p0[2], mat));
    r[2] = orc_add_rect(s, 1, p0[0], p1[0], p0[2], p1[2], p1[1], mat);
    r[3] = orc_add_flip_normals(s, orc_add_rect(s, 1, p0[0], p1[0], p0[2], p1[2], p0[1], mat));
    r[4] = orc_add_rect(s, 2, p0[1], p1[1], p0[2], p1[2], p1[0], mat);
    r[5] = orc_add_flip_normals(s, orc_add_rect(s, 2, p0[1], p1[1], p0[2], p1[2], p0[0], mat));
    int lst = orc_add_list(s, r, 6);
    int i = new_obj(s, OBJ_BOX);
    s->obj[i].box_list = lst; s->obj[i].mat = mat;
    s->obj[i].c0 = V(p0[0], p0[1], p0[2]); s->obj[i].c1 = V(p1[0], p1[1], p1[2]);
    return i;
}
int orc_add_translate(orc_scene* s, int child, const double off[3]) {
    int i = new_obj(s, OBJ_TRANSLATE);
    s->obj[i].child = child; s->obj[i].c0 = V(off[0], off[1], off[2]);
    s->obj[i].mat = s->obj[child].mat;
    return i;
}
/* geometry.scm:483-487: radians = pi/180 * angle */
int orc_add_rotate_y(orc_scene* s, int child, double angle) {
    int i = new_obj(s, OBJ_ROTATE_Y);
    double radians = (ORC_PI / 180.0) * angle;
    s->obj[i].child = child; s->obj[i].sin_t = sin(radians); s->obj[i].cos_t = cos(radians);
    s->obj[i].mat = s->obj[child].mat;
    return i;
}
int orc_add_bezier(orc_scene* s, const double* cps, double width, int mat) {
    int i = new_obj(s, OBJ_BEZIER);
    for (int k = 0; k < 4; ++k) s->obj[i].cp[k] = V(cps[3 * k], cps[3 * k + 1], cps[3 * k + 2]);
    s->obj[i].width = width; s->obj[i].mat = mat;
    return i;
}

int orc_add_klein(orc_scene* s, const double c[3], int mat) {
    int i = new_obj(s, OBJ_KLEIN);
    s->obj[i].c0 = V(c[0], c[1], c[2]); s->obj[i].mat = mat;
    return i;
}

int orc_add_constant_medium(orc_scene* s, int boundary, double density, int tex) {
    int phase = orc_add_material_lambertian(s, tex);     /* (m:make-lambertian a), geometry.scm:546 */
    int i = new_obj(s, OBJ_MEDIUM);
    s->obj[i].child = boundary; s->obj[i].density = density; s->obj[i].mat = phase;
    return i;
}

int orc_add_bezier_array(orc_scene* s, const double* cps, int n, double width, int mat) {
    int first = -1;
    for (int i = 0; i < n; ++i) {
        int id = orc_add_bezier(s, cps + 12 * (size_t)i, width, mat);
        if (i == 0) first = id;
    }
    return first;
}

void orc_set_camera(orc_scene* s, const double cam[24]) { memcpy(s->cam, cam, sizeof s->cam); s->bvh_ready = 0; }
/* 1: traverse every OBJ_BVH as the flat list it restates (the tie-break
 * semantics the trees reproduce); 0 (default): use the trees. */
void orc_set_bvh_flat(orc_scene* s, int flat) { s->bvh_flat = flat; }
void orc_set_sky(orc_scene* s, int sky) { s->sky = sky; }
void orc_set_light_sampling(orc_scene* s, int obj) { s->light = obj; }
void orc_set_world(orc_scene* s, int world) { s->world = world; }
void orc_set_perlin_tables(orc_scene* s, const double* ranvec, const int32_t* px, const int32_t* py,
                           const int32_t* pz) {
    for (int i = 0; i < 256; ++i) {
        s->ranvec[i] = V(ranvec[3 * i], ranvec[3 * i + 1], ranvec[3 * i + 2]);
        s->perm_x[i] = px[i]; s->perm_y[i] = py[i]; s->perm_z[i] = pz[i];
    }
    s->have_perlin = 1;
}

/* camera.scm:63-78 — make-camera */
void orc_make_camera(const double from[3], const double at[3], const double vup_[3], double vfov,
                     double aspect, double aperture, double focus, double t0, double t1, double out[24]) {
    v3 lookfrom = V(from[0], from[1], from[2]), lookat = V(at[0], at[1], at[2]);
    v3 vup = V(vup_[0], vup_[1], vup_[2]);
    double theta = vfov * (ORC_PI / 180.0);
    double half_height = tan(theta / 2);
    double half_width = aspect * half_height;
    v3 w = vunit(vsub(lookfrom, lookat));
    v3 u = vunit(vcross(vup, w));
    v3 v = vcross(w, u);
    v3 llc = vsub(vsub(vsub(lookfrom, vscale(u, half_width * focus)), vscale(v, half_height * focus)),
                  vscale(w, focus));
    v3 hor = vscale(u, 2 * half_width * focus);
    v3 ver = vscale(v, 2 * half_height * focus);
    v3 slots[7] = {llc, hor, ver, lookfrom, w, u, v};
    for (int i = 0; i < 7; ++i) { out[3 * i] = slots[i].x; out[3 * i + 1] = slots[i].y; out[3 * i + 2] = slots[i].z; }
    out[21] = aperture / 2; out[22] = t0; out[23] = t1;
}

/* ---------------------------------------------------------- util / onb */
/* util.scm:9-15 */
static v3 random_in_unit_sphere(orc_rng* g) {
    for (;;) {
        double a = orc_random_real(g), b = orc_random_real(g), c = orc_random_real(g);
        v3 p = vsub(vscale(V(a, b, c), 2), V(1, 1, 1));
        if (vdot(p, p) < 1) return p;
    }
}
/* util.scm:17-23 */
static v3 random_in_unit_disk(orc_rng* g) {
    for (;;) {
        double a = orc_random_real(g), b = orc_random_real(g);
        v3 p = vsub(vscale(V(a, b, 0), 2), V(1, 1, 0));
        if (vdot(p, p) < 1) return p;
    }
}
/* util.scm:37-44 — note the stray *2 on x and y (Q1) */
static v3 random_cosine_direction(orc_rng* g) {
    double r1 = orc_random_real(g);
    double r2 = orc_random_real(g);
    double z = sqrt(1 - r2);
    double phi = 2 * ORC_PI * r1;
    double x = cos(phi) * 2 * sqrt(r2);
    double y = sin(phi) * 2 * sqrt(r2);
    return V(x, y, z);
}
typedef struct { v3 u, v, w; } onb_t;
static onb_t make_onb_from_w(v3 n) {                                   /* onb.scm:8-16 */
    onb_t b;
    v3 axis2 = vunit(n);
    v3 a = (fabs(axis2.x) > 0.9) ? V(0, 1, 0) : V(1, 0, 0);
    v3 axis1 = vunit(vcross(axis2, a));
    v3 axis0 = vcross(axis2, axis1);
    b.u = axis0; b.v = axis1; b.w = axis2;
    return b;
}
static v3 onb_local(onb_t b, v3 a) {                                   /* onb.scm:27-36 */
    return vadd(vadd(vscale(b.u, a.x), vscale(b.v, a.y)), vscale(b.w, a.z));
}

/* ----------------------------------------------------------- perlin.scm */
static double perlin_noise(const orc_scene* s, v3 p) {
    double fx = floor(p.x), fy = floor(p.y), fz = floor(p.z);
    double u = p.x - fx, v = p.y - fy, w = p.z - fz;
    long i = (long)fx, j = (long)fy, k = (long)fz;
    /* perlin.scm:76 — (make-vector 2 (make-vector 2 (make-vector 2))) shares
     * one innermost vector, so after the fill loop c[*][*][dk] holds the
     * value written at di = dj = 1 (Q2). */
    v3 c[2];
    for (int dk = 0; dk < 2; ++dk) {
        int h = s->perm_x[(i + 1) & 255] ^ s->perm_y[(j + 1) & 255] ^ s->perm_z[(k + dk) & 255];
        c[dk] = s->ranvec[h];
    }
    /* perlin-interp :51-67 */
    double uu = u * u * (3 - 2 * u);
    double vv = v * v * (3 - 2 * v);
    double ww = w * w * (3 - 2 * w);
    double acc = 0;
    for (int di = 0; di < 2; ++di)
        for (int dj = 0; dj < 2; ++dj)
            for (int dk = 0; dk < 2; ++dk) {
                double wi = di ? uu : (1 - uu);
                double wj = dj ? vv : (1 - vv);
                double wk = dk ? ww : (1 - ww);
                v3 weight = V(u - di, v - dj, w - dk);
                acc += wi * wj * wk * vdot(weight, c[dk]);
            }
    return acc;
}
static double perlin_turb(const orc_scene* s, v3 p) {                  /* perlin.scm:92-103 */
    double acc = 0, weight = 1;
    for (int depth = 0; depth < 7; ++depth) {
        acc = acc + weight * perlin_noise(s, p);
        p = vscale(p, 2);
        weight = weight * 0.5;
    }
    return fabs(acc);
}

/* ---------------------------------------------------------- texture.scm */
static v3 tex_value(const orc_scene* s, int id, double u, double v, v3 p) {
    const orc_tex* t = &s->tex[id];
    switch (t->type) {
    case TEX_CONSTANT: return t->rgb;
    case TEX_CHECKER: {                                                 /* :16-23 */
        double sines = sin(10 * p.x) * sin(10 * p.y) * sin(10 * p.z);
        return (sines < 0) ? tex_value(s, t->b, u, v, p) : tex_value(s, t->a, u, v, p);
    }
    case TEX_NOISE:                                                     /* :25-28 */
        return vscale(V(1, 1, 1), perlin_noise(s, vscale(p, t->scale)));
    case TEX_MARBLE: {                                                  /* :30-34 */
        double m = 0.5 * (1 + sin(t->scale * p.z + 10 * perlin_turb(s, p)));
        return vscale(V(1, 1, 1), m);
    }
    }
    return V(0, 0, 0);
}

/* --------------------------------------------------------- geometry.scm */
typedef struct { double t; v3 p, n; int mat; double u, v; } hitrec;

/* ------------------------------------------------------------ bezier.scm */
/* A cubic Bezier curve of a given width (bezier.scm:61-223). */
typedef struct { v3 p[4]; } bez4;

static v3 bez_point(const bez4* c, double t) {                          /* bez-p :67-77 */
    double t2 = t * t, t3 = t2 * t;
    double u = 1 - t, u2 = u * u, u3 = u2 * u;
    return vadd(vadd(vadd(vscale(c->p[0], u3), vscale(c->p[1], 3 * u2 * t)), vscale(c->p[2], 3 * u * t2)),
                vscale(c->p[3], t3));
}
static v3 idiv(v3 a, v3 b, double t) { return vadd(vscale(a, 1 - t), vscale(b, t)); }   /* :45-47 */
static void bez_split(const bez4* c, double t, bez4* l, bez4* r) {      /* split :78-87 */
    v3 sp = bez_point(c, t);
    v3 nbc = idiv(c->p[1], c->p[2], t);
    v3 lb = idiv(c->p[0], c->p[1], t);
    v3 lc = idiv(lb, nbc, t);
    v3 rc = idiv(c->p[2], c->p[3], t);
    v3 rb = idiv(nbc, rc, t);
    l->p[0] = c->p[0]; l->p[1] = lb; l->p[2] = lc; l->p[3] = sp;
    r->p[0] = sp; r->p[1] = rb; r->p[2] = rc; r->p[3] = c->p[3];
}
/* bez-tan-vec :106-117 (t is the exact integer 0 or 1 at its call sites) */
static v3 bez_tan(const bez4* c, int t) {
    const v3 a = c->p[0], b = c->p[1], cc = c->p[2], d = c->p[3];
    v3 coef_a = vadd(vadd(vadd(vscale(b, 3), d), vscale(cc, -3)), vscale(a, -1));
    v3 coef_b = vscale(vadd(vadd(a, vscale(b, -2)), cc), 3);
    v3 coef_c = vscale(vsub(b, a), 3);
    double t2 = (double)(t * t);
    return vunit(vadd(vadd(vscale(coef_a, 3 * t2), vscale(coef_b, 2 * t)), coef_c));
}
static double dot2d(v3 a, v3 b) { return vdot(V(a.x, a.y, 0), V(b.x, b.y, 0)); }   /* :57-59 */

/* get-projection-mat :13-43, as a 4x4 row-major matrix M (array-mul of the
 * translation and the rotation: s = 0; s += T[i][k]*R[k][j], k = 0..3) */
static void projection_mat(ray_t r, double M[16]) {
    double ox = -r.o.x, oy = -(-r.o.z), oz = -r.o.y;
    v3 rd = vunit(r.d);
    double lx = rd.x, ly = -rd.z, lz = rd.y;
    double d = sqrt(lx * lx + lz * lz);
    double R[16];
    if (d == 0) {
        double angle = (ly >= 0) ? -(ORC_PI / 2) : (ORC_PI / 2);
        double cs = cos(angle), sn = sin(angle);
        double Rr[16] = {1, 0, 0, 0, 0, cs, -sn, 0, 0, sn, cs, 0, 0, 0, 0, 1};
        memcpy(R, Rr, sizeof R);
    } else {
        double Rr[16] = {lz / d, (-1 * lx * ly) / d, lx, 0, 0, d, ly, 0,
                         (-lx) / d, (-1 * ly * lz) / d, lz, 0, 0, 0, 0, 1};
        memcpy(R, Rr, sizeof R);
    }
    double T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, ox, oy, oz, 1};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double sum = 0;
            for (int k = 0; k < 4; ++k) sum = sum + T[4 * i + k] * R[4 * k + j];
            M[4 * i + j] = sum;
        }
}
/* transform :49-55 — row vector (x, -z, y, 1) times M */
static v3 bez_transform(v3 p, const double M[16]) {
    double row[4] = {p.x, -p.z, p.y, 1};
    double out[3];
    for (int j = 0; j < 3; ++j) {
        double sum = 0;
        for (int k = 0; k < 4; ++k) sum = sum + row[k] * M[4 * k + j];
        out[j] = sum;
    }
    return V(out[0], out[1], out[2]);
}

/* converge :121-175.  Both children of a split see the t the parent was
 * called with, so the recursion returns min z over every leaf hit with
 * z <= t_entry; *found tells whether any leaf hit. */
static void bez_converge(const bez4* c, int depth, double v0, double vn, double t, double width1,
                         double width2, int* found, double* best) {
    double mn[3] = {ORC_TMAX, ORC_TMAX, ORC_TMAX}, mx[3] = {-ORC_TMAX, -ORC_TMAX, -ORC_TMAX};
    for (int i = 0; i < 4; ++i) {                                  /* bbox :88-98 */
        double pc[3] = {c->p[i].x, c->p[i].y, c->p[i].z};
        for (int a = 0; a < 3; ++a) {
            double lo = pc[a] - width1, hi = pc[a] + width1;
            mn[a] = (lo < mn[a]) ? lo : mn[a];
            mx[a] = (hi > mx[a]) ? hi : mx[a];
        }
    }
    if (mn[2] >= t || mx[2] <= 0.000001 || mn[0] >= width1 || mx[0] <= -width1 || mn[1] >= width1 ||
        mx[1] <= -width1)
        return;
    if (depth < 0) {                                               /* leaf :130-166 */
        v3 dir = vsub(c->p[3], c->p[0]);
        v3 dp0 = bez_tan(c, 0);
        if (dot2d(dir, dp0) < 0) dp0 = vscale(dp0, -1);
        if (dot2d(dp0, vscale(c->p[0], -1)) < 0) return;
        v3 dpn = bez_tan(c, 1);
        if (dot2d(dir, dpn) < 0) dpn = vscale(dpn, -1);
        if (dot2d(dpn, c->p[3]) < 0) return;
        double w = dir.x * dir.x + dir.y * dir.y;
        if (w == 0) return;
        w = (c->p[0].x * dir.x + c->p[0].y * dir.y) / (-w);
        w = (w < 0) ? 0 : ((w > 1) ? 1 : w);                       /* clamp */
        double v = v0 * (1 - w) + vn * w;
        v3 p = bez_point(c, v);                                    /* sub-curve at the global v (Q11) */
        if (p.x * p.x + p.y * p.y >= width2 || p.z <= 0.0001 || t < p.z) return;
        if (!*found || p.z < *best) *best = p.z;
        *found = 1;
        return;
    }
    double vm = (v0 + vn) / 2;
    bez4 l, r;
    bez_split(c, 0.5, &l, &r);
    bez_converge(&l, depth - 1, v0, vm, t, width1, width2, found, best);
    bez_converge(&r, depth - 1, vm, vn, t, width1, width2, found, best);
}

/* hit :176-214 */
static int bezier_hit(const orc_obj* o, ray_t r, double tmin, double tmax, hitrec* rec) {
    double width1 = o->width / 2, width2 = width1 * width1, eps = o->width / 20;
    double M[16];
    projection_mat(r, M);
    bez4 c;
    for (int k = 0; k < 4; ++k) c.p[k] = bez_transform(o->cp[k], M);
    double l0 = -ORC_TMAX;
    for (int i = 0; i < 2; ++i) {
        double x = fabs(c.p[i].x + -2 * c.p[i + 1].x + c.p[i + 2].x);
        double y = fabs(c.p[i].y + -2 * c.p[i + 1].y + c.p[i + 2].y);
        double m = x;
        if (y > m) m = y;
        if (l0 > m) m = l0;
        l0 = m;
    }
    double md = log((sqrt(2) * 4 * 3 * l0) / (8 * eps)) / log(4);
    int max_depth = (md == -INFINITY) ? 0 : (int)ceil(md);
    int found = 0;
    double t = tmax;
    bez_converge(&c, max_depth, 0, 1, tmax, width1, width2, &found, &t);
    if (!found) t = tmax;
    if (!(found && tmin < t)) return 0;
    rec->t = t;
    rec->p = point_at(r, t);                 /* t is a ray-space distance used on the raw ray (Q10) */
    rec->n = vscale(r.d, -1);                /* un-normalised (Q12) */
    rec->mat = o->mat;
    rec->u = 0; rec->v = 0;
    return 1;
}

static int hit_obj(const orc_scene* s, int id, ray_t r, double tmin, double tmax, hitrec* rec);

/* ---------------------------------------- Kleinian limit set, geometry.scm:590-664 */
static const double KLEIN_SP[6][3] = {{300, 300, 0}, {300, -300, 0}, {-300, 300, 0},
                                      {-300, -300, 0}, {0, 0, 424.26}, {0, 0, -424.26}};
/* dist-func :609-635: sphere inversions (at most 10), then a scaled sphere distance */
static double klein_dist(v3 center, v3 p) {
    v3 pos = vsub(p, center);
    double dr = 1;
    for (int iter = 0;; ++iter) {
        if (iter >= 10) return 0.7 * ((vlength(pos) - 125) / fabs(dr));
        int idx = 0;
        for (; idx < 6; ++idx)
            if (vlength(vsub(pos, V(KLEIN_SP[idx][0], KLEIN_SP[idx][1], KLEIN_SP[idx][2]))) < 300) break;
        if (idx == 6) return 0.7 * ((vlength(pos) - 125) / fabs(dr));
        v3 sp = V(KLEIN_SP[idx][0], KLEIN_SP[idx][1], KLEIN_SP[idx][2]);
        v3 diff = vsub(pos, sp);
        dr = dr * (90000 / vdot(diff, diff));
        double l = vlength(diff);
        pos = vadd(vscale(vscale(diff, 90000), 1 / (l * l)), sp);
    }
}
/* get-normal :637-643 */
static v3 klein_normal(v3 center, v3 p) {
    return vunit(V(klein_dist(center, vadd(p, V(0.01, 0, 0))) - klein_dist(center, vsub(p, V(0.01, 0, 0))),
                   klein_dist(center, vadd(p, V(0, 0.01, 0))) - klein_dist(center, vsub(p, V(0, 0.01, 0))),
                   klein_dist(center, vadd(p, V(0, 0, 0.01))) - klein_dist(center, vsub(p, V(0, 0, 0.01)))));
}
/* make-klein's hit :655-670: sphere tracing with the raw direction */
static int klein_hit(const orc_obj* o, ray_t r, double tmin, double tmax, hitrec* rec) {
    double len = 0;
    v3 pos = r.o;
    for (int iter = 0; iter < 100; ++iter) {
        double dist = klein_dist(o->c0, pos);
        len = len + dist;
        pos = vadd(r.o, vscale(r.d, len));
        if (dist < 0.001 && tmin < len && len < tmax) {
            rec->t = len;
            rec->p = point_at(r, len);
            rec->n = klein_normal(o->c0, pos);
            rec->mat = o->mat;
            rec->u = 0; rec->v = 0;
            return 1;
        }
    }
    return 0;
}

/* The path's random stream, for hit functions that draw (the constant
 * medium, geometry.scm:564): set by color() around each world hit. */
static __thread orc_rng* tl_rng;

static int hit_list(const orc_scene* s, int first, int count, ray_t r, double tmin, double tmax,
                    hitrec* rec) {                                      /* :33-50 */
    int hit_anything = 0;
    double closest = tmax;
    hitrec tmp;
    for (int i = 0; i < count; ++i) {
        if (hit_obj(s, s->kids[first + i], r, tmin, closest, &tmp)) {
            hit_anything = 1; closest = tmp.t; *rec = tmp;
        }
    }
    return hit_anything;
}

static int sphere_hit(v3 center, double radius, int mat, ray_t r, double tmin, double tmax, hitrec* rec) {
    v3 oc = vsub(r.o, center);
    double a = vdot(r.d, r.d);
    double b = vdot(oc, r.d);
    double c = vdot(oc, oc) - radius * radius;
    double disc = b * b - a * c;
    if (disc <= 0) return 0;
    double temp = (-b - sqrt(disc)) / a;
    if (!(tmin < temp && temp < tmax)) {
        temp = (-b + sqrt(disc)) / a;
        if (!(tmin < temp && temp < tmax)) return 0;
    }
    rec->t = temp;
    rec->p = point_at(r, temp);
    rec->n = vscale(vsub(rec->p, center), 1.0 / radius);
    rec->mat = mat;
    /* get-sphere-uv (:138-144) is dead for every reference texture (Q3) */
    rec->u = 0; rec->v = 0;
    return 1;
}

static int rect_hit(const orc_obj* o, ray_t r, double tmin, double tmax, hitrec* rec) {
    /* axis 0: xy (k on z), 1: xz (k on y), 2: yz (k on x) — :376-431 */
    double ok, dk, oa, da, ob, db;
    v3 n;
    if (o->axis == 0) { ok = r.o.z; dk = r.d.z; oa = r.o.x; da = r.d.x; ob = r.o.y; db = r.d.y; n = V(0, 0, 1); }
    else if (o->axis == 1) { ok = r.o.y; dk = r.d.y; oa = r.o.x; da = r.d.x; ob = r.o.z; db = r.d.z; n = V(0, 1, 0); }
    else { ok = r.o.x; dk = r.d.x; oa = r.o.y; da = r.d.y; ob = r.o.z; db = r.d.z; n = V(1, 0, 0); }
    double t = (o->k - ok) / dk;
    if (t < tmin || t > tmax) return 0;
    double a = oa + t * da;
    double b = ob + t * db;
    if (a < o->a0 || a > o->a1 || b < o->b0 || b > o->b1) return 0;
    rec->t = t;
    rec->p = point_at(r, t);
    rec->n = n;
    rec->mat = o->mat;
    rec->u = (a - o->a0) / (o->a1 - o->a0);
    rec->v = (b - o->b0) / (o->b1 - o->b0);
    return 1;
}

/* ------------------------------------------------------------------ BVH
 * geometry.scm:226-260 (make-bvh-node) and :294-371 (make-bvh-with-sah) build
 * trees whose hit visits both children with the same t-max and keeps the
 * closer record; their closest hit does not depend on the tree's shape (SURVEY
 * App. A Q13-Q15).  The oracle restates an OBJ_BVH as the closest-hit list of
 * its objects (hit-obj-list, geometry.scm:33-50) and, so that a 2^20-curve
 * scene (C5) can be checked at all, evaluates that list through a
 * conservative f64 tree whose result is the list's, tie-breaks included:
 *  - nested lists flatten exactly: a list scanned with the running closest t
 *    is the same scan as its elements spliced in;
 *  - a sphere / moving sphere / curve has a candidate t that does not depend
 *    on the t-max it is asked with, only whether it is reported: spheres
 *    report t < t-max (geometry.scm:157,165), curves t <= t-max (bezier.scm:164
 *    rejects only `(< t (v:z p))`; converge's cull :126 never removes a leaf
 *    hit, which lies in every ancestor's hull);
 *  - a list scan therefore returns the element with the smallest t; among the
 *    elements tied there, the first in list order, unless a later tied one
 *    reports at t == t-max (a curve), in which case the last such.  The
 *    incoming t-max acts as a virtual first element at that t.
 * Trees are built only over lists of spheres, moving spheres and curves (a
 * rect can report t = NaN, Q20, which no tree can order); anything else stays
 * a flat list.  Boxes: sphere c +- |r|; moving sphere the union over the ray
 * times that occur (the camera shutter and 0, Q4); curve = control points +-
 * width/2 (a curve hit lies within width/2 of its hull, bezier.scm:88-98,
 * 159-166).  Every box is padded by 1e-6 x the scene's coordinate bound, far
 * above the rounding of the hit tests (the worst, a near-tangent sphere root,
 * is off by ~3e-8 x the origin distance), so culling is conservative. */
typedef struct { double lo[3], hi[3], c[3]; int obj, order; unsigned char ns; } orc_bprim;

static int bvh_flatten(const orc_scene* s, int id, int** out, int* n, int* cap) {
    const orc_obj* o = &s->obj[id];
    if (o->type == OBJ_LIST || o->type == OBJ_BVH) {
        for (int j = 0; j < o->count; ++j)
            if (!bvh_flatten(s, s->kids[o->first + j], out, n, cap)) return 0;
        return 1;
    }
    if (o->type != OBJ_SPHERE && o->type != OBJ_MOVING_SPHERE && o->type != OBJ_BEZIER) return 0;
    GROW(*out, *n, *cap);
    (*out)[(*n)++] = id;
    return 1;
}

static double fin_abs(double x) { return isfinite(x) ? fabs(x) : 0.0; }

static double sa_of(const double lo[3], const double hi[3]) {
    double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    double a = 2 * (dx * dy + dx * dz + dy * dz);
    return isfinite(a) ? a : 1e300;
}

static int bvh_new_node(orc_bvh* B) {
    GROW(B->node, B->nnode, B->cnode);
    memset(&B->node[B->nnode], 0, sizeof(orc_bnode));
    return B->nnode++;
}

static int cmp_axis;
static int cmp_centroid(const void* a, const void* b) {
    double x = ((const orc_bprim*)a)->c[cmp_axis], y = ((const orc_bprim*)b)->c[cmp_axis];
    return (x < y) ? -1 : (x > y) ? 1 : 0;
}

static int bvh_build(orc_bvh* B, orc_bprim* P, int lo, int hi, int depth) {
    int id = bvh_new_node(B);
    double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = lo; i < hi; ++i)
        for (int a = 0; a < 3; ++a) {
            if (P[i].lo[a] < blo[a]) blo[a] = P[i].lo[a];
            if (P[i].hi[a] > bhi[a]) bhi[a] = P[i].hi[a];
            if (P[i].c[a] < clo[a]) clo[a] = P[i].c[a];
            if (P[i].c[a] > chi[a]) chi[a] = P[i].c[a];
        }
    memcpy(B->node[id].lo, blo, sizeof blo);
    memcpy(B->node[id].hi, bhi, sizeof bhi);
    int n = hi - lo;
    if (n <= 4) {
        B->node[id].first = lo; B->node[id].count = n; B->node[id].left = B->node[id].right = -1;
        return id;
    }
    /* binned SAH over centroids (16 bins per axis); median split as the fallback */
    enum { NB = 16 };
    int best_axis = -1, best_bin = -1;
    double best_cost = INFINITY;
    for (int a = 0; a < 3 && depth < 64; ++a) {
        double ext = chi[a] - clo[a];
        if (!(ext > 0) || !isfinite(ext)) continue;
        int cnt[NB] = {0};
        double bl[NB][3], bh[NB][3];
        for (int k = 0; k < NB; ++k)
            for (int q = 0; q < 3; ++q) { bl[k][q] = INFINITY; bh[k][q] = -INFINITY; }
        for (int i = lo; i < hi; ++i) {
            int k = (int)((P[i].c[a] - clo[a]) / ext * NB);
            k = k < 0 ? 0 : (k >= NB ? NB - 1 : k);
            cnt[k]++;
            for (int q = 0; q < 3; ++q) {
                if (P[i].lo[q] < bl[k][q]) bl[k][q] = P[i].lo[q];
                if (P[i].hi[q] > bh[k][q]) bh[k][q] = P[i].hi[q];
            }
        }
        double rsa[NB]; int rcnt[NB];
        double rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY};
        int rc = 0;
        for (int k = NB - 1; k > 0; --k) {
            rc += cnt[k];
            for (int q = 0; q < 3; ++q) {
                if (bl[k][q] < rl[q]) rl[q] = bl[k][q];
                if (bh[k][q] > rh[q]) rh[q] = bh[k][q];
            }
            rsa[k] = rc ? sa_of(rl, rh) : 0; rcnt[k] = rc;
        }
        double ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
        int lc = 0;
        for (int k = 0; k < NB - 1; ++k) {
            lc += cnt[k];
            for (int q = 0; q < 3; ++q) {
                if (bl[k][q] < ll[q]) ll[q] = bl[k][q];
                if (bh[k][q] > lh[q]) lh[q] = bh[k][q];
            }
            if (!lc || !rcnt[k + 1]) continue;
            double cost = sa_of(ll, lh) * lc + rsa[k + 1] * rcnt[k + 1];
            if (cost < best_cost) { best_cost = cost; best_axis = a; best_bin = k; }
        }
    }
    int mid;
    if (best_axis >= 0) {
        const int a = best_axis;
        const double ext = chi[a] - clo[a];
        int i = lo, j = hi - 1;
        while (i <= j) {
            int k = (int)((P[i].c[a] - clo[a]) / ext * NB);
            k = k < 0 ? 0 : (k >= NB ? NB - 1 : k);
            if (k <= best_bin) { ++i; } else { orc_bprim t = P[i]; P[i] = P[j]; P[j] = t; --j; }
        }
        mid = i;
    } else {
        mid = lo;
    }
    if (mid <= lo || mid >= hi) {            /* no usable SAH split: median on the widest centroid axis */
        int a = 0;
        double w = -1;
        for (int q = 0; q < 3; ++q) {
            double e = chi[q] - clo[q];
            if (isfinite(e) && e > w) { w = e; a = q; }
        }
        cmp_axis = a;
        qsort(P + lo, (size_t)n, sizeof(orc_bprim), cmp_centroid);
        mid = lo + n / 2;
    }
    int l = bvh_build(B, P, lo, mid, depth + 1);
    int r = bvh_build(B, P, mid, hi, depth + 1);
    B->node[id].left = l; B->node[id].right = r; B->node[id].count = 0;
    return id;
}

/* Build every OBJ_BVH's tree (idempotent until the scene or camera changes). */
static void scene_prepare(orc_scene* s) {
    if (s->bvh_ready) return;
    bvh_clear(s);
    s->bvh_of = malloc(sizeof(int) * (size_t)(s->nobj ? s->nobj : 1));
    s->nbvh_of = s->nobj;
    for (int i = 0; i < s->nobj; ++i) s->bvh_of[i] = -1;
    /* coordinate bound of the scene: every ray origin and hit point lies within it */
    double R = fin_abs(s->cam[9]) + fin_abs(s->cam[10]) + fin_abs(s->cam[11]) + fin_abs(s->cam[21]);
    for (int i = 0; i < s->nobj; ++i) {
        const orc_obj* o = &s->obj[i];
        double m = 0, t = 0;
        switch (o->type) {
        case OBJ_SPHERE: m = fmax(fmax(fin_abs(o->c0.x), fin_abs(o->c0.y)), fin_abs(o->c0.z)) + fin_abs(o->r); break;
        case OBJ_MOVING_SPHERE:
            m = fmax(fmax(fmax(fin_abs(o->c0.x), fin_abs(o->c0.y)), fmax(fin_abs(o->c0.z), fin_abs(o->c1.x))),
                     fmax(fin_abs(o->c1.y), fin_abs(o->c1.z))) + fin_abs(o->r);
            break;
        case OBJ_RECT: m = fmax(fmax(fmax(fin_abs(o->a0), fin_abs(o->a1)), fmax(fin_abs(o->b0), fin_abs(o->b1))),
                                fin_abs(o->k)); break;
        case OBJ_BOX: m = fmax(fmax(fmax(fin_abs(o->c0.x), fin_abs(o->c0.y)), fin_abs(o->c0.z)),
                               fmax(fmax(fin_abs(o->c1.x), fin_abs(o->c1.y)), fin_abs(o->c1.z))); break;
        case OBJ_TRANSLATE: t = fin_abs(o->c0.x) + fin_abs(o->c0.y) + fin_abs(o->c0.z); break;
        case OBJ_BEZIER:
            for (int k = 0; k < 4; ++k)
                m = fmax(m, fmax(fmax(fin_abs(o->cp[k].x), fin_abs(o->cp[k].y)), fin_abs(o->cp[k].z)));
            m += fin_abs(o->width);
            break;
        default: break;
        }
        if (m > R) R = m;
        R += t;                               /* instance offsets move geometry outward */
    }
    const double pad = 1e-6 * fmax(R, 1e4);
    double tlo = 0, thi = 0;                  /* ray times: the shutter and 0 */
    if (isfinite(s->cam[22])) { tlo = fmin(tlo, s->cam[22]); thi = fmax(thi, s->cam[22]); }
    if (isfinite(s->cam[23])) { tlo = fmin(tlo, s->cam[23]); thi = fmax(thi, s->cam[23]); }
    int* ids = 0; int cap = 0;
    for (int i = 0; i < s->nobj; ++i) {
        if (s->obj[i].type != OBJ_BVH) continue;
        int n = 0;
        if (!bvh_flatten(s, i, &ids, &n, &cap) || n < 8) continue;
        orc_bprim* P = malloc(sizeof(orc_bprim) * (size_t)n);
        for (int j = 0; j < n; ++j) {
            const orc_obj* o = &s->obj[ids[j]];
            double lo[3], hi[3];
            if (o->type == OBJ_SPHERE) {
                double c[3] = {o->c0.x, o->c0.y, o->c0.z}, rr = fabs(o->r);
                for (int a = 0; a < 3; ++a) { lo[a] = c[a] - rr; hi[a] = c[a] + rr; }
            } else if (o->type == OBJ_MOVING_SPHERE) {
                double rr = fabs(o->r);
                double ts[2] = {tlo, thi};
                for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
                for (int k = 0; k < 2; ++k) {
                    v3 c = vadd(o->c0, vscale(vsub(o->c1, o->c0), (ts[k] - o->t0) / (o->t1 - o->t0)));
                    double cc[3] = {c.x, c.y, c.z};
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = fmin(lo[a], cc[a] - rr); hi[a] = fmax(hi[a], cc[a] + rr);
                    }
                }
            } else {
                double w = fabs(o->width) / 2;
                for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
                for (int k = 0; k < 4; ++k) {
                    double cc[3] = {o->cp[k].x, o->cp[k].y, o->cp[k].z};
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = fmin(lo[a], cc[a] - w); hi[a] = fmax(hi[a], cc[a] + w);
                    }
                }
            }
            for (int a = 0; a < 3; ++a) {
                if (!isfinite(lo[a]) || !isfinite(hi[a])) { lo[a] = -INFINITY; hi[a] = INFINITY; }
                else { lo[a] -= pad; hi[a] += pad; }
                P[j].lo[a] = lo[a]; P[j].hi[a] = hi[a];
                P[j].c[a] = isfinite(lo[a]) ? 0.5 * (lo[a] + hi[a]) : 0.0;
            }
            P[j].obj = ids[j]; P[j].order = j; P[j].ns = (o->type == OBJ_BEZIER);
        }
        s->bvh = realloc(s->bvh, sizeof(orc_bvh) * (size_t)(s->nbvh + 1));
        orc_bvh* B = &s->bvh[s->nbvh];
        memset(B, 0, sizeof *B);
        bvh_build(B, P, 0, n, 0);
        B->nprim = n;
        B->prim = malloc(sizeof(int) * (size_t)n);
        B->order = malloc(sizeof(int) * (size_t)n);
        B->nonstrict = malloc((size_t)n);
        for (int j = 0; j < n; ++j) { B->prim[j] = P[j].obj; B->order[j] = P[j].order; B->nonstrict[j] = P[j].ns; }
        free(P);
        s->bvh_of[i] = s->nbvh++;
    }
    free(ids);
    s->bvh_ready = 1;
}

/* Slab test of a padded box against [0, cut] along the raw ray (geometry.scm:
 * 73-105 tests each axis against the original interval; intersecting the axes
 * as done here only culls more, and only boxes the ray cannot reach). */
static int bvh_slab(const orc_bnode* nd, const double o[3], const double d[3], const double inv[3], double cut,
                    double* tnear) {
    double t0 = -INFINITY, t1 = INFINITY;
    for (int a = 0; a < 3; ++a) {
        if (d[a] == 0) {
            if (o[a] < nd->lo[a] || o[a] > nd->hi[a]) return 0;
            continue;
        }
        double ta = (nd->lo[a] - o[a]) * inv[a], tb = (nd->hi[a] - o[a]) * inv[a];
        if (ta > tb) { double t = ta; ta = tb; tb = t; }
        /* the padding covers the rounding for origins near the scene; a ray may start anywhere (a curve
         * reports its hit off the ribbon for |dir| != 1, Q10): widen by the origin's own share */
        const double e = 0x1p-40 * fabs(o[a] * inv[a]);
        ta -= e; tb += e;
        if (ta > t0) t0 = ta;
        if (tb < t1) t1 = tb;
    }
    if (t0 > t1 || t1 < 0 || t0 > cut) return 0;
    *tnear = t0;
    return 1;
}

static int prim_hit(const orc_scene* s, int id, ray_t r, double tmin, double tmax, hitrec* rec);

static int bvh_hit(const orc_scene* s, const orc_bvh* B, const orc_obj* flat, ray_t r, double tmin, double tmax,
                   hitrec* rec) {
    const double dl = vlength(r.d);
    /* a curve reports distance along unit(dir) (Q10): raw parameter = t / |dir| */
    const double scale = (dl < 1) ? 1 / dl : 1;
    if (!(scale < INFINITY) || B->nnode == 0) return hit_list(s, flat->first, flat->count, r, tmin, tmax, rec);
    const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    const double inv[3] = {1 / d[0], 1 / d[1], 1 / d[2]};
    double best = tmax;
    int first = -1, ns = -1, first_ns = 0;   /* first = -1: the virtual element at t-max */
    hitrec first_rec, ns_rec, h;
    int stack[256], sp = 0;
    double tn;
    if (!bvh_slab(&B->node[0], o, d, inv, best * scale * (1 + 1e-12), &tn)) return 0;
    stack[sp++] = 0;
    while (sp) {
        const orc_bnode* nd = &B->node[stack[--sp]];
        const double cut = best * scale * (1 + 1e-12);
        if (nd->count) {
            for (int k = nd->first; k < nd->first + nd->count; ++k) {
                if (!prim_hit(s, B->prim[k], r, tmin, nextafter(best, INFINITY), &h)) continue;
                const int idx = B->order[k], hns = B->nonstrict[k];
                if (h.t < best) {
                    best = h.t; first = idx; first_rec = h; first_ns = hns; ns = -1;
                } else if (h.t == best) {
                    if (idx < first) {                  /* the displaced first is a later tied element */
                        if (first_ns && first >= 0 && first > ns) { ns = first; ns_rec = first_rec; }
                        first = idx; first_rec = h; first_ns = hns;
                    } else if (hns && idx > ns) {
                        ns = idx; ns_rec = h;
                    }
                }
            }
            continue;
        }
        double tl, tr;
        int hl = bvh_slab(&B->node[nd->left], o, d, inv, cut, &tl);
        int hr = bvh_slab(&B->node[nd->right], o, d, inv, cut, &tr);
        if (hl && hr) {
            if (tl <= tr) { stack[sp++] = nd->right; stack[sp++] = nd->left; }
            else { stack[sp++] = nd->left; stack[sp++] = nd->right; }
        } else if (hl) {
            stack[sp++] = nd->left;
        } else if (hr) {
            stack[sp++] = nd->right;
        }
    }
    if (ns >= 0 && ns > first) { *rec = ns_rec; return 1; }
    if (first >= 0) { *rec = first_rec; return 1; }
    return 0;
}

static int hit_obj(const orc_scene* s, int id, ray_t r, double tmin, double tmax, hitrec* rec) {
    const orc_obj* o = &s->obj[id];
    switch (o->type) {
    case OBJ_SPHERE: return sphere_hit(o->c0, o->r, o->mat, r, tmin, tmax, rec);
    case OBJ_MOVING_SPHERE: {                                           /* :177-208 */
        v3 center = vadd(o->c0, vscale(vsub(o->c1, o->c0), (r.time - o->t0) / (o->t1 - o->t0)));
        return sphere_hit(center, o->r, o->mat, r, tmin, tmax, rec);
    }
    case OBJ_RECT: return rect_hit(o, r, tmin, tmax, rec);
    case OBJ_FLIP:                                                      /* :433-442 */
        if (!hit_obj(s, o->child, r, tmin, tmax, rec)) return 0;
        rec->n = vscale(rec->n, -1);
        return 1;
    case OBJ_BOX: {                                                     /* :444-463 */
        const orc_obj* l = &s->obj[o->box_list];
        return hit_list(s, l->first, l->count, r, tmin, tmax, rec);
    }
    case OBJ_TRANSLATE: {                                               /* :465-481 */
        ray_t moved = {vsub(r.o, o->c0), r.d, r.time};
        if (!hit_obj(s, o->child, moved, tmin, tmax, rec)) return 0;
        rec->p = vadd(rec->p, o->c0);
        return 1;
    }
    case OBJ_ROTATE_Y: {                                                /* :511-540 */
        double sn = o->sin_t, cs = o->cos_t;
        ray_t rr;
        rr.o = V(cs * r.o.x - sn * r.o.z, r.o.y, sn * r.o.x + cs * r.o.z);
        rr.d = V(cs * r.d.x - sn * r.d.z, r.d.y, sn * r.d.x + cs * r.d.z);
        rr.time = r.time;
        if (!hit_obj(s, o->child, rr, tmin, tmax, rec)) return 0;
        v3 p = V(cs * rec->p.x + sn * rec->p.z, rec->p.y, (-sn) * rec->p.x + cs * rec->p.z);
        v3 n = V(cs * rec->n.x + sn * rec->n.z, rec->n.y, (-sn) * rec->n.x + cs * rec->n.z);
        rec->p = p; rec->n = n; rec->mat = o->mat;
        return 1;
    }
    case OBJ_LIST:
        return hit_list(s, o->first, o->count, r, tmin, tmax, rec);
    case OBJ_BVH:
        if (!s->bvh_flat && id < s->nbvh_of && s->bvh_of[id] >= 0)
            return bvh_hit(s, &s->bvh[s->bvh_of[id]], o, r, tmin, tmax, rec);
        return hit_list(s, o->first, o->count, r, tmin, tmax, rec);
    case OBJ_BEZIER:
        return bezier_hit(o, r, tmin, tmax, rec);
    case OBJ_KLEIN:
        return klein_hit(o, r, tmin, tmax, rec);
    case OBJ_MEDIUM: {                                                  /* :545-578 */
        hitrec r1, r2;
        if (!hit_obj(s, o->child, r, -ORC_TMAX, ORC_TMAX, &r1)) return 0;
        if (!hit_obj(s, o->child, r, r1.t + 0.0001, ORC_TMAX, &r2)) return 0;
        double t1 = (r1.t < tmin) ? tmin : r1.t;
        double t2 = (r2.t > tmax) ? tmax : r2.t;
        if (t1 >= t2) return 0;
        if (t1 < 0) t1 = 0;
        double inside = (t2 - t1) * vlength(r.d);
        if (!tl_rng) return 0;                    /* hit_world KATs: no path stream */
        double hd = (-(1 / o->density)) * log(orc_random_real(tl_rng));
        if (!(hd < inside)) return 0;
        double nt = t1 + hd / vlength(r.d);
        rec->t = nt;
        rec->p = point_at(r, nt);
        rec->n = V(1, 0, 0);
        rec->mat = o->mat;
        rec->u = 0; rec->v = 0;
        return 1;
    }
    }
    return 0;
}

static int prim_hit(const orc_scene* s, int id, ray_t r, double tmin, double tmax, hitrec* rec) {
    return hit_obj(s, id, r, tmin, tmax, rec);
}

/* ---------------------------------------------------------- material.scm */
static v3 reflect(v3 v, v3 n) { return vsub(v, vscale(n, 2 * vdot(v, n))); }  /* :41-43 */
static double schlick(double cosine, double ref_idx) {                         /* :69-74 */
    double r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1 - r0) * pow(1 - cosine, 5);
}
static int refract(v3 v, v3 n, double ni_over_nt, v3* out) {                   /* :59-67 */
    v3 uv = vunit(v);
    double dt = vdot(uv, n);
    double disc = 1 - ni_over_nt * ni_over_nt * (1 - dt * dt);
    if (disc > 0) {
        *out = vsub(vscale(vsub(v, vscale(n, dt)), ni_over_nt), vscale(n, sqrt(disc)));
        return 1;
    }
    return 0;
}

/* exported KAT helpers */
double orc_schlick(double c, double r) { return schlick(c, r); }
int orc_refract(const double v[3], const double n[3], double ni, double out[3]) {
    v3 o;
    int ok = refract(V(v[0], v[1], v[2]), V(n[0], n[1], n[2]), ni, &o);
    if (ok) { out[0] = o.x; out[1] = o.y; out[2] = o.z; }
    return ok;
}
void orc_reflect(const double v[3], const double n[3], double out[3]) {
    v3 o = reflect(V(v[0], v[1], v[2]), V(n[0], n[1], n[2]));
    out[0] = o.x; out[1] = o.y; out[2] = o.z;
}
double orc_noise(const orc_scene* s, const double p[3]) { return perlin_noise(s, V(p[0], p[1], p[2])); }
double orc_turb(const orc_scene* s, const double p[3]) { return perlin_turb(s, V(p[0], p[1], p[2])); }
void orc_tex_value(const orc_scene* s, int tex, const double p[3], double out[3]) {
    v3 c = tex_value(s, tex, 0, 0, V(p[0], p[1], p[2]));
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
void orc_onb(const double n[3], double out[9]) {
    onb_t b = make_onb_from_w(V(n[0], n[1], n[2]));
    out[0] = b.u.x; out[1] = b.u.y; out[2] = b.u.z;
    out[3] = b.v.x; out[4] = b.v.y; out[5] = b.v.z;
    out[6] = b.w.x; out[7] = b.w.y; out[8] = b.w.z;
}
/* closest hit of the world list: returns 1 on hit, rec = {t, p(3), n(3), mat} */
int orc_hit_world(const orc_scene* s, const double o[3], const double d[3], double time, double out[8]) {
    scene_prepare((orc_scene*)s);
    ray_t r = {V(o[0], o[1], o[2]), V(d[0], d[1], d[2]), time};
    hitrec rec;
    const orc_obj* w = &s->obj[s->world];
    if (!hit_list(s, w->first, w->count, r, ORC_TMIN, ORC_TMAX, &rec)) return 0;
    out[0] = rec.t; out[1] = rec.p.x; out[2] = rec.p.y; out[3] = rec.p.z;
    out[4] = rec.n.x; out[5] = rec.n.y; out[6] = rec.n.z; out[7] = rec.mat;
    return 1;
}

/* -------------------------------------------------------------- main.scm */
static v3 sky(const orc_scene* s, ray_t r) {
    if (s->sky == 1) return V(0, 0, 0);                                 /* black :97-98 */
    v3 unit_dir = vunit(r.d);                                           /* sky-color :91-95 */
    double t = 0.5 * (1.0 + unit_dir.y);
    return vadd(vscale(V(1, 1, 1), 1 - t), vscale(V(0.5, 0.7, 1.0), t));
}

/* ------------------------------------------- pdf.scm light sampling (f2)
 * pdf.scm (make-cosine-pdf :18-26, make-hitable-pdf :28-32, make-mixture-pdf
 * :34-41) calls g:pdf-value / g:random, which geometry.scm never defines, and
 * main.scm never wires the pdfs into `color`.  This extension defines them as
 * "The Rest of Your Life" does, for an axis rect or a sphere, and uses the
 * mixture (light, cosine) for lambertian bounces.  Scheme semantics are kept:
 * onb `local` is the syntax-rules macro, so a sampler passed to it runs three
 * times (Q29).  Not pinned against the reference (it has no such path). */
static const orc_obj* light_obj(const orc_scene* s) {
    const orc_obj* o = &s->obj[s->light];
    while (o->type == OBJ_FLIP) o = &s->obj[o->child];
    return o;
}
/* g:pdf-value: density of direction v from origin o */
static double light_pdf_value(const orc_scene* s, v3 o, v3 v) {
    const orc_obj* L = light_obj(s);
    hitrec rec;
    ray_t r = {o, v, 0.0};
    if (L->type == OBJ_RECT) {
        if (!rect_hit(L, r, ORC_TMIN, ORC_TMAX, &rec)) return 0;
        double area = (L->a1 - L->a0) * (L->b1 - L->b0);
        double distance_squared = rec.t * rec.t * vdot(v, v);
        double cosine = fabs(vdot(v, rec.n) / vlength(v));
        return distance_squared / (cosine * area);
    }
    if (!sphere_hit(L->c0, L->r, L->mat, r, ORC_TMIN, ORC_TMAX, &rec)) return 0;
    v3 oc = vsub(L->c0, o);
    double cos_theta_max = sqrt(1 - L->r * L->r / vdot(oc, oc));
    double solid_angle = 2 * ORC_PI * (1 - cos_theta_max);
    return 1 / solid_angle;
}
static v3 random_to_sphere(double radius, double distance_squared, orc_rng* g) {
    double r1 = orc_random_real(g);
    double r2 = orc_random_real(g);
    double z = 1 + r2 * (sqrt(1 - radius * radius / distance_squared) - 1);
    double phi = 2 * ORC_PI * r1;
    double x = cos(phi) * sqrt(1 - z * z);
    double y = sin(phi) * sqrt(1 - z * z);
    return V(x, y, z);
}
/* g:random: a direction from o toward the light */
static v3 light_random(const orc_scene* s, v3 o, orc_rng* g) {
    const orc_obj* L = light_obj(s);
    if (L->type == OBJ_RECT) {
        double a = L->a0 + orc_random_real(g) * (L->a1 - L->a0);
        double b = L->b0 + orc_random_real(g) * (L->b1 - L->b0);
        v3 pnt = (L->axis == 0) ? V(a, b, L->k) : (L->axis == 1) ? V(a, L->k, b) : V(L->k, a, b);
        return vsub(pnt, o);
    }
    v3 direction = vsub(L->c0, o);
    double distance_squared = vdot(direction, direction);
    onb_t uvw = make_onb_from_w(direction);
    double x = random_to_sphere(L->r, distance_squared, g).x;       /* local: three evaluations (Q29) */
    double y = random_to_sphere(L->r, distance_squared, g).y;
    double z = random_to_sphere(L->r, distance_squared, g).z;
    return onb_local(uvw, V(x, y, z));
}
/* make-cosine-pdf's value (pdf.scm:19-23) */
static double cosine_pdf_value(onb_t uvw, v3 dir) {
    double cosine = vdot(vunit(dir), uvw.w);
    return (cosine > 0) ? cosine / ORC_PI : 0;
}
double orc_light_pdf_value(const orc_scene* s, const double o[3], const double v[3]) {
    return light_pdf_value(s, V(o[0], o[1], o[2]), V(v[0], v[1], v[2]));
}

typedef struct { uint64_t segments; int max_depth; } orc_counters;

/* main.scm:100-121 — recursive colour */
/* debugging aid (orc_trace_sample): per segment o, d, hit?, t, p, mat, draw counter */
static __thread double* tl_trace;
static __thread int tl_trace_n, tl_trace_cap;

static v3 color(const orc_scene* s, ray_t r, int depth, orc_rng* g, orc_counters* cnt) {
    hitrec rec;
    const orc_obj* w = &s->obj[s->world];
    cnt->segments++;
    if (depth > cnt->max_depth) cnt->max_depth = depth;
    tl_rng = g;
    int hit = hit_list(s, w->first, w->count, r, ORC_TMIN, ORC_TMAX, &rec);
    tl_rng = 0;
    if (tl_trace && tl_trace_n < tl_trace_cap) {
        double* q = tl_trace + 13 * tl_trace_n++;
        q[0] = r.o.x; q[1] = r.o.y; q[2] = r.o.z; q[3] = r.d.x; q[4] = r.d.y; q[5] = r.d.z;
        q[6] = hit; q[7] = hit ? rec.t : 0; q[8] = hit ? rec.p.x : 0; q[9] = hit ? rec.p.y : 0;
        q[10] = hit ? rec.p.z : 0; q[11] = hit ? rec.mat : -1; q[12] = g->ctr;
    }
    if (!hit) return sky(s, r);
    const orc_mat* m = &s->mat[rec.mat];
    switch (m->type) {
    case MAT_LAMBERTIAN: {                                              /* material.scm:24-39 */
        if (s->light >= 0) {
            /* mixture of (hitable-pdf light p) and (cosine-pdf normal), pdf.scm:34-41 */
            onb_t uvw = make_onb_from_w(rec.n);
            v3 dir;
            if (orc_random_real(g) < 0.5) {
                dir = light_random(s, rec.p, g);
            } else {
                double cx = random_cosine_direction(g).x;
                double cy = random_cosine_direction(g).y;
                double cz = random_cosine_direction(g).z;
                dir = onb_local(uvw, V(cx, cy, cz));
            }
            ray_t scattered = {rec.p, dir, 0.0};
            double pdf_val = 0.5 * light_pdf_value(s, rec.p, dir) + 0.5 * cosine_pdf_value(uvw, dir);
            /* a direction neither pdf can produce (a light sample that grazes
             * past the light, below the surface) ends the path: no 0 * inf */
            if (!(pdf_val > 0)) return V(0, 0, 0);
            v3 att = tex_value(s, m->tex, 0, 0, rec.p);
            if (depth < ORC_MAX_DEPTH) {
                double cosine = vdot(rec.n, vunit(scattered.d));
                if (cosine < 0) cosine = 0;
                double spdf = cosine / ORC_PI;
                v3 L = color(s, scattered, depth + 1, g, cnt);
                return vadd(V(0, 0, 0), vscale(vmul(vscale(att, spdf), L), 1 / pdf_val));
            }
            return V(0, 0, 0);
        }
        onb_t uvw = make_onb_from_w(rec.n);
        /* (local uvw (random-cosine-direction)) — `local` is a syntax-rules
         * macro (onb.scm:27-36) that substitutes its argument EXPRESSION into
         * (v:x a), (v:y a) and (v:z a): random-cosine-direction runs three
         * times, left to right, and each call contributes one component (Q29). */
        double cx = random_cosine_direction(g).x;
        double cy = random_cosine_direction(g).y;
        double cz = random_cosine_direction(g).z;
        v3 target = onb_local(uvw, V(cx, cy, cz));
        ray_t scattered = {rec.p, vunit(target), 0.0};
        v3 att = tex_value(s, m->tex, 0, 0, rec.p);
        double pdf = vdot(uvw.w, scattered.d) / ORC_PI;
        if (depth < ORC_MAX_DEPTH) {
            double cosine = vdot(rec.n, vunit(scattered.d));
            if (cosine < 0) cosine = 0;
            double spdf = cosine / ORC_PI;
            v3 L = color(s, scattered, depth + 1, g, cnt);
            /* emitted (0,0,0) + ((att*spdf) (*) L) * (1/pdf) */
            return vadd(V(0, 0, 0), vscale(vmul(vscale(att, spdf), L), 1 / pdf));
        }
        return V(0, 0, 0);
    }
    case MAT_METAL: {                                                   /* material.scm:45-57 (R2) */
        v3 reflected = reflect(vunit(r.d), rec.n);
        v3 dir = vadd(reflected, vscale(random_in_unit_sphere(g), m->fuzz));
        int valid = vdot(dir, rec.n) > 0;
        v3 att = tex_value(s, m->tex, 0, 0, rec.p);
        if (depth < ORC_MAX_DEPTH && valid) {
            ray_t scattered = {rec.p, dir, 0.0};
            return vmul(att, color(s, scattered, depth + 1, g, cnt));
        }
        return V(0, 0, 0);
    }
    case MAT_DIELECTRIC: {                                              /* material.scm:76-101 (R2) */
        double ref_idx = m->ref_idx;
        v3 reflected = reflect(r.d, rec.n);
        double dd = vdot(r.d, rec.n);
        v3 outward = (dd > 0) ? vscale(rec.n, -1) : rec.n;
        double ni = (dd > 0) ? ref_idx : 1 / ref_idx;
        double cosine = (dd > 0) ? (dd * ref_idx) / vlength(r.d) : (-dd) / vlength(r.d);
        v3 refracted;
        int ok = refract(r.d, outward, ni, &refracted);
        double reflect_prob = ok ? schlick(cosine, ref_idx) : 1;
        ray_t scattered;
        scattered.o = rec.p; scattered.time = 0.0;
        scattered.d = (orc_random_real(g) < reflect_prob) ? reflected : refracted;
        if (depth < ORC_MAX_DEPTH) return vmul(V(1, 1, 1), color(s, scattered, depth + 1, g, cnt));
        return V(0, 0, 0);
    }
    case MAT_DIFFUSE_LIGHT:                                             /* material.scm:103-111 */
        if (vdot(rec.n, r.d) < 0.0) return tex_value(s, m->tex, rec.u, rec.v, rec.p);
        return V(0, 0, 0);
    }
    return V(0, 0, 0);
}

/* camera.scm:80-92 — get-ray */
static ray_t get_ray(const double* cam, double s_, double t_, orc_rng* g) {
    v3 llc = V(cam[0], cam[1], cam[2]), hor = V(cam[3], cam[4], cam[5]), ver = V(cam[6], cam[7], cam[8]);
    v3 origin = V(cam[9], cam[10], cam[11]);
    v3 u = V(cam[15], cam[16], cam[17]), v = V(cam[18], cam[19], cam[20]);
    double lens = cam[21], t0 = cam[22], t1 = cam[23];
    v3 rd = vscale(random_in_unit_disk(g), lens);
    v3 offset = vadd(vscale(u, rd.x), vscale(v, rd.y));
    double time = t0 + orc_random_real(g) * (t1 - t0);
    ray_t r;
    r.o = vadd(origin, offset);
    r.d = vsub(vsub(vadd(vadd(llc, vscale(hor, s_)), vscale(ver, t_)), origin), offset);
    r.time = time;
    return r;
}

/* One camera sample of pixel (x, y), sample index smp (0-based pass index):
 * the body of trace-all (main.scm:476-479). */
static v3 sample_pixel(const orc_scene* s, int nx, int ny, int x, int y, uint64_t seed, uint32_t smp,
                       orc_counters* cnt) {
    orc_rng g = {(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)(y * nx + x), smp, 0};
    double u = (x + orc_random_real(&g)) / nx;
    double v = (y + orc_random_real(&g)) / ny;
    ray_t r = get_ray(s->cam, u, v, &g);
    return color(s, r, 0, &g, cnt);
}

void orc_sample(const orc_scene* s, int nx, int ny, int x, int y, uint64_t seed, uint32_t smp,
                double out[3]) {
    scene_prepare((orc_scene*)s);
    orc_counters cnt = {0, 0};
    v3 c = sample_pixel(s, nx, ny, x, y, seed, smp, &cnt);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}

/* Render pixels [pix_begin, pix_end) of an nx*ny image, passes spp_begin ..
 * spp_begin+spp_count-1, adding each sample colour to accum in sample order
 * (the *raw-data* running sum, main.scm:480,488).  nthreads > 1 uses OpenMP
 * over pixels (pixels are independent; per-pixel order is preserved).
 * Returns the number of ray segments (closest-hit queries). */
uint64_t orc_render(const orc_scene* s, int nx, int ny, int spp_begin, int spp_count, uint64_t seed,
                    double* accum, long pix_begin, long pix_end, int nthreads) {
    uint64_t total = 0;
    scene_prepare((orc_scene*)s);
    if (pix_end < 0 || pix_end > (long)nx * ny) pix_end = (long)nx * ny;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total)
#endif
    for (long j = pix_begin; j < pix_end; ++j) {
        int x = (int)(j % nx), y = (int)(j / nx);
        orc_counters cnt = {0, 0};
        double r = accum[3 * j], gg = accum[3 * j + 1], b = accum[3 * j + 2];
        for (int k = 0; k < spp_count; ++k) {
            v3 c = sample_pixel(s, nx, ny, x, y, seed, (uint32_t)(spp_begin + k), &cnt);
            r = r + c.x; gg = gg + c.y; b = b + c.z;
        }
        accum[3 * j] = r; accum[3 * j + 1] = gg; accum[3 * j + 2] = b;
        total += cnt.segments;
    }
    (void)nthreads;
    return total;
}

/* Same as orc_render for an explicit pixel list (multi-rank tests). */
uint64_t orc_render_pixels(const orc_scene* s, int nx, int ny, int spp_begin, int spp_count, uint64_t seed,
                           double* accum, const uint32_t* pix, long npix, int nthreads) {
    uint64_t total = 0;
    scene_prepare((orc_scene*)s);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total)
#endif
    for (long q = 0; q < npix; ++q) {
        const long j = pix[q];
        int x = (int)(j % nx), y = (int)(j / nx);
        orc_counters cnt = {0, 0};
        double r = accum[3 * j], gg = accum[3 * j + 1], b = accum[3 * j + 2];
        for (int k = 0; k < spp_count; ++k) {
            v3 c = sample_pixel(s, nx, ny, x, y, seed, (uint32_t)(spp_begin + k), &cnt);
            r = r + c.x; gg = gg + c.y; b = b + c.z;
        }
        accum[3 * j] = r; accum[3 * j + 1] = gg; accum[3 * j + 2] = b;
        total += cnt.segments;
    }
    (void)nthreads;
    return total;
}

/* debugging aid: one sample's path, 13 doubles per segment (see color()); returns the segment count */
int orc_trace_sample(const orc_scene* s, int nx, int ny, int x, int y, uint64_t seed, uint32_t smp, double* out,
                     int cap) {
    scene_prepare((orc_scene*)s);
    orc_counters cnt = {0, 0};
    tl_trace = out; tl_trace_n = 0; tl_trace_cap = cap;
    (void)sample_pixel(s, nx, ny, x, y, seed, smp, &cnt);
    tl_trace = 0;
    return tl_trace_n;
}

/* exported KAT helper: util.scm:37-44 with given (r1, r2) */
void orc_cosine_direction(double r1, double r2, double out[3]) {
    double z = sqrt(1 - r2);
    double phi = 2 * ORC_PI * r1;
    out[0] = cos(phi) * 2 * sqrt(r2);
    out[1] = sin(phi) * 2 * sqrt(r2);
    out[2] = z;
}

/* main.scm:481-491 — correct-gamma of sum/count, then floor(255.99*min(1,c)) */
void orc_resolve_u8(const double* accum, long npix, int count, uint8_t* out) {
    for (long i = 0; i < 3 * npix; ++i) {
        double c = sqrt(accum[i] / count);
        double m = (1 < c) ? 1.0 : c;
        out[i] = (uint8_t)floor(255.99 * m);
    }
}
