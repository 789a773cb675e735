/*
 * rt.h — C ABI of the MI355X wavefront path tracer (librtamd.so).
 *
 * This is the drop-in boundary for the reference's hot path: the per-pixel
 * `trace-all` → recursive `color` loop of soma-arc/scheme-raytrace
 * (main.scm:100-121, 471-491) and everything it calls through the
 * closure-vector protocol (geometry.scm:14-15, material.scm:15-22,
 * texture.scm:9-10).  Scheme closures are opaque to C, so the drop-in keeps
 * the reference's *constructor* names and arities and has each constructor
 * append a typed descriptor to a scene builder.
 *
 * Conventions
 *   - every entry point returns an int status: 0 = ok, nonzero = error, with
 *     a thread-local message from rt_last_error();
 *   - handles (contexts, scenes, object/material/texture ids) are ints;
 *   - the caller owns every host buffer; the library copies descriptors at
 *     commit time and owns all device memory it allocates;
 *   - vectors are `const double v[3]` (the reference's f64vector vec3,
 *     vec.scm:7);
 *   - one host thread per context (the reference renders on one thread,
 *     main.scm:633-634); multi-GPU = one process per GPU.
 *   - arithmetic is f64 throughout, as in the reference (Gauche flonums).
 */
#ifndef RTAMD_RT_H
#define RTAMD_RT_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 7

/* Sky functions (scene slot 4, geometry.scm:30-31).  The reference stores an
 * arbitrary closure; the two it defines are sky-color (main.scm:91-95) and
 * black (main.scm:97-98). */
enum { RT_SKY_GRADIENT = 0, RT_SKY_BLACK = 1 };

/* Axis-aligned rect planes (geometry.scm:376-431). */
enum { RT_RECT_XY = 0, RT_RECT_XZ = 1, RT_RECT_YZ = 2 };

/* Number of doubles in a camera vector: the reference's 10-slot camera
 * (camera.scm:33-78) flattened = llc(3) horizontal(3) vertical(3) origin(3)
 * w(3) u(3) v(3) lens-radius time0 time1. */
#define RT_CAMERA_DOUBLES 24

/* ---- library / context ------------------------------------------------ */
int rt_abi_version(void);
const char* rt_last_error(void);
int rt_device_count(int* out_count);
/* Context on one HIP device; owns a HIP stream and all device memory.
 * The render lanes' path pools belong to the context and are shared by every
 * scene rendered on it.  They are sized at the context's first render to
 * hold up to 384Mi paths, but at most 65 % of the device memory free at that
 * moment (RT_OPT_MAX_PATHS overrides), and are kept for later renders;
 * rt_context_release_pools frees them (the next render sizes them again),
 * e.g. before the caller allocates large buffers of its own. */
int rt_context_create(int device, int* out_ctx);
int rt_context_destroy(int ctx);
int rt_context_release_pools(int ctx);

/* Render-schedule options of a context (every scene rendered on it).  Value 0
 * = the library's automatic choice (the default); negative values are refused.
 * None of them changes an image: renders are bit-identical for any lane count,
 * pool size and tail threshold (per-sample counter RNG, sample-ordered
 * accumulation).
 *   RT_OPT_LANES      render lanes (path pool + stream) kept in flight, 1..4;
 *                     auto = 2, or 1 for scenes whose world BVH holds curves
 *                     (the persistent curve kernel fills the chip by itself);
 *                     raising it above the lanes the pools were sized for
 *                     sizes them again at the next render, lowering it keeps
 *                     the pools as they are (each lane then holds the smaller
 *                     per-lane share of the larger count; RT_OPT_MAX_PATHS or
 *                     rt_context_release_pools resizes them)
 *   RT_OPT_MAX_PATHS  paths per pool (chunk of samples), >= 1024; auto = 384Mi,
 *                     at most 65 % of free device memory for the lanes together
 *                     (setting it makes the next render size the pools again)
 *   RT_OPT_TAIL_PATHS a chunk with at most max(TAIL_PATHS, B / TAIL_DIV) live
 *   RT_OPT_TAIL_DIV   paths (B = the chunk's camera samples) finishes in the
 *                     persistent tail kernel; with neither set the threshold
 *                     follows the render: one chunk max(32768,
 *                     min(B / 4, 524288), B / 256), else
 *                     max(32768, min(B / 64, 262144), B / 256) (curve-kernel
 *                     scenes: max(32768, B / 256)); either set: the other's
 *                     auto value is 32768 / 256
 *   RT_OPT_TAIL_OFF   nonzero: no tail kernel, every depth in the wavefront
 *                     kernels (tests and A/B runs)
 * One option selects arithmetic, not the schedule:
 *   RT_OPT_EXACT_LIBM the sin / cos of the lambertian bounce directions
 *                     (random-cosine-direction, util.scm:37-44, and the light
 *                     mixture's sphere sampler): RT_LIBM_EXACT = the reference
 *                     runtime's C library bit for bit (glibc's algorithm,
 *                     restated on the device), RT_LIBM_DEVICE = the device
 *                     library (within 1 ulp, ~1.4 % faster on the cover scene),
 *                     RT_LIBM_AUTO (0) = exact in scenes with curves (where an
 *                     ulp of a bounce direction changes which ribbon a grazing
 *                     ray hits) or noise / marble textures (C3: 0.8 % of the
 *                     horizon rows' pixels moved by > 1e-9 otherwise; exact
 *                     costs it 1.7 %), the device library elsewhere (the cover
 *                     scene: 0.3 % of those pixels, exact would cost 1.4 %).
 *                     The marble texture's sin is exact in every mode. */
enum { RT_OPT_LANES = 1, RT_OPT_MAX_PATHS = 2, RT_OPT_TAIL_PATHS = 3, RT_OPT_TAIL_DIV = 4, RT_OPT_TAIL_OFF = 5,
       RT_OPT_EXACT_LIBM = 6 };
enum { RT_LIBM_AUTO = 0, RT_LIBM_EXACT = 1, RT_LIBM_DEVICE = 2 };
int rt_context_set_option(int ctx, int option, int64_t value);
int rt_context_get_option(int ctx, int option, int64_t* out_value);

/* ---- scene building (replaces the closure-vector constructors) ---------- */
int rt_scene_begin(int ctx, int* out_scene);
int rt_scene_destroy(int scene);

/* textures — texture.scm:12-34 */
int rt_add_texture_constant(int scene, const double rgb[3], int* out_tex);     /* t:constant-texture :12 */
int rt_add_texture_checker(int scene, int even_tex, int odd_tex, int* out_tex); /* t:checker-texture :16 */
int rt_add_texture_noise(int scene, double scale, int* out_tex);               /* t:noise-texture :25 */
int rt_add_texture_marble(int scene, double scale, int* out_tex);              /* t:marble-texture :30 */

/* materials — material.scm:24-111 */
int rt_add_material_lambertian(int scene, int albedo_tex, int* out_mat);            /* m:make-lambertian :24 */
int rt_add_material_metal(int scene, int albedo_tex, double fuzz, int* out_mat);    /* m:make-metal :45 */
int rt_add_material_dielectric(int scene, double ref_idx, int* out_mat);            /* m:make-dielectric :76 */
int rt_add_material_diffuse_light(int scene, int emit_tex, int* out_mat);           /* m:make-diffuse-light :103 */

/* hitables — geometry.scm / bezier.scm.  Objects may be shared and nested. */
int rt_add_sphere(int scene, const double center[3], double radius, int mat, int* out_obj);   /* g:make-sphere :146 */
int rt_add_moving_sphere(int scene, const double center0[3], const double center1[3],
                         double time0, double time1, double radius, int mat, int* out_obj);     /* g:make-moving-sphere :177 */
/* axis: RT_RECT_XY (a=x,b=y,k=z), RT_RECT_XZ (a=x,b=z,k=y), RT_RECT_YZ (a=y,b=z,k=x) */
int rt_add_rect(int scene, int axis, double a0, double a1, double b0, double b1, double k,
                int mat, int* out_obj);                                                          /* g:make-{xy,xz,yz}-rect :376-431 */
/* cubic Bezier curve a,b,c,d of the given width (b:make-bezier bezier.scm:61); hit t is the distance
 * along unit(dir) and the normal is -dir (bezier.scm:176-214).  width: positive and finite (for width
 * <= 0 the reference's depth estimate takes the log of a number <= 0 and raises on the first hit test) */
int rt_add_bezier(int scene, const double a[3], const double b[3], const double c[3], const double d[3],
                  double width, int mat, int* out_obj);
/* n curves at once (bezier->objs points.scm:45-53 over points->bezier output): cps holds n*12 doubles
 * (a,b,c,d per curve); the curves get the consecutive object ids *out_first .. *out_first + n - 1 */
int rt_add_bezier_array(int scene, const double* cps, int n, double width, int mat, int* out_first);
int rt_add_flip_normals(int scene, int obj, int* out_obj);                                       /* g:flip-normals :433 */
/* g:make-constant-medium boundary density a (geometry.scm:545): a volume of the given density inside
 * `boundary` (spheres / rects / boxes / instances); the phase function is a lambertian material with
 * texture albedo_tex, created by this call.  Its hit test draws one random number (like the reference),
 * so media are evaluated in object-list order relative to the objects before them. */
int rt_add_constant_medium(int scene, int boundary, double density, int albedo_tex, int* out_obj);
/* g:make-klein center mat (geometry.scm:645): Kleinian limit set, sphere traced (no bounding box) */
int rt_add_klein(int scene, const double center[3], int mat, int* out_obj);
int rt_add_box(int scene, const double p0[3], const double p1[3], int mat, int* out_obj);       /* g:make-box :444 */
int rt_add_translate(int scene, int obj, const double offset[3], int* out_obj);                 /* g:translate :465 */
int rt_add_rotate_y(int scene, int obj, double angle_deg, int* out_obj);                        /* g:rotate-y :483 */
/* An object list (make-scene's obj-list, geometry.scm:52; a nested list). */
int rt_add_list(int scene, const int* objs, int n, int* out_obj);
/* g:make-bvh-node :226 / g:make-bvh-with-sah :294.  Closest-hit over the
 * children; the library builds its own acceleration structure. */
int rt_add_bvh(int scene, const int* objs, int n, double time0, double time1, int sah, int* out_obj);

/* camera — cam:make-camera (camera.scm:63-78) evaluated on the host side;
 * the 24 doubles are the 10 slots the reference's get-ray reads. */
int rt_make_camera(const double lookfrom[3], const double lookat[3], const double vup[3],
                   double vfov_deg, double aspect, double aperture, double focus_dist,
                   double time0, double time1, double out_cam[RT_CAMERA_DOUBLES]);
int rt_set_camera(int scene, const double cam[RT_CAMERA_DOUBLES]);
/* Extension (pdf.scm:18-41): lambertian bounces sample the mixture of
 * (hitable-pdf light p) and (cosine-pdf normal), with g:pdf-value / g:random defined for an axis rect
 * or a sphere as in "The Rest of Your Life".  light_obj = a rect or sphere object (flips allowed),
 * -1 = off (the reference's own cosine sampling).  The reference never wires pdf.scm, so this path
 * is checked against the oracle's restatement only. */
int rt_set_light_sampling(int scene, int light_obj);
int rt_set_sky(int scene, int sky);
/* Perlin tables (perlin.scm:32-36): the reference draws them from the global
 * RNG at module load; here they are data.  ranvec: 256 unit vec3, perm: 256
 * entries each (a permutation of 0..255). */
int rt_set_perlin_tables(int scene, const double ranvec[256 * 3], const int32_t perm_x[256],
                         const int32_t perm_y[256], const int32_t perm_z[256]);
/* Fix the world (make-scene's obj-list) and upload the scene to the device. */
int rt_scene_commit(int scene, int world_list_obj);

/* ---- rendering -------------------------------------------------------- */
/* One call = `spp_count` successive trace-all passes (main.scm:471-491) with
 * pass indices spp_begin+1 .. spp_begin+spp_count: for every pixel j = y*nx+x
 * (y = 0 is the bottom row) the per-sample colours are added to accum[3j..3j+2]
 * in sample order, exactly the `*raw-data*` running sum.  Random numbers come
 * from a counter-based stream keyed by (seed, pixel, sample), so results do
 * not depend on launch geometry, batching or sharding.
 *
 * rt_render: accum is a caller-owned HOST buffer (nx*ny*3 doubles), copied to
 * the device and back (PCIe-inclusive).
 * rt_render_device: accum is caller-owned DEVICE memory on the context's GPU
 * (e.g. a torch tensor's data_ptr); stream is a hipStream_t or NULL for the
 * context's own stream.  shard_index/shard_count select an interleaved subset
 * of 16x16 pixel tiles (tile (tx, ty) belongs to shard (tx + k ty) % shard_count, k the
 * smallest odd prime that does not divide shard_count: 3, or 5 for 3, 6, 9, ... shards);
 * pixels of other shards are left untouched. */
int rt_render(int scene, int nx, int ny, int spp_begin, int spp_count, uint64_t seed,
              double* accum_host);
int rt_render_device(int scene, int nx, int ny, int spp_begin, int spp_count, uint64_t seed,
                     int shard_index, int shard_count, double* accum_device, void* stream);

/* Rows [y_begin, y_begin + y_count) only (same pass semantics as rt_render): the
 * band of the frame trace-line (main.scm:452-469) renders one row of.  accum is
 * the whole nx*ny*3 frame; only the band's entries are read or written (the
 * host version copies only the band across PCIe). */
int rt_render_rows(int scene, int nx, int ny, int y_begin, int y_count, int spp_begin, int spp_count,
                   uint64_t seed, double* accum_host);
int rt_render_rows_device(int scene, int nx, int ny, int y_begin, int y_count, int spp_begin, int spp_count,
                          uint64_t seed, double* accum_device, void* stream);
/* trace-line (main.scm:452-469), as animate calls it (main.scm:533-544): add
 * sample number `sample_count` (1-based) of every pixel of row y to raw_data
 * (the *raw-data* running sum, nx*ny*3 doubles, y-up rows) and re-resolve row
 * y of image (*image*, nx*ny*3 bytes) with sqrt(sum/sample_count).  Host
 * buffers, caller-owned.  A frame done row by row equals the trace-all pass
 * with the same sample_count bit for bit. */
int rt_trace_line(int scene, int nx, int ny, int y, int sample_count, uint64_t seed, double* raw_data,
                  uint8_t* image);
/* One shard's tiles (as rt_render_device's shard arguments) into a COMPACT
 * accumulator: accum_compact[3q..3q+2] is the running sum of pixel
 * rt_shard_pixels(...)[q], so a rank holds and ships only its own pixels
 * (multi-GPU gather, bench.py / rtamd.dist). */
int rt_render_shard_device(int scene, int nx, int ny, int spp_begin, int spp_count, uint64_t seed,
                           int shard_index, int shard_count, double* accum_compact, void* stream);

/* The pixels shard `shard_index` of `shard_count` renders (host-only, no GPU
 * needed): interleaved 16x16 tiles in row-major tile order, tile (tx, ty)
 * belongs to shard (tx + k ty) % shard_count, k = the smallest odd prime not
 * dividing shard_count (diagonal and coprime, so no shard gets whole columns
 * or only some residues of them); pixel j = y*nx + x, listed tile by tile.
 * Pass out_pix = NULL to get the count only. */
int rt_shard_pixels(int nx, int ny, int shard_index, int shard_count, uint32_t* out_pix, int64_t* out_count);

/* ---- multi-GPU frame (one process per GPU) ----------------
 * Each rank renders its tiles with rt_render_shard_device into a compact
 * accumulator; at frame end rt_gather_shards moves every rank's accumulator to
 * rank 0 over RCCL (xGMI between the GPUs of a node) and places the pixels into
 * rank 0's y-up frame.  Replaces nothing in the reference, which renders on one
 * thread (main.scm:471-491, 633-634): it is the frame's only exchange step.
 *
 * rt_comm_unique_id: rank 0 makes the communicator's id (ncclGetUniqueId); the
 *   host program ships the RT_COMM_ID_BYTES bytes to the other ranks (e.g.
 *   over its own process group or a file).
 * rt_comm_create: every rank, with the same id, its rank and the world size;
 *   collective (returns once all ranks have called it).  The communicator
 *   runs on the context's device.
 * rt_gather_shards: every rank, collective.  accum_compact = the rank's
 *   compact accumulator (device, 3 doubles per pixel of
 *   rt_shard_pixels(nx, ny, rank, world)); frame_device = rank 0's nx*ny*3
 *   frame (device; NULL on other ranks), whose pixels of every shard are
 *   overwritten.  Enqueued on `stream` (NULL: the context's stream), which the
 *   call synchronises before it returns.  The frame equals a one-process
 *   rt_render_device of the same passes bit for bit (disjoint pixels, nothing
 *   is summed).  The communicator stays valid through the call even if another
 *   thread destroys its handle; its context must outlive the call.
 * rt_gather_layout: host-only (no GPU, no RCCL): for each rank r of `world`,
 *   out_count[r] = its shard's pixel count and out_offset[r] = the offset of
 *   its pixels in the ranks' concatenated rt_shard_pixels lists (out_offset[0]
 *   = 0).  Rank 0 receives rank r's compact accumulator at doubles
 *   3 * (out_offset[r] - out_count[0]) of its receive buffer.
 * rt_gather_shards_local: the same gather within one process (every shard of
 *   `world` on the context's device, e.g. several shards rendered by one
 *   GPU): accum_compact = a host array of `world` device pointers, shard r's
 *   compact accumulator in entry r; the same receive layout and placement as
 *   rt_gather_shards, with device copies in place of the sends and receives. */
#define RT_COMM_ID_BYTES 128
int rt_comm_unique_id(uint8_t out_id[RT_COMM_ID_BYTES]);
int rt_comm_create(int ctx, const uint8_t unique_id[RT_COMM_ID_BYTES], int rank, int world, int* out_comm);
int rt_comm_destroy(int comm);
int rt_gather_shards(int comm, int nx, int ny, const double* accum_compact, double* frame_device, void* stream);
int rt_gather_layout(int nx, int ny, int world, int64_t* out_count, int64_t* out_offset);
int rt_gather_shards_local(int ctx, int nx, int ny, int world, const double* const* accum_compact,
                           double* frame_device, void* stream);

/* Errors raised on the device.  Every loop of the kernels that waits on data
 * (rejection samplers, curve subdivision walks, persistent kernels' per-path
 * loops) has an iteration cap a valid random stream cannot reach, and queue
 * appends never pass their shard's capacity: a kernel that would instead sets
 * one of these bits and leaves the loop, and the render call fails with
 * rt_last_error() naming them ("device fault (flags N): ..."). */
enum { RT_FAULT_REJECT = 1, RT_FAULT_CURVE = 2, RT_FAULT_PATH = 4, RT_FAULT_SHARD = 8, RT_FAULT_LDS = 16 };

/* The world's closest hit for n rays (hit-obj-list over the scene list,
 * geometry.scm:33-50, with t in (0.001, 999999999999) as color asks it,
 * main.scm:104): rays = n x {ox, oy, oz, dx, dy, dz, time} (host memory);
 * out_t[i] = the hit's t and out_mat[i] = its material id (rt_add_material_*),
 * or out_mat[i] = -1 (and t 0) for a miss.  A diagnostic and test probe (the
 * oracle's orc_hit_world); scenes with constant media are refused, since the
 * medium's hit test draws from the path's random stream. */
int rt_hit_rays(int scene, int n, const double* rays, double* out_t, int32_t* out_mat);

/* converge's subdivision depth (bezier.scm:179-193) as the curve kernels compute it (bez_maxd): for n
 * curves given in ray space (cps = n x 12 doubles, the control points after bezier-transform) and 8 eps
 * each (eps = width / 20), out_depth[i] = ceiling((log z) / (log 4)) with z = sqrt(2) n (n-1) l0 / (8 eps),
 * 0 where the log is -inf, saturated at 25 (one past the 24 levels the walk supports; deeper curves fault
 * the render).  A test probe of the device's log against the C library's. */
int rt_curve_depth_probe(int ctx, int n, const double* cps, const double* eps8, int32_t* out_depth);

/* Statistics of the last render on this scene. */
typedef struct rt_stats {
    uint64_t segments;    /* closest-hit queries issued by the integrator (ray segments) */
    uint64_t paths;       /* camera samples */
    double   ms_total;    /* wall time of the render call */
    double   ms_extend;   /* summed device time of the extend (closest-hit) kernel */
    double   ms_shade;    /* summed device time of the shade kernel */
    uint64_t extend_launches;
    uint64_t extend_rays; /* segments the extend kernels traced (the wavefront launches and the fused curve extend; the rest ran in the tail kernel) */
    uint32_t max_depth_seen;  /* deepest wavefront iteration (the tail kernel and the fused curve extend run the deeper ones) */
    uint32_t reserved;
    double   ms_finish;       /* summed device time of the tail kernel */
    uint64_t finish_paths;    /* paths handed to the tail kernel */
    uint64_t shade_hits_d0;   /* camera-ray hits shaded by the wavefront shade kernels */
    uint64_t shade_hits;      /* deeper hits shaded by the wavefront shade kernels */
    uint64_t shade_survivors; /* paths the shade kernels wrote on to the next iteration */
    uint32_t chunks;          /* sample chunks the render was cut into (path pools) */
    uint32_t lanes;           /* render lanes (path pool + stream) kept in flight */
    uint64_t curve_pooled_batches; /* curve subdivision passes over a full survivor pool (wavefront curve kernels) */
    uint64_t curve_flat_pooled;    /* curves those passes walked whose root is a leaf (flat: depth estimate < 0) */
} rt_stats;
int rt_get_stats(int scene, rt_stats* out);

/* What a committed scene became on the device (diagnostics for benchmarks
 * and tests): primitive and tree sizes, and the LDS footprint and resident
 * grid of the persistent LDS kernels (0 = the scene does not use them). */
typedef struct rt_scene_info {
    int32_t  leaves;          /* flattened primitives (leaf records) */
    int32_t  groups;          /* closest-hit groups (a BVH counts as one) */
    int32_t  bvh_nodes;       /* inner nodes of the all-times tree */
    int32_t  bvh0_nodes;      /* inner nodes of the time-0 tree */
    int32_t  tree_depth;      /* deepest tree level (the per-lane traversal stack) */
    int32_t  bvh_solo;        /* 1: the world is exactly one BVH group */
    uint32_t extend_lds_bytes, extend_lds_blocks;   /* k_extend_lds: LDS per block, resident blocks */
    uint32_t camera_lds_bytes, camera_lds_blocks;   /* k_camera: the same */
    int32_t  cus;             /* compute units of the context's device */
    int32_t  curve_stack;     /* curve trees: stack entries the BVH4 walk of k_extend_curves may hold (0: none) */
    double   commit_ms;       /* rt_scene_commit's wall time: flattening, BVH builds (SAH, BVH4 collapse), upload */
    double   commit_upload_ms; /* of it: device allocations and host-to-device copies */
    double   commit_sah_ms;   /* of it: the SAH builds of the world BVH (on commit_threads host threads) */
    int32_t  commit_threads;  /* host threads the SAH builds may use (the process's CPUs, at most 16) */
    int32_t  reserved0;
} rt_scene_info;
int rt_get_scene_info(int scene, rt_scene_info* out);
/* Record per-kernel HIP events during renders (adds a little host overhead). */
int rt_set_profiling(int scene, int enabled);

/* Resolve (main.scm:481-491): c = sqrt(sum/sample_count) per channel, then
 * floor(255.99*min(1,c)) into out (nx*ny*3 bytes, same y-up layout). Host. */
int rt_resolve_u8(const double* accum, int nx, int ny, int sample_count, uint8_t* out);
/* Same on the device (accum_device and out_device are device pointers). */
int rt_resolve_u8_device(int ctx, const double* accum_device, int nx, int ny, int sample_count,
                         uint8_t* out_device, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RTAMD_RT_H */
