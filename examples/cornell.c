/* cornell.c — the cornell-box scene (main.scm:330-351) built and rendered
 * through the C ABI alone (include/rt.h), the way a foreign-function binding
 * of the reference would drive librtamd: constructors in the reference's
 * order, trace-all passes, resolve to 8-bit and a P3 PPM (main.scm:439-450).
 *
 *   gcc -O2 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ examples/cornell.c \
 *       -Lscheme-raytrace_amd/rtamd -l:librtamd.so -L/opt/rocm/lib -lamdhip64 \
 *       -Wl,-rpath,$PWD/scheme-raytrace_amd/rtamd -o cornell
 *   ./cornell 128 128 16 cornell.ppm          (needs a GPU)
 *   ./cornell 128 128 16 cornell.ppm gather   (the multi-GPU frame's path at world size 1: the
 *                                              rank's tiles into a compact device accumulator,
 *                                              rt_render_shard_device, then the frame-end RCCL
 *                                              gather into the device frame, rt_gather_shards)
 *   ./cornell --abi                           (prints the ABI version; no GPU)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "rt.h"

#define CHECK(call)                                                             \
    do {                                                                        \
        if (call) {                                                             \
            fprintf(stderr, "%s failed: %s\n", #call, rt_last_error());         \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

static int lambertian(int sc, double r, double g, double b) {
    const double rgb[3] = {r, g, b};
    int tex, mat;
    CHECK(rt_add_texture_constant(sc, rgb, &tex));
    CHECK(rt_add_material_lambertian(sc, tex, &mat));
    return mat;
}

static int rect(int sc, int axis, double a0, double a1, double b0, double b1, double k, int mat, int flip) {
    int o;
    CHECK(rt_add_rect(sc, axis, a0, a1, b0, b1, k, mat, &o));
    if (flip) CHECK(rt_add_flip_normals(sc, o, &o));
    return o;
}

static int box(int sc, const double p0[3], const double p1[3], int mat, double angle, const double off[3]) {
    int o;
    CHECK(rt_add_box(sc, p0, p1, mat, &o));
    CHECK(rt_add_rotate_y(sc, o, angle, &o));
    CHECK(rt_add_translate(sc, o, off, &o));
    return o;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "--abi") == 0) {
        printf("rt_abi_version %d\n", rt_abi_version());
        return 0;
    }
    const int nx = argc > 1 ? atoi(argv[1]) : 128, ny = argc > 2 ? atoi(argv[2]) : 128;
    const int spp = argc > 3 ? atoi(argv[3]) : 16;
    const char* out = argc > 4 ? argv[4] : "cornell.ppm";

    int ctx, sc;
    CHECK(rt_context_create(0, &ctx));
    CHECK(rt_scene_begin(ctx, &sc));
    const int red = lambertian(sc, 0.65, 0.05, 0.05), white = lambertian(sc, 0.73, 0.73, 0.73);
    const int green = lambertian(sc, 0.12, 0.45, 0.15);
    const double three[3] = {3, 3, 3};
    int ltex, light;
    CHECK(rt_add_texture_constant(sc, three, &ltex));
    CHECK(rt_add_material_diffuse_light(sc, ltex, &light));
    const double z[3] = {0, 0, 0}, b1[3] = {165, 165, 165}, b2[3] = {165, 330, 165};
    const double o1[3] = {130, 0, 65}, o2[3] = {265, 0, 295};
    int objs[8];
    objs[0] = rect(sc, RT_RECT_YZ, 0, 555, 0, 555, 555, green, 1);
    objs[1] = rect(sc, RT_RECT_YZ, 0, 555, 0, 555, 0, red, 0);
    objs[2] = rect(sc, RT_RECT_XZ, 213, 343, 227, 332, 554, light, 1);
    objs[3] = rect(sc, RT_RECT_XZ, 0, 555, 0, 555, 555, white, 1);
    objs[4] = rect(sc, RT_RECT_XZ, 0, 555, 0, 555, 0, white, 0);
    objs[5] = rect(sc, RT_RECT_XY, 0, 555, 0, 555, 555, white, 1);
    objs[6] = box(sc, z, b1, white, -18, o1);
    objs[7] = box(sc, z, b2, white, 15, o2);
    int world;
    CHECK(rt_add_list(sc, objs, 8, &world));
    /* *cornell-camera* (main.scm:129-139) with aspect nx/ny */
    const double from[3] = {278, 278, -800}, at[3] = {278, 278, 0}, up[3] = {0, 1, 0};
    double cam[RT_CAMERA_DOUBLES];
    CHECK(rt_make_camera(from, at, up, 40, (double)nx / ny, 0, 1, 0, 1, cam));
    CHECK(rt_set_camera(sc, cam));
    CHECK(rt_set_sky(sc, RT_SKY_GRADIENT));
    CHECK(rt_scene_commit(sc, world));

    double* accum = calloc((size_t)nx * ny * 3, sizeof(double));
    uint8_t* img = malloc((size_t)nx * ny * 3);
    if (argc > 5 && strcmp(argv[5], "gather") == 0) {
        /* one process of a multi-GPU frame (here world size 1): its communicator, its tiles into a
         * compact device accumulator, the frame-end gather into rank 0's device frame */
        const int rank = 0, world = 1;
        uint8_t id[RT_COMM_ID_BYTES];
        int comm;
        CHECK(rt_comm_unique_id(id));                /* rank 0; a multi-process host ships it to the others */
        CHECK(rt_comm_create(ctx, id, rank, world, &comm));
        int64_t npix = 0;
        CHECK(rt_shard_pixels(nx, ny, rank, world, NULL, &npix));
        double *d_shard = NULL, *d_frame = NULL;
        if (hipMalloc((void**)&d_shard, (size_t)npix * 3 * sizeof(double)) != hipSuccess ||
            hipMalloc((void**)&d_frame, (size_t)nx * ny * 3 * sizeof(double)) != hipSuccess) {
            fprintf(stderr, "hipMalloc failed\n");
            return 1;
        }
        hipMemset(d_shard, 0, (size_t)npix * 3 * sizeof(double));
        hipMemset(d_frame, 0, (size_t)nx * ny * 3 * sizeof(double));
        hipDeviceSynchronize();
        CHECK(rt_render_shard_device(sc, nx, ny, 0, spp, 0x5EED0002ull, rank, world, d_shard, NULL));
        CHECK(rt_gather_shards(comm, nx, ny, d_shard, d_frame, NULL));
        if (hipMemcpy(accum, d_frame, (size_t)nx * ny * 3 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
            fprintf(stderr, "hipMemcpy failed\n");
            return 1;
        }
        hipFree(d_shard);
        hipFree(d_frame);
        CHECK(rt_comm_destroy(comm));
    } else {
        CHECK(rt_render(sc, nx, ny, 0, spp, 0x5EED0002ull, accum));     /* spp trace-all passes */
    }
    CHECK(rt_resolve_u8(accum, nx, ny, spp, img));

    FILE* f = fopen(out, "w");
    if (!f) { perror(out); return 1; }
    fprintf(f, "P3\n %d %d\n255\n", nx, ny);                           /* main.scm:441 */
    for (int y = ny - 1; y >= 0; --y)                                     /* rows top-down, main.scm:445 */
        for (int x = 0; x < nx; ++x) {
            const uint8_t* p = img + 3 * ((size_t)y * nx + x);
            fprintf(f, "%d %d %d\n", p[0], p[1], p[2]);
        }
    fclose(f);
    double mean = 0;
    for (size_t i = 0; i < (size_t)nx * ny * 3; ++i) mean += accum[i];
    printf("cornell %dx%dx%d -> %s, mean radiance %.6f\n", nx, ny, spp, out, mean / ((double)nx * ny * 3 * spp));
    free(accum); free(img);
    CHECK(rt_scene_destroy(sc));
    CHECK(rt_context_destroy(ctx));
    return 0;
}
