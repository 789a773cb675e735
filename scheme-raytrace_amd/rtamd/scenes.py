"""The reference's scene definitions (main.scm:31-426) as descriptor graphs.

Scene generation draws from a HostStream (the reference's global stream at
load / scene-construction time); arguments and `let` bindings are evaluated
left to right.  `random_scene` applies repair R1: the
reference's `(g:make-scene obj-list)` (main.scm:89) lacks the camera and sky
arguments, so the cover scene is completed with `*camera*` (main.scm:141-153,
aspect nx/ny — repair R3) and `sky-color`.
"""
from . import perlin as _perlin
from . import scene as g
from . import vec as v
from .camera import make_camera
from .rng import HostStream

# aliases following the reference's module prefixes
m = g
t = g

#: default host-stream seeds (scene construction / Perlin tables)
SCENE_SEED = 0x5EED0001
PERLIN_SEED = 0x5EED0003


def camera_for(nx, ny):
    """*camera* (main.scm:141-153) with aspect nx/ny (R3)."""
    return make_camera(v.vec3(0, 5, 5), v.vec3(0, 0, 0), v.vec3(0, 1, 0), 40, nx / ny, 0, 1, 0, 1)


def cornell_camera_for(nx, ny):
    """*cornell-camera* (main.scm:129-139) with aspect nx/ny."""
    return make_camera(v.vec3(278, 278, -800), v.vec3(278, 278, 0), v.vec3(0, 1, 0), 40, nx / ny, 0, 1, 0, 1)


def random_scene_objects(rr, ground=None):
    """The obj-list of random-scene (main.scm:31-88), drawing from ``rr``.

    The list is in the reference's order: push! prepends, so the last pushed
    object comes first.  ``ground`` overrides the ground texture (config C3).
    """
    checker = g.checker_texture(g.constant_texture(v.vec3(0.2, 0.3, 0.1)),
                                g.constant_texture(v.vec3(0.9, 0.9, 0.9)))
    pushed = [g.make_sphere(v.vec3(0, -1000, 0), 1000, g.make_lambertian(ground or checker))]
    for a in range(-5, 10):
        for b in range(-5, 10):
            choose_mat = rr()
            cx = a + 0.9 * rr()
            cz = b + 0.9 * rr()
            center = v.vec3(cx, 0.2, cz)
            if v.length(v.diff(center, v.vec3(4, 0.2, 0))) > 0.9:
                if choose_mat < 0.8:
                    c1 = v.sum(center, v.vec3(0, 0.5 * rr(), 0))
                    r0 = rr() * rr()
                    g0 = rr() * rr()
                    b0 = rr() * rr()
                    pushed.append(g.make_moving_sphere(center, c1, 0, 1, 0.2,
                                                       g.make_lambertian(g.constant_texture(v.vec3(r0, g0, b0)))))
                elif choose_mat < 0.95:
                    r0 = 0.5 * (1 + rr())
                    g0 = 0.5 * (1 + rr())
                    b0 = 0.5 * (1 + rr())
                    fuzz = 0.5 * rr()
                    pushed.append(g.make_sphere(center, 0.2,
                                                g.make_metal(g.constant_texture(v.vec3(r0, g0, b0)), fuzz)))
                else:
                    pushed.append(g.make_sphere(center, 0.2, g.make_dielectric(1.5)))
    pushed.append(g.make_sphere(v.vec3(0, 1, 0), 1, g.make_dielectric(1.5)))
    pushed.append(g.make_sphere(v.vec3(-4, 1, 0), 1, g.make_lambertian(g.constant_texture(v.vec3(0.4, 0.2, 0.1)))))
    pushed.append(g.make_sphere(v.vec3(4, 1, 0), 1, g.make_metal(g.constant_texture(v.vec3(0.7, 0.6, 0.5)), 0)))
    return list(reversed(pushed))


def random_scene(nx, ny, seed=SCENE_SEED):
    """Cover scene (configs C1/C2): random-scene + R1 + R3."""
    objs = random_scene_objects(HostStream(seed))
    return g.make_scene(objs, camera_for(nx, ny), g.sky_color)


def marble_random_scene(nx, ny, seed=SCENE_SEED, perlin_seed=PERLIN_SEED):
    """Config C3: the cover scene with the ground's checker replaced by
    (t:marble-texture 1) as in test-scene2 (main.scm:317-320); moving spheres
    kept.  Perlin tables drawn in the reference's load order."""
    tables = _perlin.from_seed(perlin_seed)
    objs = random_scene_objects(HostStream(seed), ground=g.marble_texture(1))
    return g.make_scene(objs, camera_for(nx, ny), g.sky_color, perlin=tables)


def test_scene(nx, ny):
    """test-scene (main.scm:155-174), black sky."""
    objs = [
        g.make_sphere(v.vec3(0, 0, -1), 0.5, g.make_lambertian(g.constant_texture(v.vec3(0.1, 0.2, 0.5)))),
        g.make_sphere(v.vec3(0, -100.5, -1), 100,
                      g.make_lambertian(g.checker_texture(g.constant_texture(v.vec3(0.2, 0.3, 0.1)),
                                                          g.constant_texture(v.vec3(0.9, 0.9, 0.9))))),
        g.make_sphere(v.vec3(1, 0, -1), 0.5, g.make_metal(g.constant_texture(v.vec3(0.8, 0.6, 0.2)), 0.3)),
        g.make_sphere(v.vec3(-1, 0, -1), 0.5, g.make_dielectric(1.5)),
        g.make_sphere(v.vec3(-1, 0, -1), -0.45, g.make_dielectric(1.5)),
    ]
    return g.make_scene(objs, camera_for(nx, ny), g.black)


def test_scene2(nx, ny, perlin_seed=PERLIN_SEED):
    """test-scene2 (main.scm:316-328): marble spheres, two lights, black sky."""
    per_tex = g.marble_texture(1)
    light = g.make_diffuse_light(g.constant_texture(v.vec3(4, 4, 4)))
    objs = [
        g.make_sphere(v.vec3(0, -1000, -1), 1000, g.make_lambertian(per_tex)),
        g.make_sphere(v.vec3(0, 2, 0), 2, g.make_lambertian(per_tex)),
        g.make_sphere(v.vec3(0, 7, 0), 2, g.make_diffuse_light(g.constant_texture(v.vec3(4, 4, 4)))),
        g.make_xy_rect(3, 5, 1, 3, -2, light),
    ]
    return g.make_scene(objs, camera_for(nx, ny), g.black, perlin=_perlin.from_seed(perlin_seed))


def cornell_box(nx, ny):
    """cornell-box (main.scm:330-351): rects, two rotated/translated boxes,
    a flipped ceiling light; sky-color as in the reference (Q22)."""
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    white = g.make_lambertian(g.constant_texture(v.vec3(0.73, 0.73, 0.73)))
    green = g.make_lambertian(g.constant_texture(v.vec3(0.12, 0.45, 0.15)))
    light = g.make_diffuse_light(g.constant_texture(v.vec3(3, 3, 3)))
    objs = [
        g.flip_normals(g.make_yz_rect(0, 555, 0, 555, 555, green)),
        g.make_yz_rect(0, 555, 0, 555, 0, red),
        g.flip_normals(g.make_xz_rect(213, 343, 227, 332, 554, light)),
        g.flip_normals(g.make_xz_rect(0, 555, 0, 555, 555, white)),
        g.make_xz_rect(0, 555, 0, 555, 0, white),
        g.flip_normals(g.make_xy_rect(0, 555, 0, 555, 555, white)),
        g.translate(g.rotate_y(g.make_box(v.vec3(0, 0, 0), v.vec3(165, 165, 165), white), -18), v.vec3(130, 0, 65)),
        g.translate(g.rotate_y(g.make_box(v.vec3(0, 0, 0), v.vec3(165, 330, 165), white), 15), v.vec3(265, 0, 295)),
    ]
    return g.make_scene(objs, cornell_camera_for(nx, ny), g.sky_color)


def cornell_mixture(nx, ny):
    """cornell-box with the pdf.scm mixture (extension f2, config C4's
    "mixture/cosine importance sampling"): lambertian bounces sample the
    ceiling light and the cosine lobe half and half."""
    sc = cornell_box(nx, ny)
    light = sc.obj_list[2]                      # (g:flip-normals (g:make-xz-rect 213 343 227 332 554 light))
    return g.make_scene(sc.obj_list, sc.camera, sc.sky_function, light=light)


def line_upped_spheres(nx, ny, rr):
    """line-upped-spheres (main.scm:177-191)."""
    out = []
    for x in range(nx):
        for y in range(ny):
            r0, g0, b0 = rr(), rr(), rr()
            out.insert(0, g.make_sphere(v.vec3(x, 0, y), 0.5,
                                        g.make_lambertian(g.constant_texture(v.vec3(r0, g0, b0)))))
    return out


def test_scene_bvh_sah(nx, ny, seed=SCENE_SEED):
    """test-scene-bvh-sah (main.scm:226-235), the reference's default *scene*."""
    ground = g.make_sphere(v.vec3(0, -100.5, -1), 100,
                           g.make_lambertian(g.checker_texture(g.constant_texture(v.vec3(0.2, 0.3, 0.1)),
                                                               g.constant_texture(v.vec3(0.9, 0.9, 0.9)))))
    spheres = line_upped_spheres(10, 10, HostStream(seed))
    return g.make_scene([ground, g.make_bvh_with_sah(spheres, 0, 0)], camera_for(nx, ny), g.sky_color)


def test_bezier(nx, ny):
    """test-bezier (main.scm:237-277): checker ground, six spheres and three
    width-0.1 curves under one make-bvh-node; *camera*, sky-color."""
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    green = g.make_lambertian(g.constant_texture(v.vec3(0.12, 0.45, 0.15)))
    blue = g.make_lambertian(g.constant_texture(v.vec3(0.12, 0.15, 0.45)))
    ground = g.make_sphere(v.vec3(0, -100.5, -1), 100,
                           g.make_lambertian(g.checker_texture(g.constant_texture(v.vec3(0.2, 0.3, 0.1)),
                                                               g.constant_texture(v.vec3(0.9, 0.9, 0.9)))))
    inner = [
        g.make_sphere(v.vec3(2, 0, 2), 0.5, red),
        g.make_sphere(v.vec3(-2, 0, -2), 0.5, green),
        g.make_sphere(v.vec3(-1, 0, -1), 0.1, blue),
        g.make_sphere(v.vec3(-0.8, 1, 1), 0.1, blue),
        g.make_sphere(v.vec3(0.8, -1, 1), 0.1, blue),
        g.make_sphere(v.vec3(1, 0, -1), 0.1, blue),
        g.make_bezier(v.vec3(-1, 0, -1), v.vec3(-0.8, 1, 1), v.vec3(0.8, -1, 1), v.vec3(1, 0, -1), 0.1, red),
        g.make_bezier(v.vec3(-1, 0, 1), v.vec3(-0.8, 1, -1), v.vec3(0.8, -1, -1), v.vec3(1, 0, 1), 0.1, red),
        g.make_bezier(v.vec3(-1, 0, 2), v.vec3(-0.8, 1, -2), v.vec3(0.8, -1, -2), v.vec3(1, 0, 2), 0.1, red),
    ]
    return g.make_scene([ground, g.make_bvh_node(inner, 0, 0)], camera_for(nx, ny), g.sky_color)


def cornell_bezier(nx, ny):
    """cornell-bezier (main.scm:353-373): the Cornell frame with one width-10
    red curve in place of the boxes."""
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    white = g.make_lambertian(g.constant_texture(v.vec3(0.73, 0.73, 0.73)))
    green = g.make_lambertian(g.constant_texture(v.vec3(0.12, 0.45, 0.15)))
    light = g.make_diffuse_light(g.constant_texture(v.vec3(3, 3, 3)))
    objs = [
        g.flip_normals(g.make_yz_rect(0, 555, 0, 555, 555, green)),
        g.make_yz_rect(0, 555, 0, 555, 0, red),
        g.flip_normals(g.make_xz_rect(213, 343, 227, 332, 554, light)),
        g.flip_normals(g.make_xz_rect(0, 555, 0, 555, 555, white)),
        g.make_xz_rect(0, 555, 0, 555, 0, white),
        g.flip_normals(g.make_xy_rect(0, 555, 0, 555, 555, white)),
        g.make_bezier(v.vec3(130, 0, 65), v.vec3(150, 0, 190), v.vec3(130, 0, 190), v.vec3(265, 0, 295), 10, red),
    ]
    return g.make_scene(objs, cornell_camera_for(nx, ny), g.sky_color)


def cornell_smoke(nx, ny):
    """cornell-smoke (main.scm:375-398): the Cornell boxes as constant media
    of density 0.01 (white and black smoke), a larger light, black sky."""
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    white = g.make_lambertian(g.constant_texture(v.vec3(0.73, 0.73, 0.73)))
    green = g.make_lambertian(g.constant_texture(v.vec3(0.12, 0.45, 0.15)))
    light = g.make_diffuse_light(g.constant_texture(v.vec3(3, 3, 3)))
    b1 = g.translate(g.rotate_y(g.make_box(v.vec3(0, 0, 0), v.vec3(165, 165, 165), white), -18), v.vec3(130, 0, 65))
    b2 = g.translate(g.rotate_y(g.make_box(v.vec3(0, 0, 0), v.vec3(165, 330, 165), white), 15), v.vec3(265, 0, 295))
    objs = [
        g.flip_normals(g.make_yz_rect(0, 555, 0, 555, 555, green)),
        g.make_yz_rect(0, 555, 0, 555, 0, red),
        g.flip_normals(g.make_xz_rect(113, 443, 127, 432, 554, light)),
        g.flip_normals(g.make_xz_rect(0, 555, 0, 555, 555, white)),
        g.make_xz_rect(0, 555, 0, 555, 0, white),
        g.flip_normals(g.make_xy_rect(0, 555, 0, 555, 555, white)),
        g.make_constant_medium(b1, 0.01, g.constant_texture(v.vec3(1, 1, 1))),
        g.make_constant_medium(b2, 0.01, g.constant_texture(v.vec3(0, 0, 0))),
    ]
    return g.make_scene(objs, cornell_camera_for(nx, ny), g.black)


def klein_scene(nx, ny):
    """klein-scene (main.scm:400-407): ground sphere and a Kleinian limit set."""
    white = g.make_lambertian(g.constant_texture(v.vec3(0.73, 0.73, 0.73)))
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    objs = [g.make_sphere(v.vec3(0, -1003, -1), 1000, white), g.make_klein(v.vec3(0, 2, 0), red)]
    return g.make_scene(objs, camera_for(nx, ny), g.sky_color)


def cornell_klein(nx, ny):
    """cornell-klein (main.scm:409-426): the limit set inside the Cornell frame."""
    blue = g.make_lambertian(g.constant_texture(v.vec3(0.05, 0.65, 0.65)))
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    white = g.make_lambertian(g.constant_texture(v.vec3(0.73, 0.73, 0.73)))
    green = g.make_lambertian(g.constant_texture(v.vec3(0.12, 0.45, 0.15)))
    light = g.make_diffuse_light(g.constant_texture(v.vec3(3, 3, 3)))
    objs = [
        g.flip_normals(g.make_yz_rect(0, 555, 0, 555, 555, green)),
        g.make_yz_rect(0, 555, 0, 555, 0, red),
        g.flip_normals(g.make_xz_rect(113, 443, 127, 432, 554, light)),
        g.flip_normals(g.make_xz_rect(0, 555, 0, 555, 555, white)),
        g.make_xz_rect(0, 555, 0, 555, 0, white),
        g.flip_normals(g.make_xy_rect(0, 555, 0, 555, 555, white)),
        g.make_klein(v.vec3(250, 200, 280), blue),
    ]
    return g.make_scene(objs, cornell_camera_for(nx, ny), g.sky_color)


CURVE_SEED = 0x5EED0005


def random_polyline_curves(n_curves, seed=CURVE_SEED, segs_per_line=256, lo=10.0, hi=545.0, step=6.0):
    """Control points of ``n_curves`` curves: seeded random-walk polylines
    inside the Cornell frame, each turned into ``segs_per_line`` segments by
    the points->bezier rule (points.scm:22-43, vectorised with the same
    operation order as rtamd.points).  Returns an (n, 12) float64 array."""
    import numpy as np
    rng = np.random.default_rng(seed)
    n_lines = max(1, -(-n_curves // segs_per_line))
    npts = segs_per_line + 3
    start = rng.uniform(lo + 70.0, hi - 70.0, size=(n_lines, 1, 3))
    steps = rng.uniform(-step, step, size=(n_lines, npts - 1, 3))
    pts = np.concatenate([start, start + np.cumsum(steps, axis=1)], axis=1)
    pts = np.clip(pts, lo, hi)
    pt, p1, p2, p3 = pts[:, :-3], pts[:, 1:-2], pts[:, 2:-1], pts[:, 3:]
    d1 = (p2 - pt) * (1 / 6)
    d2 = (p3 - p1) * (1 / 6)
    cps = np.concatenate([p1, p1 + d1, p2 - d2, p2], axis=2).reshape(-1, 12)
    return np.ascontiguousarray(cps[:n_curves])


def cornell_curves(nx, ny, n_curves=1 << 20, width=0.5, seed=CURVE_SEED):
    """Config C5: ~1M red lambertian curves (width 0.1 x scale 5) in a BVH
    inside the cornell-bezier frame (main.scm:353-373), *cornell-camera*."""
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    white = g.make_lambertian(g.constant_texture(v.vec3(0.73, 0.73, 0.73)))
    green = g.make_lambertian(g.constant_texture(v.vec3(0.12, 0.45, 0.15)))
    light = g.make_diffuse_light(g.constant_texture(v.vec3(3, 3, 3)))
    curves = g.bezier_array(random_polyline_curves(n_curves, seed), width, red)
    objs = [
        g.flip_normals(g.make_yz_rect(0, 555, 0, 555, 555, green)),
        g.make_yz_rect(0, 555, 0, 555, 0, red),
        g.flip_normals(g.make_xz_rect(213, 343, 227, 332, 554, light)),
        g.flip_normals(g.make_xz_rect(0, 555, 0, 555, 555, white)),
        g.make_xz_rect(0, 555, 0, 555, 0, white),
        g.flip_normals(g.make_xy_rect(0, 555, 0, 555, 555, white)),
        g.make_bvh_node([curves], 0, 0),
    ]
    return g.make_scene(objs, cornell_camera_for(nx, ny), g.sky_color)


def cornell_curves_small(nx, ny):
    """C5's generator at 4096 curves (oracle-checkable without a BVH)."""
    return cornell_curves(nx, ny, n_curves=4096, width=3.0)


SCENES = {
    "cover": random_scene,
    "cover_marble": marble_random_scene,
    "test_scene": test_scene,
    "test_scene2": test_scene2,
    "cornell": cornell_box,
    "bvh_sah": test_scene_bvh_sah,
    "test_bezier": test_bezier,
    "cornell_bezier": cornell_bezier,
    "cornell_smoke": cornell_smoke,
    "cornell_mixture": cornell_mixture,
    "klein": klein_scene,
    "cornell_klein": cornell_klein,
    "curves": cornell_curves,
    "curves_small": cornell_curves_small,
}
