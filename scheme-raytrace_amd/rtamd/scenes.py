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


SCENES = {
    "cover": random_scene,
    "cover_marble": marble_random_scene,
    "test_scene": test_scene,
    "test_scene2": test_scene2,
    "cornell": cornell_box,
    "bvh_sah": test_scene_bvh_sah,
}
