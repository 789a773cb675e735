"""Known-answer tests of the oracle's restatement of the reference functions.

Expected values are derived by hand from the Scheme text (file:line cited per
test), evaluated here in Python floats (IEEE f64, libm) in the reference's
operation order — an independent second transliteration of each function.
"""
import math

import numpy as np
import pytest

from rtamd import scene as g
from rtamd import vec as v
from rtamd.camera import make_camera


def py_reflect(vv, n):                       # material.scm:41-43
    return v.diff(vv, v.scale(n, 2 * v.dot(vv, n)))


def py_refract(vv, n, ni):                   # material.scm:59-67 (raw v, Q5)
    uv = v.unit(vv)
    dt = v.dot(uv, n)
    disc = 1 - ni * ni * (1 - dt * dt)
    if disc > 0:
        return v.diff(v.scale(v.diff(vv, v.scale(n, dt)), ni), v.scale(n, math.sqrt(disc)))
    return None


def py_schlick(c, r):                        # material.scm:69-74
    r0 = (1 - r) / (1 + r)
    r0 = r0 * r0
    return r0 + (1 - r0) * (1 - c) ** 5


def test_reflect(oracle_mod):
    for vv, n in (((1.0, -1.0, 0.5), (0.0, 1.0, 0.0)), ((0.3, 0.2, -0.9), v.unit((1.0, 2.0, 3.0)))):
        assert oracle_mod.reflect(vv, n) == py_reflect(vv, n)


def test_refract_and_total_internal_reflection(oracle_mod):
    n = (0.0, 1.0, 0.0)
    vv = (0.6, -0.8, 0.0)
    assert oracle_mod.refract(vv, n, 1 / 1.5) == py_refract(vv, n, 1 / 1.5)
    # un-normalised incident vector: the tangential term uses raw v (Q5)
    assert oracle_mod.refract((1.2, -1.6, 0.0), n, 1 / 1.5) == py_refract((1.2, -1.6, 0.0), n, 1 / 1.5)
    # grazing ray leaving glass (ni = 1.5): total internal reflection
    assert oracle_mod.refract((0.9, 0.1, 0.0), (0.0, 1.0, 0.0), 1.5) is None


def test_schlick(oracle_mod):
    for c in (0.0, 0.25, 0.7, 1.0):
        assert oracle_mod.schlick(c, 1.5) == py_schlick(c, 1.5)
    assert oracle_mod.schlick(1.0, 1.5) == pytest.approx(0.04)


def test_onb_orthonormal_and_branch(oracle_mod):
    for nrm in ((0.0, 1.0, 0.0), (0.95, 0.1, 0.2), (-0.3, 0.4, 5.0)):
        u, vv, w = oracle_mod.onb(nrm)
        assert w == v.unit(nrm)                           # onb.scm:9
        a = (0.0, 1.0, 0.0) if abs(w[0]) > 0.9 else (1.0, 0.0, 0.0)
        assert vv == v.unit(v.cross(w, a))                # onb.scm:13
        assert u == v.cross(w, vv)
        m = np.array([u, vv, w])
        assert np.allclose(m @ m.T, np.eye(3), atol=1e-14)


def test_cosine_direction_has_the_x2_quirk(oracle_mod):
    # util.scm:37-44: x, y carry a stray factor 2 (Q1)
    r1, r2 = 0.125, 0.64
    x, y, z = oracle_mod.cosine_direction(r1, r2)
    phi = 2 * math.pi * r1
    assert (x, y, z) == (math.cos(phi) * 2 * math.sqrt(r2), math.sin(phi) * 2 * math.sqrt(r2), math.sqrt(1 - r2))
    assert x * x + y * y + z * z == pytest.approx(4 * r2 + 1 - r2)   # not unit length


def _world(objs, oracle_mod):
    sc = g.make_scene(objs, make_camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 90, 1, 0, 1, 0, 1), g.black)
    return oracle_mod.build_scene(sc)


def test_sphere_hit_and_negative_radius(oracle_mod):
    mat = g.make_dielectric(1.5)
    o = _world([g.make_sphere((0, 0, -1), 0.5, mat)], oracle_mod)
    t, px, py, pz, nx, ny, nz, _ = o.hit_world((0, 0, 0), (0, 0, -1))
    assert t == 0.5 and (px, py, pz) == (0, 0, -0.5) and (nx, ny, nz) == (0, 0, 1.0)   # geometry.scm:155-162
    # from inside: the far root (geometry.scm:163-170)
    t, *_ = o.hit_world((0, 0, -1), (0, 0, -1))
    assert t == 0.5
    # negative radius flips the normal (Q18, main.scm:171)
    o2 = _world([g.make_sphere((0, 0, -1), -0.45, mat)], oracle_mod)
    hit = o2.hit_world((0, 0, 0), (0, 0, -1))
    assert hit[6] == pytest.approx(-1.0) and hit[0] == pytest.approx(0.55)
    # tangent ray: discriminant == 0 is a miss (Q18)
    o3 = _world([g.make_sphere((0, 1, -2), 1.0, mat)], oracle_mod)
    assert o3.hit_world((0, 0, 0), (0, 0, -1)) is None


def test_closest_hit_strict_ties_keep_earlier(oracle_mod):
    a = g.make_lambertian(g.constant_texture((1, 0, 0)))
    b = g.make_lambertian(g.constant_texture((0, 1, 0)))
    o = _world([g.make_sphere((0, 0, -2), 0.5, a), g.make_sphere((0, 0, -2), 0.5, b),
                g.make_sphere((0, 0, -5), 0.5, b)], oracle_mod)
    hit = o.hit_world((0, 0, 0), (0, 0, -1))
    assert hit[0] == 1.5 and hit[7] == 0                 # first material wins the tie (geometry.scm:41-46)


def test_rect_bounds_nonstrict_and_flip(oracle_mod):
    m = g.make_lambertian(g.constant_texture((1, 1, 1)))
    o = _world([g.make_xy_rect(-1, 1, -1, 1, -3, m)], oracle_mod)
    assert o.hit_world((1, 1, 0), (0, 0, -1))[0] == 3.0       # on the corner: non-strict (Q20)
    assert o.hit_world((1.0000001, 0, 0), (0, 0, -1)) is None
    of = _world([g.flip_normals(g.make_xy_rect(-1, 1, -1, 1, -3, m))], oracle_mod)
    assert of.hit_world((0, 0, 0), (0, 0, -1))[6] == -1.0
    # xz and yz planes
    o2 = _world([g.make_xz_rect(-1, 1, -1, 1, 2, m), g.make_yz_rect(-1, 1, -1, 1, 4, m)], oracle_mod)
    assert o2.hit_world((0, 0, 0), (0, 1, 0))[:7] == (2.0, 0.0, 2.0, 0.0, 0.0, 1.0, 0.0)
    assert o2.hit_world((0, 0, 0), (1, 0, 0))[:7] == (4.0, 4.0, 0.0, 0.0, 1.0, 0.0, 0.0)


def test_instanced_box_hit(oracle_mod):
    """translate(rotate-y(box)) as in cornell-box (main.scm:343-345)."""
    m = g.make_lambertian(g.constant_texture((1, 1, 1)))
    box = g.translate(g.rotate_y(g.make_box((0, 0, 0), (165, 165, 165), m), -18), (130, 0, 65))
    o = _world([box], oracle_mod)
    hit = o.hit_world((200, 80, -500), (0, 0, 1))
    assert hit is not None
    # hand transform: ray into the instance, hit the rotated box face, back out
    th = (math.pi / 180) * -18
    s, c = math.sin(th), math.cos(th)
    ox, oy, oz = 200 - 130, 80.0, -500 - 65
    rx, rz = c * ox - s * oz, s * ox + c * oz
    dx, dz = c * 0 - s * 1, s * 0 + c * 1
    # the ray enters the box through its z0 face (flipped normal, geometry.scm:448)
    t = (0 - rz) / dz
    assert hit[0] == t
    lx, lz = rx + t * dx, rz + t * dz
    assert 0 <= lx <= 165
    px = c * lx + s * lz + 130
    assert hit[1] == pytest.approx(px, abs=1e-12)
    assert hit[4:7] == pytest.approx((-s, 0.0, -c), abs=1e-15)      # -(R^T e_z)


def test_camera_host_matches_oracle_and_library(oracle_mod):
    args = ((0, 5, 5), (0, 0, 0), (0, 1, 0), 40, 1920 / 1080, 0, 1, 0, 1)
    py = make_camera(*args).slots()
    assert oracle_mod.make_camera(*args) == py
    import ctypes
    from rtamd import _lib
    out = (ctypes.c_double * 24)()
    _lib.call("rt_make_camera", _lib.dvec(args[0]), _lib.dvec(args[1]), _lib.dvec(args[2]), args[3], args[4],
              args[5], args[6], args[7], args[8], out)
    assert list(out) == py


def test_checker_texture(oracle_mod):
    even = g.constant_texture((0.2, 0.3, 0.1))
    odd = g.constant_texture((0.9, 0.9, 0.9))
    m = g.make_lambertian(g.checker_texture(even, odd))
    o = _world([g.make_sphere((0, 0, 0), 1, m)], oracle_mod)
    for p in ((0.1, 0.2, 0.3), (-0.1, 0.2, 0.3), (0.5, -1.7, 2.2)):
        sines = math.sin(10 * p[0]) * math.sin(10 * p[1]) * math.sin(10 * p[2])   # texture.scm:18-20
        want = (0.9, 0.9, 0.9) if sines < 0 else (0.2, 0.3, 0.1)
        assert o.tex_value(2, p) == want


def py_noise(t, p):
    """perlin.scm:69-90 transliterated independently, including the shared
    inner vector of (make-vector 2 (make-vector 2 (make-vector 2))) (Q2)."""
    i, j, k = math.floor(p[0]), math.floor(p[1]), math.floor(p[2])
    u, vv, w = p[0] - i, p[1] - j, p[2] - k
    inner = [None, None]                      # the one innermost vector
    c = [[inner, inner], [inner, inner]]
    for di in range(2):
        for dj in range(2):
            for dk in range(2):
                h = t.perm_x[(i + di) & 255] ^ t.perm_y[(j + dj) & 255] ^ t.perm_z[(k + dk) & 255]
                c[di][dj][dk] = tuple(t.ranvec[3 * h:3 * h + 3])
    uu, vv2, ww = u * u * (3 - 2 * u), vv * vv * (3 - 2 * vv), w * w * (3 - 2 * w)
    acc = 0
    for di in range(2):
        for dj in range(2):
            for dk in range(2):
                acc += ((di * uu + (1 - di) * (1 - uu)) * (dj * vv2 + (1 - dj) * (1 - vv2))
                        * (dk * ww + (1 - dk) * (1 - ww)) * v.dot((u - di, vv - dj, w - dk), c[di][dj][dk]))
    return acc


def test_perlin_noise_turb_marble(oracle_mod):
    from rtamd import perlin
    t = perlin.from_seed(77)
    sc = g.make_scene([g.make_sphere((0, 0, 0), 1, g.make_lambertian(g.marble_texture(1)))],
                      make_camera((0, 0, 3), (0, 0, 0), (0, 1, 0), 40, 1, 0, 1, 0, 1), g.black, perlin=t)
    o = oracle_mod.build_scene(sc)
    for p in ((0.3, 0.7, 1.1), (-2.5, 0.25, 7.75), (123.4, -55.5, 0.001)):
        assert o.noise(p) == py_noise(t, p)
        acc, q, wgt = 0, p, 1
        for _ in range(7):                                     # perlin.scm:92-103
            acc = acc + wgt * py_noise(t, q)
            q = v.scale(q, 2)
            wgt = wgt * 0.5
        assert o.turb(p) == abs(acc)
        m = 0.5 * (1 + math.sin(1 * p[2] + 10 * abs(acc)))     # texture.scm:30-34
        assert o.tex_value(0, p) == (m, m, m)


def test_perlin_tables_shape():
    from rtamd import perlin
    t = perlin.from_seed(5)
    for perm in (t.perm_x, t.perm_y, t.perm_z):
        assert sorted(perm) == list(range(256))
    vecs = np.array(t.ranvec).reshape(256, 3)
    assert np.allclose((vecs ** 2).sum(axis=1), 1.0)
    assert len(t.ranfloat) == 256
