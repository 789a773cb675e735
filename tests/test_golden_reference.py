"""The oracle pinned against the REFERENCE ITSELF.

tests/golden/ref_*.json were produced by tests/golden/make_golden.py, which
executes the reference's own Scheme source (/root/reference, soma-arc/
scheme-raytrace) with a small Gauche-subset evaluator in the build container,
binding srfi-27 random-real to the same counter-based streams, with repairs
R1-R3 applied as overlays (see that script's header).  These tests check the
oracle (oracle/rt_oracle.c) and the host-side constructors (rtamd) against
those recorded outputs BIT FOR BIT; the GPU is checked against the same
fixtures in test_gpu_parity.py.
"""
import json
import math
import os

import numpy as np
import pytest

from rtamd import perlin, scenes
from rtamd.camera import make_camera

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCENES = ["test_scene", "test_scene2", "cornell", "cover", "bvh_sah", "test_bezier", "cornell_bezier",
          "cornell_smoke", "klein", "cornell_klein"]


def F(x):
    if isinstance(x, list):
        return [F(v) for v in x]
    if x is None or isinstance(x, bool):
        return x
    return float.fromhex(x)


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def kat():
    return load("ref_kat.json")


@pytest.mark.parametrize("name", SCENES)
def test_oracle_samples_bit_exact_vs_reference(name, oracle_mod):
    g = load("ref_%s.json" % name)
    nx, ny, spp = g["nx"], g["ny"], g["spp"]
    o = oracle_mod.build_scene(scenes.SCENES[name](nx, ny))
    bad = []
    for j, s, col, _ in g["samples"]:
        got = o.sample(nx, ny, j % nx, j // nx, g["path_seed"], s)
        if list(got) != F(col):
            bad.append((j, s, F(col), got))
    assert not bad, bad[:3]
    # the running sum and the 8-bit image (main.scm:480-491)
    acc, _ = o.render(nx, ny, 0, spp, g["path_seed"])
    assert list(acc) == [v for px in g["accum"] for v in F(px)]
    assert list(oracle_mod.resolve_u8(acc, spp)) == g["image"]


def test_fixtures_are_not_trivial():
    for name in SCENES:
        g = load("ref_%s.json" % name)
        acc = np.array([F(px) for px in g["accum"]])
        if name == "test_scene":            # black sky, no emitter: the reference renders black
            assert (acc == 0).all()
        else:
            assert (acc > 0).mean() > 0.1, name


def test_reference_draws_three_cosine_directions_per_lambertian_bounce(kat):
    """onb.scm's `local` is syntax-rules: (local uvw (random-cosine-direction))
    evaluates its argument three times (Q29), so a lambertian bounce consumes
    6 draws.  The per-sample draw counts in the fixtures show it: a camera
    path whose first hit is lambertian and whose bounce escapes uses
    2 (jitter) + 2k (disk) + 1 (time) + 6 draws."""
    g = load("ref_cornell.json")
    counts = {nd for _, _, _, nd in g["samples"]}
    assert any((nd - 5) % 2 == 0 and nd >= 11 for nd in counts)


def test_cosine_direction(kat, oracle_mod):
    for r1, r2, want in kat["cosine_direction"]:
        assert list(oracle_mod.cosine_direction(F(r1), F(r2))) == F(want)


def test_reflect_refract_schlick(kat, oracle_mod):
    for v, n, want in kat["reflect"]:
        assert list(oracle_mod.reflect(F(v), F(n))) == F(want)
    for v, n, ni, ok, want in kat["refract"]:
        got = oracle_mod.refract(F(v), F(n), F(ni))
        assert (got is not None) == ok
        if ok:
            assert list(got) == F(want)
    for c, r, want in kat["schlick"]:
        assert oracle_mod.schlick(F(c), F(r)) == F(want)


def test_onb(kat, oracle_mod):
    for n, u, v, w in kat["onb"]:
        gu, gv, gw = oracle_mod.onb(F(n))
        assert (list(gu), list(gv), list(gw)) == (F(u), F(v), F(w))


def test_camera_slots(kat, oracle_mod):
    def flat(slots):
        out = []
        for s in slots[:7]:
            out += F(s)
        return out + [F(x) for x in slots[7:]]
    c = make_camera((0, 5, 5), (0, 0, 0), (0, 1, 0), 40, 1920 / 1080, 0, 1, 0, 1).slots()
    assert c == flat(kat["camera_cover_1920x1080"])
    c2 = make_camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20, 3 / 2, 0.1, 10, 0, 1).slots()
    assert c2 == flat(kat["camera_lens"])
    assert oracle_mod.make_camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20, 3 / 2, 0.1, 10, 0, 1) == c2


def test_get_ray_with_lens(kat):
    """camera.scm:80-92 restated (the GPU's k_raygen follows the same order)."""
    from rtamd import vec as v
    cam = make_camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20, 3 / 2, 0.1, 10, 0, 1)
    draws = iter([0.9, 0.95, 0.3, 0.6, 0.25])
    while True:
        a, b = next(draws), next(draws)
        p = v.diff(v.scale(v.vec3(a, b, 0), 2), v.vec3(1, 1, 0))
        if v.dot(p, p) < 1:
            break
    rd = v.scale(p, cam.lens_radius)
    off = v.sum(v.scale(cam.u, rd[0]), v.scale(cam.v, rd[1]))
    time = cam.time0 + next(draws) * (cam.time1 - cam.time0)
    s, t = 0.25, 0.75
    o = v.sum(cam.origin, off)
    d = v.diff(v.sum(cam.llc, v.scale(cam.horizontal, s), v.scale(cam.vertical, t)), cam.origin, off)
    r = kat["get_ray_lens"]
    assert list(o) == F(r["origin"]) and list(d) == F(r["dir"]) and time == F(r["time"])


def test_perlin_tables_and_noise(kat, oracle_mod):
    t = perlin.from_seed(kat["perlin_seed"])
    assert t.ranvec == [x for vec in F(kat["perlin_ranvec"]) for x in vec]
    assert [t.perm_x, t.perm_y, t.perm_z] == kat["perlin_perm"]
    from rtamd import scene as g
    sc = g.make_scene([g.make_sphere((0, 0, 0), 1, g.make_lambertian(g.marble_texture(1))),
                       g.make_sphere((0, 5, 0), 1, g.make_lambertian(
                           g.checker_texture(g.constant_texture((0.2, 0.3, 0.1)),
                                             g.constant_texture((0.9, 0.9, 0.9)))))],
                      make_camera((0, 0, 3), (0, 0, 0), (0, 1, 0), 40, 1, 0, 1, 0, 1), g.black, perlin=t)
    o = oracle_mod.build_scene(sc)
    for p, want in kat["noise"]:
        assert o.noise(F(p)) == F(want)
    for p, want in kat["turb"]:
        assert o.turb(F(p)) == F(want)
    for p, want in kat["marble"]:
        assert list(o.tex_value(0, F(p))) == F(want)
    for p, want in kat["checker"]:
        assert list(o.tex_value(3, F(p))) == F(want)


def test_closest_hits(kat, oracle_mod):
    from rtamd import scene as g
    lam = g.make_lambertian
    ct = g.constant_texture
    worlds = {
        "spheres": [g.make_sphere((0, 0, -1), 0.5, lam(ct((1, 0, 0)))),
                    g.make_sphere((0, -100.5, -1), 100, lam(ct((0, 1, 0)))),
                    g.make_sphere((-1, 0, -1), -0.45, g.make_dielectric(1.5)),
                    g.make_moving_sphere((1, 0, -1), (1, 0.5, -1), 0, 1, 0.3, lam(ct((0, 0, 1))))],
        "cornell_boxes": [
            g.translate(g.rotate_y(g.make_box((0, 0, 0), (165, 165, 165), lam(ct((0.73, 0.73, 0.73)))), -18),
                        (130, 0, 65)),
            g.translate(g.rotate_y(g.make_box((0, 0, 0), (165, 330, 165), lam(ct((0.73, 0.73, 0.73)))), 15),
                        (265, 0, 295)),
            g.flip_normals(g.make_xz_rect(213, 343, 227, 332, 554, g.make_diffuse_light(ct((3, 3, 3)))))],
    }
    for name, objs in worlds.items():
        sc = g.make_scene(objs, make_camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 90, 1, 0, 1, 0, 1), g.black)
        o = oracle_mod.build_scene(sc)
        for orig, d, tm, rec in kat["hits"][name]:
            got = o.hit_world(F(orig), F(d), F(tm))
            if rec is None:
                assert got is None
            else:
                assert got is not None
                assert [got[0]] + list(got[1:4]) + list(got[4:7]) == [F(rec[0])] + F(rec[1]) + F(rec[2])


def test_moving_sphere_time_semantics(kat):
    """The same ray hits the moving sphere at time 0 and misses it at time
    0.7, when its centre has risen to y = 0.35 (geometry.scm:178-182)."""
    rays = kat["hits"]["spheres"]
    t07 = [r for r in rays if F(r[2]) == 0.7][0]
    t00 = [r for r in rays if F(r[2]) == 0.0 and r[1] == t07[1]][0]
    assert t07[3] is None and t00[3] is not None


def test_bezier_hits(kat, oracle_mod):
    """Closest hits against two curves (bezier.scm:176-214) through the
    reference's hit-obj-list: t (a distance along unit(dir), Q10), the point
    on the raw ray at that t and the normal -dir (Q12), bit for bit.  The
    rays include the straight-down-z case (get-projection-mat's d = 0 branch)
    and |dir| != 1."""
    from rtamd import scene as g
    lam = g.make_lambertian
    ct = g.constant_texture
    objs = [g.make_bezier((-1, 0, -1), (-0.8, 1, 1), (0.8, -1, 1), (1, 0, -1), 0.1, lam(ct((0.65, 0.05, 0.05)))),
            g.make_bezier((130, 0, 65), (150, 0, 190), (130, 0, 190), (265, 0, 295), 10,
                          lam(ct((0.73, 0.73, 0.73))))]
    sc = g.make_scene(objs, make_camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 90, 1, 0, 1, 0, 1), g.black)
    o = oracle_mod.build_scene(sc)
    rays = kat["hits"]["bezier"]
    assert sum(r[3] is not None for r in rays) >= 40
    for orig, d, tm, rec in rays:
        got = o.hit_world(F(orig), F(d), F(tm))
        if rec is None:
            assert got is None
        else:
            assert got is not None
            assert [got[0]] + list(got[1:4]) + list(got[4:7]) == [F(rec[0])] + F(rec[1]) + F(rec[2])


def test_points_to_bezier(kat):
    """points->bezier (points.scm:28-43): Catmull-Rom control points."""
    from rtamd import points
    k = kat["points_to_bezier"]
    got = points.points_to_bezier([tuple(p) for p in F(k["points"])])
    assert [[list(c) for c in b] for b in got] == [[F(c) for c in b] for b in k["beziers"]]
