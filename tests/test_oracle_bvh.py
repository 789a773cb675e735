"""The oracle's BVH trees against the flat list they restate (CPU).

An OBJ_BVH (g:make-bvh-node geometry.scm:226-260, g:make-bvh-with-sah
:294-371) is, in the oracle, the closest-hit list of its objects
(hit-obj-list :33-50).  oracle/rt_oracle.c evaluates it through a
conservative f64 tree so that C5 (2^20 curves) can be checked at all; these
tests require the tree to return exactly what the flat list returns — the
same record, tie-breaks included — on the reference-fixture scenes, on C5's
generator at a size the flat list can still render, and on scenes built to
collide: duplicated spheres and curves (ties in t), moving spheres under a
shutter that does not start at 0, rays with |dir| < 1 and zero components.
"""
import math

import numpy as np
import pytest

from rtamd import scenes
from rtamd import scene as g
from rtamd import vec as v
from rtamd.camera import make_camera


def _render_both(oracle_mod, scene, nx, ny, spp, seed=0x5EED0002):
    o = oracle_mod.build_scene(scene)
    o.set_bvh_flat(False)
    tree, s1 = o.render(nx, ny, 0, spp, seed, nthreads=8)
    o.set_bvh_flat(True)
    flat, s2 = o.render(nx, ny, 0, spp, seed, nthreads=8)
    return tree, flat, s1, s2


@pytest.mark.parametrize("name,nx,ny,spp", [("bvh_sah", 48, 27, 2), ("test_bezier", 40, 24, 2),
                                            ("cornell_bezier", 32, 32, 2), ("curves_small", 48, 27, 1)])
def test_tree_equals_flat_list_bitwise(oracle_mod, name, nx, ny, spp):
    tree, flat, s1, s2 = _render_both(oracle_mod, scenes.SCENES[name](nx, ny), nx, ny, spp)
    assert s1 == s2
    assert np.array_equal(tree, flat)


def _collision_scene(nx, ny):
    """Spheres, moving spheres and curves in one BVH, each duplicated, some
    shifted by one ulp; a camera shutter over [0.25, 0.75]."""
    rng = np.random.default_rng(7)
    mats = [g.make_lambertian(g.constant_texture(v.vec3(0.3 + 0.1 * i, 0.5, 0.2))) for i in range(4)]
    objs = []
    for i in range(60):
        c = rng.uniform(-3, 3, 3)
        c[1] = abs(c[1]) * 0.3
        r = float(rng.uniform(0.1, 0.5))
        m = mats[i % 4]
        if i % 3 == 0:
            c1 = c + np.array([0.0, float(rng.uniform(0, 0.6)), 0.0])
            a = g.make_moving_sphere(v.vec3(*c), v.vec3(*c1), 0.0, 1.0, r, m)
            objs += [a, g.make_moving_sphere(v.vec3(*c), v.vec3(*c1), 0.0, 1.0, r, mats[(i + 1) % 4])]
        else:
            objs += [g.make_sphere(v.vec3(*c), r, m), g.make_sphere(v.vec3(*c), r, mats[(i + 2) % 4])]
            if i % 5 == 0:
                objs.append(g.make_sphere(v.vec3(math.nextafter(c[0], 9), c[1], c[2]), r, mats[(i + 3) % 4]))
    cps = rng.uniform(-3, 3, (40, 12))
    cps[:, 1::3] = np.abs(cps[:, 1::3]) * 0.5
    objs.append(g.bezier_array(cps, 0.2, mats[1]))
    objs.append(g.bezier_array(cps[:20].copy(), 0.2, mats[2]))       # the same curves again: exact ties
    cam = make_camera(v.vec3(0, 2, 9), v.vec3(0, 0.3, 0), v.vec3(0, 1, 0), 40, nx / ny, 0.05, 9.0, 0.25, 0.75)
    ground = g.make_sphere(v.vec3(0, -1000, 0), 1000, mats[3])
    return g.make_scene([ground, g.make_bvh_with_sah(objs, 0, 0)], cam, g.sky_color)


def test_tree_equals_flat_list_on_collisions(oracle_mod):
    nx, ny = 40, 24
    tree, flat, s1, s2 = _render_both(oracle_mod, _collision_scene(nx, ny), nx, ny, 3)
    assert s1 == s2
    assert np.array_equal(tree, flat)


def test_tree_equals_flat_list_per_ray(oracle_mod):
    """hit_world records for rays of every kind: unit and raw directions,
    |dir| < 1 (a curve reports distance along unit(dir)), axis-parallel
    directions (zero components), times 0 and inside the shutter."""
    o = oracle_mod.build_scene(_collision_scene(40, 24))
    rng = np.random.default_rng(11)
    rays = []
    for k in range(3000):
        orig = rng.uniform(-4, 4, 3) + np.array([0, 1.5, 0])
        d = rng.normal(size=3)
        if k % 4 == 1:
            d *= 0.05                               # |dir| << 1
        elif k % 4 == 2:
            d[rng.integers(3)] = 0.0                # a zero component
        elif k % 4 == 3:
            d = np.zeros(3)
            d[rng.integers(3)] = rng.choice([-1.0, 1.0]) * rng.uniform(0.3, 2)
        rays.append((orig, d, [0.0, 0.25, 0.5, 0.75][k % 4]))
    hits = 0
    for orig, d, t in rays:
        o.set_bvh_flat(False)
        a = o.hit_world(orig, d, t)
        o.set_bvh_flat(True)
        b = o.hit_world(orig, d, t)
        assert a == b, (orig, d, t, a, b)
        hits += a is not None
    assert hits > 1000


def test_c5_band_tree_runs(oracle_mod):
    """C5 at its full 2^20 curves: the tree makes a band of pixels renderable
    (the flat list would test every curve per segment)."""
    nx, ny = 1920, 1080
    o = oracle_mod.build_scene(scenes.cornell_curves(nx, ny))
    acc = np.zeros(nx * ny * 3)
    lo = 540 * nx + 900
    _, segs = o.render(nx, ny, 0, 1, 0x5EED0002, acc, lo, lo + 64, 8)
    assert segs >= 64 and np.isfinite(acc).all()
