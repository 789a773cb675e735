"""pdf.scm light sampling (an extension the reference never
wires): the oracle's g:pdf-value is a normalised density, the mixture path is
finite, and the host rejects lights the extension does not define."""
import math

import numpy as np
import pytest

from rtamd import scene as g
from rtamd import scenes
from rtamd.camera import make_camera


def _uniform_dirs(n, seed):
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(n, 3))
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def _pdf_integral(o_scene, origin, n=200000, seed=1):
    vals = np.array([o_scene.light_pdf_value(origin, tuple(d)) for d in _uniform_dirs(n, seed)])
    return vals.mean() * 4 * math.pi


def test_rect_light_pdf_integrates_to_one(oracle_mod):
    sc = scenes.cornell_mixture(32, 32)
    o = oracle_mod.build_scene(sc)
    est = _pdf_integral(o, (278.0, 100.0, 278.0))
    assert abs(est - 1.0) < 0.03, est


def test_sphere_light_pdf_integrates_to_one(oracle_mod):
    lam = g.make_lambertian(g.constant_texture((0.5, 0.5, 0.5)))
    light = g.make_sphere((0, 3, 0), 0.7, g.make_diffuse_light(g.constant_texture((4, 4, 4))))
    sc = g.make_scene([g.make_sphere((0, -1000, 0), 1000, lam), light],
                      make_camera((0, 1, 5), (0, 1, 0), (0, 1, 0), 40, 1, 0, 1, 0, 1), g.black, light=light)
    o = oracle_mod.build_scene(sc)
    est = _pdf_integral(o, (0.3, 0.5, 0.2))
    assert abs(est - 1.0) < 0.03, est


def test_mixture_render_is_finite(oracle_mod):
    sc = scenes.cornell_mixture(16, 16)
    o = oracle_mod.build_scene(sc)
    acc, _ = o.render(16, 16, 0, 4, 0x5EED0002, nthreads=4)
    assert np.isfinite(acc).all() and (acc > 0).mean() > 0.5


def test_light_must_be_rect_or_sphere():
    lam = g.make_lambertian(g.constant_texture((0.5, 0.5, 0.5)))
    box = g.make_box((0, 0, 0), (1, 1, 1), lam)
    cam = make_camera((0, 1, 5), (0, 1, 0), (0, 1, 0), 40, 1, 0, 1, 0, 1)
    with pytest.raises(ValueError):
        g.make_scene([box], cam, g.black, light=box)
