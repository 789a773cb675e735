"""rtamd — host side of the MI355X wavefront path tracer.

Mirrors the reference's Scheme API (soma-arc/scheme-raytrace): the scene /
camera / material / texture constructors keep their names and arities
(``rtamd.scene``: g:/m:/t: prefixes collapse into one module; ``rtamd.camera``
for cam:), ``rtamd.render.Renderer`` is trace-all / save-as-ppm, and the
closest-hit + shading loop runs in librtamd's HIP kernels for gfx950.
"""
from . import vec, rng, scene, camera, perlin, scenes  # noqa: F401

__all__ = ["vec", "rng", "scene", "camera", "perlin", "scenes", "gpu", "render"]


def __getattr__(name):
    # gpu / render import numpy + ctypes-load lazily; the library is required
    if name in ("gpu", "render"):
        import importlib
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
