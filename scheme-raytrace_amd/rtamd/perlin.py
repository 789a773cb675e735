"""Perlin tables (perlin.scm:10-36) generated on the host.

In the reference the tables are drawn from the global RNG when the module is
loaded: 256 `+ranfloat+` draws (unused by noise/turb, but they consume the
stream), 256 random unit vectors (3 draws each, perlin.scm:15-19), then three
Fisher-Yates permutations (i = 255..1, target = floor(xi*(i+1)),
perlin.scm:21-30).  Here the same procedure runs on a HostStream and the
tables are shipped to the GPU as data (LDS-staged by k_shade).
"""
import math

from . import vec as v
from .rng import HostStream


class PerlinTables:
    __slots__ = ("ranfloat", "ranvec", "perm_x", "perm_y", "perm_z")


def _permute(p, n, rr):
    i = n - 1
    while i > 0:                                   # perlin.scm:21-26
        target = math.floor(rr() * (i + 1))
        p[i], p[target] = p[target], p[i]
        i -= 1
    return p


def generate(stream):
    """perlin.scm:32-36 in load order, drawing from ``stream`` (a callable)."""
    t = PerlinTables()
    t.ranfloat = [stream() for _ in range(256)]                    # +ranfloat+
    ranvec = []
    for _ in range(256):                                           # +ranvec+
        a = -1 + 2 * stream()
        b = -1 + 2 * stream()
        c = -1 + 2 * stream()
        ranvec.append(v.unit(v.vec3(a, b, c)))
    t.ranvec = [x for vv in ranvec for x in vv]
    t.perm_x = _permute(list(range(256)), 256, stream)             # +perm-x+
    t.perm_y = _permute(list(range(256)), 256, stream)
    t.perm_z = _permute(list(range(256)), 256, stream)
    return t


def from_seed(seed):
    return generate(HostStream(seed))
