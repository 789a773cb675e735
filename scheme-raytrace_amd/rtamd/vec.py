"""vec.scm (vec.scm:7-70) on the host: 3-vectors of f64.

Used host-side only (scene generation, camera construction).  Each function
keeps the reference's evaluation order: ``sum``/``diff`` are left folds of
f64vector-add/-sub, ``unit`` multiplies by 1/|v| (not a division), ``dot``
accumulates from 0.0 left to right.  Python floats are IEEE doubles and
``math`` calls the platform libm, as Gauche does.
"""
import math


def vec3(x, y, z):
    """vec.scm:7 — an f64vector of three elements."""
    return (float(x), float(y), float(z))


def x(v):
    return v[0]


def y(v):
    return v[1]


def z(v):
    return v[2]


def _num(k):
    return float(k)


def sum(*vs):  # noqa: A001 - mirrors v:sum
    """vec.scm:20-24 (reduce f64vector-add #f64(0 0 0) vs)."""
    if not vs:
        return (0.0, 0.0, 0.0)
    acc = vs[0]
    for v in vs[1:]:
        acc = (acc[0] + v[0], acc[1] + v[1], acc[2] + v[2])
    return acc


def diff(v1, *vs):
    """vec.scm:26-33 left fold of f64vector-sub."""
    acc = v1
    for v in vs:
        acc = (acc[0] - v[0], acc[1] - v[1], acc[2] - v[2])
    return acc


def scale(v, k):
    """vec.scm:41 (f64vector-mul v k): k a scalar or a vector."""
    if isinstance(k, tuple):
        return (v[0] * k[0], v[1] * k[1], v[2] * k[2])
    k = _num(k)
    return (v[0] * k, v[1] * k, v[2] * k)


def prod(a, b):
    return (a[0] * b[0], a[1] * b[1], a[2] * b[2])


def dot(a, b):
    """f64vector-dot: r = 0.0; r += a_i * b_i."""
    r = 0.0
    r += a[0] * b[0]
    r += a[1] * b[1]
    r += a[2] * b[2]
    return r


def length(v):
    return math.sqrt(dot(v, v))


def unit(v):
    """vec.scm:60-62 — v * (1/|v|)."""
    k = 1.0 / length(v)
    return scale(v, k)


def cross(a, b):
    """vec.scm:64-70."""
    return (a[1] * b[2] - b[1] * a[2],
            a[2] * b[0] - b[2] * a[0],
            a[0] * b[1] - b[0] * a[1])
