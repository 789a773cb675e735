"""points.scm on the host: polylines read from CSV, turned into Catmull-Rom
style cubic Bezier segments (tightness 0.5) and then into curve objects.

Mirrors points.scm:10-57 (same names with Python spelling).  The arithmetic
keeps the reference's order: d1 = (p2 - pt) * (1/6), d2 = (p3 - p1) * (1/6),
control points (p1, p1 + d1, p2 - d2, p2).
"""
from . import scene as g
from . import vec as v


def load_points(file_name, magnitude):
    """load-points (points.scm:10-19): one "x,y,z" point per line, each
    coordinate multiplied by ``magnitude``."""
    pts = []
    with open(file_name) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            pts.append(v.vec3(*[magnitude * _number(p) for p in line.split(",")]))
    return pts


def _number(s):
    s = s.strip()
    try:
        return int(s)
    except ValueError:
        return float(s)


def calc_bezier_cp(pt, p1, p2, p3):
    """calc-bezier-cp (points.scm:22-26)."""
    d1 = v.scale(v.diff(p2, pt), 1 / 6)
    d2 = v.scale(v.diff(p3, p1), 1 / 6)
    return [p1, v.sum(p1, d1), v.diff(p2, d2), p2]


def points_to_bezier(points):
    """points->bezier (points.scm:28-43): one segment between points i and
    i+1 for i = 1 .. len-3 (the first and last points only steer tangents)."""
    last = len(points) - 2
    return [calc_bezier_cp(points[i - 1], points[i], points[i + 1], points[i + 2]) for i in range(1, max(1, last))]


def bezier_to_objs(beziers, width, material):
    """bezier->objs (points.scm:45-53)."""
    return [g.make_bezier(b[0], b[1], b[2], b[3], width, material) for b in beziers]
