"""cam:make-camera (camera.scm:63-78) on the host.

The camera is the reference's 10-slot vector (camera.scm:33-61): lower-left
corner, horizontal, vertical, origin, w, u, v, lens radius, time0, time1.
``get-ray`` (camera.scm:80-92) runs on the GPU (k_raygen).
"""
import math

from . import vec as v


class Camera:
    __slots__ = ("llc", "horizontal", "vertical", "origin", "w", "u", "v", "lens_radius", "time0", "time1")

    def slots(self):
        """The 24 doubles rt_set_camera takes (include/rt.h RT_CAMERA_DOUBLES)."""
        out = []
        for vv in (self.llc, self.horizontal, self.vertical, self.origin, self.w, self.u, self.v):
            out.extend(vv)
        out.extend([self.lens_radius, self.time0, self.time1])
        return out


def make_camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist, time0, time1):
    """camera.scm:63-78, in the reference's evaluation order."""
    lookfrom, lookat, vup = v.vec3(*lookfrom), v.vec3(*lookat), v.vec3(*vup)
    theta = float(vfov) * (math.pi / 180.0)
    half_height = math.tan(theta / 2)
    half_width = float(aspect) * half_height
    w = v.unit(v.diff(lookfrom, lookat))
    u = v.unit(v.cross(vup, w))
    vv = v.cross(w, u)
    focus = float(focus_dist)
    c = Camera()
    c.llc = v.diff(lookfrom, v.scale(u, half_width * focus), v.scale(vv, half_height * focus), v.scale(w, focus))
    c.horizontal = v.scale(u, 2 * half_width * focus)
    c.vertical = v.scale(vv, 2 * half_height * focus)
    c.origin = lookfrom
    c.w, c.u, c.v = w, u, vv
    c.lens_radius = float(aperture) / 2
    c.time0, c.time1 = float(time0), float(time1)
    return c


def aspect(nx, ny):
    """(/ *size-x* *size-y*) — an exact rational in the reference, rounded once."""
    return nx / ny
