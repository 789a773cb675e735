"""ctypes wrapper of liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker (or the timed CPU baseline).
The oracle is the C f64 restatement of the reference hot path in
oracle/rt_oracle.c (see its header for the reference file:line map).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_L = None
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        V = ctypes.c_void_p
        sig = {
            "orc_scene_new": ([], V),
            "orc_scene_free": ([V], None),
            "orc_add_texture_constant": ([V, _dp], ctypes.c_int),
            "orc_add_texture_checker": ([V, ctypes.c_int, ctypes.c_int], ctypes.c_int),
            "orc_add_texture_noise": ([V, ctypes.c_double], ctypes.c_int),
            "orc_add_texture_marble": ([V, ctypes.c_double], ctypes.c_int),
            "orc_add_material_lambertian": ([V, ctypes.c_int], ctypes.c_int),
            "orc_add_material_metal": ([V, ctypes.c_int, ctypes.c_double], ctypes.c_int),
            "orc_add_material_dielectric": ([V, ctypes.c_double], ctypes.c_int),
            "orc_add_material_diffuse_light": ([V, ctypes.c_int], ctypes.c_int),
            "orc_add_sphere": ([V, _dp, ctypes.c_double, ctypes.c_int], ctypes.c_int),
            "orc_add_moving_sphere": ([V, _dp, _dp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_int], ctypes.c_int),
            "orc_add_rect": ([V, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              ctypes.c_double, ctypes.c_double, ctypes.c_int], ctypes.c_int),
            "orc_add_flip_normals": ([V, ctypes.c_int], ctypes.c_int),
            "orc_add_bezier": ([V, _dp, ctypes.c_double, ctypes.c_int], ctypes.c_int),
            "orc_add_constant_medium": ([V, ctypes.c_int, ctypes.c_double, ctypes.c_int], ctypes.c_int),
            "orc_add_klein": ([V, _dp, ctypes.c_int], ctypes.c_int),
            "orc_add_bezier_array": ([V, _dp, ctypes.c_int, ctypes.c_double, ctypes.c_int], ctypes.c_int),
            "orc_add_box": ([V, _dp, _dp, ctypes.c_int], ctypes.c_int),
            "orc_add_translate": ([V, ctypes.c_int, _dp], ctypes.c_int),
            "orc_add_rotate_y": ([V, ctypes.c_int, ctypes.c_double], ctypes.c_int),
            "orc_add_list": ([V, ctypes.POINTER(ctypes.c_int), ctypes.c_int], ctypes.c_int),
            "orc_add_bvh": ([V, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_double, ctypes.c_double,
                             ctypes.c_int], ctypes.c_int),
            "orc_set_camera": ([V, _dp], None),
            "orc_set_sky": ([V, ctypes.c_int], None),
            "orc_set_light_sampling": ([V, ctypes.c_int], None),
            "orc_light_pdf_value": ([V, _dp, _dp], ctypes.c_double),
            "orc_set_world": ([V, ctypes.c_int], None),
            "orc_set_perlin_tables": ([V, _dp, _ip, _ip, _ip], None),
            "orc_make_camera": ([_dp, _dp, _dp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp], None),
            "orc_render": ([V, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, _dp,
                            ctypes.c_long, ctypes.c_long, ctypes.c_int], ctypes.c_uint64),
            "orc_sample": ([V, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                            ctypes.c_uint32, _dp], None),
            "orc_render_pixels": ([V, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                   _dp, ctypes.POINTER(ctypes.c_uint32), ctypes.c_long, ctypes.c_int],
                                  ctypes.c_uint64),
            "orc_cosine_direction": ([ctypes.c_double, ctypes.c_double, _dp], None),
            "orc_resolve_u8": ([_dp, ctypes.c_long, ctypes.c_int, ctypes.POINTER(ctypes.c_uint8)], None),
            "orc_philox": ([ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_uint32,
                            ctypes.POINTER(ctypes.c_uint32)], None),
            "orc_stream": ([ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                            _dp], None),
            "orc_schlick": ([ctypes.c_double, ctypes.c_double], ctypes.c_double),
            "orc_refract": ([_dp, _dp, ctypes.c_double, _dp], ctypes.c_int),
            "orc_reflect": ([_dp, _dp, _dp], None),
            "orc_noise": ([V, _dp], ctypes.c_double),
            "orc_turb": ([V, _dp], ctypes.c_double),
            "orc_tex_value": ([V, ctypes.c_int, _dp, _dp], None),
            "orc_onb": ([_dp, _dp], None),
            "orc_hit_world": ([V, _dp, _dp, ctypes.c_double, _dp], ctypes.c_int),
            "orc_set_bvh_flat": ([V, ctypes.c_int], None),
            "orc_trace_sample": ([V, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                  ctypes.c_uint32, _dp, ctypes.c_int], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _L = L
    return _L


def _dv(vals):
    return (ctypes.c_double * len(vals))(*[float(x) for x in vals])


class OracleScene:
    """Builder with the same method names as rtamd.gpu.GpuBuilder."""

    def __init__(self):
        self.L = lib()
        self.s = self.L.orc_scene_new()

    def __del__(self):
        try:
            self.L.orc_scene_free(self.s)
        except Exception:
            pass

    def texture_constant(self, rgb):
        return self.L.orc_add_texture_constant(self.s, _dv(rgb))

    def texture_checker(self, even, odd):
        return self.L.orc_add_texture_checker(self.s, even, odd)

    def texture_noise(self, sc):
        return self.L.orc_add_texture_noise(self.s, sc)

    def texture_marble(self, sc):
        return self.L.orc_add_texture_marble(self.s, sc)

    def material_lambertian(self, tex):
        return self.L.orc_add_material_lambertian(self.s, tex)

    def material_metal(self, tex, fuzz):
        return self.L.orc_add_material_metal(self.s, tex, fuzz)

    def material_dielectric(self, r):
        return self.L.orc_add_material_dielectric(self.s, r)

    def material_diffuse_light(self, tex):
        return self.L.orc_add_material_diffuse_light(self.s, tex)

    def sphere(self, c, r, mat):
        return self.L.orc_add_sphere(self.s, _dv(c), r, mat)

    def moving_sphere(self, c0, c1, t0, t1, r, mat):
        return self.L.orc_add_moving_sphere(self.s, _dv(c0), _dv(c1), t0, t1, r, mat)

    def rect(self, axis, a0, a1, b0, b1, k, mat):
        return self.L.orc_add_rect(self.s, axis, a0, a1, b0, b1, k, mat)

    def flip_normals(self, o):
        return self.L.orc_add_flip_normals(self.s, o)

    def klein(self, center, mat):
        return self.L.orc_add_klein(self.s, _dv(center), mat)

    def constant_medium(self, boundary, density, tex):
        return self.L.orc_add_constant_medium(self.s, boundary, density, tex)

    def bezier_array(self, cps, width, mat):
        import numpy as np
        arr = np.ascontiguousarray(cps, dtype=np.float64)
        return self.L.orc_add_bezier_array(self.s, arr.ctypes.data_as(_dp), int(arr.shape[0]), width, mat)

    def bezier(self, a, b, c, d, width, mat):
        return self.L.orc_add_bezier(self.s, _dv(list(a) + list(b) + list(c) + list(d)), width, mat)

    def box(self, p0, p1, mat):
        return self.L.orc_add_box(self.s, _dv(p0), _dv(p1), mat)

    def translate(self, o, off):
        return self.L.orc_add_translate(self.s, o, _dv(off))

    def rotate_y(self, o, angle):
        return self.L.orc_add_rotate_y(self.s, o, angle)

    def list(self, objs):
        arr = (ctypes.c_int * max(1, len(objs)))(*objs)
        return self.L.orc_add_list(self.s, arr, len(objs))

    def bvh(self, objs, t0, t1, sah):
        arr = (ctypes.c_int * max(1, len(objs)))(*objs)
        return self.L.orc_add_bvh(self.s, arr, len(objs), t0, t1, sah)

    def set_camera(self, slots):
        self.L.orc_set_camera(self.s, _dv(slots))

    def set_light(self, obj):
        self.L.orc_set_light_sampling(self.s, obj)

    def light_pdf_value(self, o, v):
        return self.L.orc_light_pdf_value(self.s, _dv(o), _dv(v))

    def set_bvh_flat(self, flat):
        """True: evaluate every BVH as the flat list it restates (no tree)."""
        self.L.orc_set_bvh_flat(self.s, 1 if flat else 0)

    def set_sky(self, code):
        self.L.orc_set_sky(self.s, code)

    def set_perlin(self, ranvec, px, py, pz):
        i32 = ctypes.c_int32 * 256
        self.L.orc_set_perlin_tables(self.s, _dv(ranvec), i32(*px), i32(*py), i32(*pz))

    def commit(self, world):
        self.L.orc_set_world(self.s, world)
        return self

    # ---- rendering / probes
    def render(self, nx, ny, spp_begin, spp_count, seed, accum=None, pix_begin=0, pix_end=-1, nthreads=1):
        if accum is None:
            accum = np.zeros(nx * ny * 3, dtype=np.float64)
        assert accum.dtype == np.float64 and accum.flags.c_contiguous and accum.size == nx * ny * 3
        segs = self.L.orc_render(self.s, nx, ny, spp_begin, spp_count, seed & (2**64 - 1),
                                 accum.ctypes.data_as(_dp), pix_begin, pix_end, nthreads)
        return accum, segs

    def render_pixels(self, nx, ny, spp_begin, spp_count, seed, accum, pix, nthreads=1):
        pix = np.ascontiguousarray(pix, dtype=np.uint32)
        return self.L.orc_render_pixels(self.s, nx, ny, spp_begin, spp_count, seed & (2**64 - 1),
                                        accum.ctypes.data_as(_dp), pix.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                        pix.size, nthreads)

    def sample(self, nx, ny, x, y, seed, smp):
        out = (ctypes.c_double * 3)()
        self.L.orc_sample(self.s, nx, ny, x, y, seed, smp, out)
        return tuple(out)

    def trace_sample(self, nx, ny, x, y, seed, smp, cap=128):
        """Debugging aid: the sample's path as rows (o3, d3, hit, t, p3, mat, draw counter)."""
        out = np.zeros(13 * cap)
        n = self.L.orc_trace_sample(self.s, nx, ny, x, y, seed, smp, out.ctypes.data_as(_dp), cap)
        return out[:13 * n].reshape(n, 13)

    def hit_world(self, o, d, time=0.0):
        out = (ctypes.c_double * 8)()
        ok = self.L.orc_hit_world(self.s, _dv(o), _dv(d), time, out)
        return (tuple(out) if ok else None)

    def noise(self, p):
        return self.L.orc_noise(self.s, _dv(p))

    def turb(self, p):
        return self.L.orc_turb(self.s, _dv(p))

    def tex_value(self, tex, p):
        out = (ctypes.c_double * 3)()
        self.L.orc_tex_value(self.s, tex, _dv(p), out)
        return tuple(out)


def build_scene(scene):
    """Emit an rtamd Scene descriptor graph into a new oracle scene."""
    from rtamd.scene import emit
    return emit(scene, OracleScene())


def resolve_u8(accum, count):
    out = np.zeros(accum.size, dtype=np.uint8)
    lib().orc_resolve_u8(np.ascontiguousarray(accum).ctypes.data_as(_dp), accum.size // 3, count,
                         out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return out


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    o = (ctypes.c_uint32 * 4)()
    lib().orc_philox(c, key[0], key[1], o)
    return tuple(o)


def stream(seed, pix, smp, first, n):
    out = (ctypes.c_double * n)()
    lib().orc_stream(seed, pix, smp, first, n, out)
    return list(out)


def schlick(c, r):
    return lib().orc_schlick(c, r)


def refract(v, n, ni):
    out = (ctypes.c_double * 3)()
    ok = lib().orc_refract(_dv(v), _dv(n), ni, out)
    return tuple(out) if ok else None


def reflect(v, n):
    out = (ctypes.c_double * 3)()
    lib().orc_reflect(_dv(v), _dv(n), out)
    return tuple(out)


def onb(n):
    out = (ctypes.c_double * 9)()
    lib().orc_onb(_dv(n), out)
    return tuple(out[0:3]), tuple(out[3:6]), tuple(out[6:9])


def make_camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus, t0, t1):
    out = (ctypes.c_double * 24)()
    lib().orc_make_camera(_dv(lookfrom), _dv(lookat), _dv(vup), vfov, aspect, aperture, focus, t0, t1, out)
    return list(out)


def cosine_direction(r1, r2):
    out = (ctypes.c_double * 3)()
    lib().orc_cosine_direction(r1, r2, out)
    return tuple(out)
