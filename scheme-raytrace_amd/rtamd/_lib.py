"""ctypes binding of librtamd.so (the C ABI declared in include/rt.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C scheme-raytrace_amd/csrc``).  There is no fallback: if the library
is missing every entry point raises, so a GPU run can never silently take a
CPU path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RTAMD_LIB selects an alternative in-tree build (e.g. an A/B variant)
LIB_PATH = os.environ.get("RTAMD_LIB") or os.path.join(_HERE, "librtamd.so")

_c_int_p = ctypes.POINTER(ctypes.c_int)
_c_double_p = ctypes.POINTER(ctypes.c_double)
_c_i32_p = ctypes.POINTER(ctypes.c_int32)
_c_u8_p = ctypes.POINTER(ctypes.c_uint8)

RT_CAMERA_DOUBLES = 24
RT_SKY_GRADIENT, RT_SKY_BLACK = 0, 1
RT_RECT_XY, RT_RECT_XZ, RT_RECT_YZ = 0, 1, 2
#: render-schedule options of a context (include/rt.h RT_OPT_*; 0 = automatic)
RT_OPTIONS = {"lanes": 1, "max_paths": 2, "tail_paths": 3, "tail_div": 4, "tail_off": 5, "exact_libm": 6}
#: RT_OPT_EXACT_LIBM values: auto (exact in scenes with curves or noise / marble textures), exact (the C
#: library's sin / cos bit for bit), device (the device library's)
RT_LIBM = {"auto": 0, "exact": 1, "device": 2}
RT_COMM_ID_BYTES = 128


class RtStats(ctypes.Structure):
    _fields_ = [
        ("segments", ctypes.c_uint64),
        ("paths", ctypes.c_uint64),
        ("ms_total", ctypes.c_double),
        ("ms_extend", ctypes.c_double),
        ("ms_shade", ctypes.c_double),
        ("extend_launches", ctypes.c_uint64),
        ("extend_rays", ctypes.c_uint64),
        ("max_depth_seen", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("ms_finish", ctypes.c_double),
        ("finish_paths", ctypes.c_uint64),
        ("shade_hits_d0", ctypes.c_uint64),
        ("shade_hits", ctypes.c_uint64),
        ("shade_survivors", ctypes.c_uint64),
        ("chunks", ctypes.c_uint32),
        ("lanes", ctypes.c_uint32),
        ("curve_pooled_batches", ctypes.c_uint64),
        ("curve_flat_pooled", ctypes.c_uint64),
    ]


class RtSceneInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("leaves", "groups", "bvh_nodes", "bvh0_nodes", "tree_depth",
                                              "bvh_solo")] + \
               [(n, ctypes.c_uint32) for n in ("extend_lds_bytes", "extend_lds_blocks", "camera_lds_bytes",
                                               "camera_lds_blocks")] + \
               [("cus", ctypes.c_int32), ("curve_stack", ctypes.c_int32), ("commit_ms", ctypes.c_double),
                ("commit_upload_ms", ctypes.c_double), ("commit_sah_ms", ctypes.c_double),
                ("commit_threads", ctypes.c_int32), ("reserved0", ctypes.c_int32)]


# name -> argtypes (restype is always c_int status, except where noted)
_SIGNATURES = {
    "rt_abi_version": [],
    "rt_device_count": [_c_int_p],
    "rt_context_create": [ctypes.c_int, _c_int_p],
    "rt_context_destroy": [ctypes.c_int],
    "rt_context_release_pools": [ctypes.c_int],
    "rt_context_set_option": [ctypes.c_int, ctypes.c_int, ctypes.c_int64],
    "rt_context_get_option": [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)],
    "rt_hit_rays": [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                    ctypes.POINTER(ctypes.c_int32)],
    "rt_scene_begin": [ctypes.c_int, _c_int_p],
    "rt_scene_destroy": [ctypes.c_int],
    "rt_add_texture_constant": [ctypes.c_int, _c_double_p, _c_int_p],
    "rt_add_texture_checker": [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_int_p],
    "rt_add_texture_noise": [ctypes.c_int, ctypes.c_double, _c_int_p],
    "rt_add_texture_marble": [ctypes.c_int, ctypes.c_double, _c_int_p],
    "rt_add_material_lambertian": [ctypes.c_int, ctypes.c_int, _c_int_p],
    "rt_add_material_metal": [ctypes.c_int, ctypes.c_int, ctypes.c_double, _c_int_p],
    "rt_add_material_dielectric": [ctypes.c_int, ctypes.c_double, _c_int_p],
    "rt_add_material_diffuse_light": [ctypes.c_int, ctypes.c_int, _c_int_p],
    "rt_add_sphere": [ctypes.c_int, _c_double_p, ctypes.c_double, ctypes.c_int, _c_int_p],
    "rt_add_moving_sphere": [ctypes.c_int, _c_double_p, _c_double_p, ctypes.c_double, ctypes.c_double,
                             ctypes.c_double, ctypes.c_int, _c_int_p],
    "rt_add_rect": [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                    ctypes.c_double, ctypes.c_double, ctypes.c_int, _c_int_p],
    "rt_add_bezier": [ctypes.c_int, _c_double_p, _c_double_p, _c_double_p, _c_double_p, ctypes.c_double,
                      ctypes.c_int, _c_int_p],
    "rt_add_bezier_array": [ctypes.c_int, _c_double_p, ctypes.c_int, ctypes.c_double, ctypes.c_int, _c_int_p],
    "rt_add_flip_normals": [ctypes.c_int, ctypes.c_int, _c_int_p],
    "rt_add_constant_medium": [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, _c_int_p],
    "rt_add_klein": [ctypes.c_int, _c_double_p, ctypes.c_int, _c_int_p],
    "rt_add_box": [ctypes.c_int, _c_double_p, _c_double_p, ctypes.c_int, _c_int_p],
    "rt_add_translate": [ctypes.c_int, ctypes.c_int, _c_double_p, _c_int_p],
    "rt_add_rotate_y": [ctypes.c_int, ctypes.c_int, ctypes.c_double, _c_int_p],
    "rt_add_list": [ctypes.c_int, _c_int_p, ctypes.c_int, _c_int_p],
    "rt_add_bvh": [ctypes.c_int, _c_int_p, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                   _c_int_p],
    "rt_make_camera": [_c_double_p, _c_double_p, _c_double_p, ctypes.c_double, ctypes.c_double,
                       ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, _c_double_p],
    "rt_set_camera": [ctypes.c_int, _c_double_p],
    "rt_set_sky": [ctypes.c_int, ctypes.c_int],
    "rt_set_light_sampling": [ctypes.c_int, ctypes.c_int],
    "rt_set_perlin_tables": [ctypes.c_int, _c_double_p, _c_i32_p, _c_i32_p, _c_i32_p],
    "rt_scene_commit": [ctypes.c_int, ctypes.c_int],
    "rt_render": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                  _c_double_p],
    "rt_render_device": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                         ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p],
    "rt_render_rows": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                       ctypes.c_int, ctypes.c_uint64, _c_double_p],
    "rt_render_rows_device": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p],
    "rt_trace_line": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                      _c_double_p, _c_u8_p],
    "rt_render_shard_device": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p],
    "rt_get_stats": [ctypes.c_int, ctypes.POINTER(RtStats)],
    "rt_set_profiling": [ctypes.c_int, ctypes.c_int],
    "rt_get_scene_info": [ctypes.c_int, ctypes.POINTER(RtSceneInfo)],
    "rt_resolve_u8": [_c_double_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_u8_p],
    "rt_shard_pixels": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32),
                        ctypes.POINTER(ctypes.c_int64)],
    "rt_resolve_u8_device": [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_void_p],
    "rt_curve_depth_probe": [ctypes.c_int, ctypes.c_int, _c_double_p, _c_double_p, _c_i32_p],
    "rt_comm_unique_id": [ctypes.POINTER(ctypes.c_uint8)],
    "rt_comm_create": [ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_int, _c_int_p],
    "rt_comm_destroy": [ctypes.c_int],
    "rt_gather_shards": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
    "rt_gather_layout": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                         ctypes.POINTER(ctypes.c_int64)],
    "rt_gather_shards_local": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_void_p],
}

#: every symbol include/rt.h declares (tests check the .so exports all of them)
EXPORTED = sorted(list(_SIGNATURES) + ["rt_last_error"])

_lib = None


class RtError(RuntimeError):
    """A nonzero status from librtamd; the message is rt_last_error()."""


def lib():
    """Load librtamd.so once.  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm bundles its own
    # libamdhip64.so.  Loading torch first makes librtamd bind to that copy, so
    # device pointers and streams from torch tensors are valid here (torch is
    # the plumbing for device memory / streams / RCCL, never the compute).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RtError(
            "librtamd.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the GPU path has no fallback)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    for name, argtypes in _SIGNATURES.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    L.rt_last_error.argtypes = []
    L.rt_last_error.restype = ctypes.c_char_p
    _lib = L
    return L


def check(status):
    if status != 0:
        msg = lib().rt_last_error()
        raise RtError(msg.decode() if msg else "librtamd error %d" % status)


def call(name, *args):
    check(getattr(lib(), name)(*args))


def dvec(values):
    arr = (ctypes.c_double * len(values))(*[float(v) for v in values])
    return arr


def out_int():
    return ctypes.c_int(0)
