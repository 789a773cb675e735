"""Device side of the drop-in: contexts, scene upload and rendering through
librtamd's C ABI.  There is no CPU fallback anywhere in this module."""
import contextlib
import ctypes

import numpy as np

from . import _lib
from ._lib import call, dvec, out_int
from .scene import emit

_default_ctx = {}


class Context:
    """A librtamd context on one HIP device (rt_context_create)."""

    def __init__(self, device=0):
        h = out_int()
        call("rt_context_create", int(device), ctypes.byref(h))
        self.handle = h.value
        self.device = device

    def set_option(self, name, value):
        """rt_context_set_option: a render-schedule option (_lib.RT_OPTIONS:
        lanes, max_paths, tail_paths, tail_div, tail_off); 0 = automatic.
        No schedule option changes an image, only how the work is scheduled.
        exact_libm (value or a _lib.RT_LIBM name: auto / exact / device)
        selects the bounce directions' sin / cos."""
        if name == "exact_libm" and isinstance(value, str):
            value = _lib.RT_LIBM[value]
        call("rt_context_set_option", self.handle, _lib.RT_OPTIONS[name], int(value))

    def get_option(self, name):
        v = ctypes.c_int64(0)
        call("rt_context_get_option", self.handle, _lib.RT_OPTIONS[name], ctypes.byref(v))
        return v.value

    @contextlib.contextmanager
    def options(self, **kv):
        """Set options for the duration of a with-block, then restore them."""
        old = {k: self.get_option(k) for k in kv}
        try:
            for k, val in kv.items():
                self.set_option(k, val)
            yield self
        finally:
            for k, val in old.items():
                self.set_option(k, val)

    def reset_options(self):
        for k in _lib.RT_OPTIONS:
            self.set_option(k, 0)

    def release_pools(self):
        """rt_context_release_pools: free the render lanes' path pools (the
        next render on this context allocates and sizes them again)."""
        call("rt_context_release_pools", self.handle)

    def close(self):
        if self.handle:
            call("rt_context_destroy", self.handle)
            self.handle = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def default_context(device=0):
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


def device_count():
    n = out_int()
    call("rt_device_count", ctypes.byref(n))
    return n.value


class GpuBuilder:
    """Replays a scene descriptor graph into rt_add_* calls (scene.emit)."""

    def __init__(self, ctx):
        h = out_int()
        call("rt_scene_begin", ctx.handle, ctypes.byref(h))
        self.scene = h.value

    def _out(self, name, *args):
        o = out_int()
        call(name, self.scene, *args, ctypes.byref(o))
        return o.value

    def texture_constant(self, rgb):
        return self._out("rt_add_texture_constant", dvec(rgb))

    def texture_checker(self, even, odd):
        return self._out("rt_add_texture_checker", even, odd)

    def texture_noise(self, sc):
        return self._out("rt_add_texture_noise", sc)

    def texture_marble(self, sc):
        return self._out("rt_add_texture_marble", sc)

    def material_lambertian(self, tex):
        return self._out("rt_add_material_lambertian", tex)

    def material_metal(self, tex, fuzz):
        return self._out("rt_add_material_metal", tex, fuzz)

    def material_dielectric(self, ref_idx):
        return self._out("rt_add_material_dielectric", ref_idx)

    def material_diffuse_light(self, tex):
        return self._out("rt_add_material_diffuse_light", tex)

    def sphere(self, c, r, mat):
        return self._out("rt_add_sphere", dvec(c), r, mat)

    def moving_sphere(self, c0, c1, t0, t1, r, mat):
        return self._out("rt_add_moving_sphere", dvec(c0), dvec(c1), t0, t1, r, mat)

    def rect(self, axis, a0, a1, b0, b1, k, mat):
        return self._out("rt_add_rect", axis, a0, a1, b0, b1, k, mat)

    def bezier(self, a, b, c, d, width, mat):
        return self._out("rt_add_bezier", dvec(a), dvec(b), dvec(c), dvec(d), width, mat)

    def bezier_array(self, cps, width, mat):
        """cps: contiguous float64 array of shape (n, 12); returns the first id."""
        cps = np.ascontiguousarray(cps, dtype=np.float64)
        ptr = cps.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        return self._out("rt_add_bezier_array", ptr, int(cps.shape[0]), width, mat)

    def klein(self, center, mat):
        return self._out("rt_add_klein", dvec(center), mat)

    def constant_medium(self, boundary, density, tex):
        return self._out("rt_add_constant_medium", boundary, density, tex)

    def flip_normals(self, obj):
        return self._out("rt_add_flip_normals", obj)

    def box(self, p0, p1, mat):
        return self._out("rt_add_box", dvec(p0), dvec(p1), mat)

    def translate(self, obj, off):
        return self._out("rt_add_translate", obj, dvec(off))

    def rotate_y(self, obj, angle):
        return self._out("rt_add_rotate_y", obj, angle)

    def list(self, objs):
        arr = (ctypes.c_int * max(1, len(objs)))(*objs)
        return self._out("rt_add_list", arr, len(objs))

    def bvh(self, objs, t0, t1, sah):
        arr = (ctypes.c_int * max(1, len(objs)))(*objs)
        return self._out("rt_add_bvh", arr, len(objs), t0, t1, sah)

    def set_camera(self, slots):
        call("rt_set_camera", self.scene, dvec(slots))

    def set_light(self, obj):
        call("rt_set_light_sampling", self.scene, obj)

    def set_sky(self, code):
        call("rt_set_sky", self.scene, code)

    def set_perlin(self, ranvec, px, py, pz):
        i32 = ctypes.c_int32 * 256
        call("rt_set_perlin_tables", self.scene, dvec(ranvec), i32(*px), i32(*py), i32(*pz))

    def commit(self, world):
        call("rt_scene_commit", self.scene, world)
        return self.scene


def upload(scene, ctx=None):
    """Commit a scene (rtamd.scene.Scene) on ctx; cached per context."""
    ctx = ctx or default_context()
    h = scene._handles.get(ctx.handle)
    if h is None:
        h = emit(scene, GpuBuilder(ctx))
        scene._handles[ctx.handle] = h
    return h


def stats(scene_handle):
    s = _lib.RtStats()
    call("rt_get_stats", scene_handle, ctypes.byref(s))
    return s


def scene_info(scene_handle):
    """rt_get_scene_info as a dict (tree sizes, LDS kernel footprints and grids)."""
    s = _lib.RtSceneInfo()
    call("rt_get_scene_info", scene_handle, ctypes.byref(s))
    return {name: getattr(s, name) for name, _ in s._fields_ if name != "reserved"}


def render_host(scene, nx, ny, spp_begin, spp_count, seed, accum, ctx=None):
    """rt_render: accum is a host float64 array of nx*ny*3 (updated in place)."""
    h = upload(scene, ctx)
    a = np.ascontiguousarray(accum, dtype=np.float64)
    if a.size != nx * ny * 3:
        raise ValueError("accum must have nx*ny*3 elements")
    call("rt_render", h, nx, ny, spp_begin, spp_count, ctypes.c_uint64(seed & (2**64 - 1)),
         a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if a is not accum:
        accum[...] = a.reshape(accum.shape)
    return h


def render_device(scene, nx, ny, spp_begin, spp_count, seed, accum_ptr, shard=0, nshard=1, stream=None,
                  ctx=None):
    """rt_render_device: accum_ptr is a device pointer (int) to nx*ny*3 doubles."""
    h = upload(scene, ctx)
    call("rt_render_device", h, nx, ny, spp_begin, spp_count, ctypes.c_uint64(seed & (2**64 - 1)), shard,
         nshard, ctypes.c_void_p(accum_ptr), ctypes.c_void_p(stream or 0))
    return h


def render_rows_device(scene, nx, ny, y_begin, y_count, spp_begin, spp_count, seed, accum_ptr, stream=None,
                       ctx=None):
    """rt_render_rows_device: passes of rows [y_begin, y_begin+y_count) into a full-frame device accumulator."""
    h = upload(scene, ctx)
    call("rt_render_rows_device", h, nx, ny, y_begin, y_count, spp_begin, spp_count,
         ctypes.c_uint64(seed & (2**64 - 1)), ctypes.c_void_p(accum_ptr), ctypes.c_void_p(stream or 0))
    return h


def render_rows_host(scene, nx, ny, y_begin, y_count, spp_begin, spp_count, seed, accum, ctx=None):
    """rt_render_rows: as render_rows_device on a host float64 frame (only the band crosses PCIe)."""
    h = upload(scene, ctx)
    if accum.dtype != np.float64 or not accum.flags.c_contiguous or accum.size != nx * ny * 3:
        raise ValueError("accum must be a contiguous float64 array of nx*ny*3 elements")
    call("rt_render_rows", h, nx, ny, y_begin, y_count, spp_begin, spp_count, ctypes.c_uint64(seed & (2**64 - 1)),
         accum.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return h


def trace_line(scene, nx, ny, y, sample_count, seed, raw_data, image, ctx=None):
    """rt_trace_line (main.scm:452-469): pass `sample_count` of row y into raw_data, row y of image resolved."""
    h = upload(scene, ctx)
    if raw_data.dtype != np.float64 or not raw_data.flags.c_contiguous or raw_data.size != nx * ny * 3:
        raise ValueError("raw_data must be a contiguous float64 array of nx*ny*3 elements")
    if image.dtype != np.uint8 or not image.flags.c_contiguous or image.size != nx * ny * 3:
        raise ValueError("image must be a contiguous uint8 array of nx*ny*3 elements")
    call("rt_trace_line", h, nx, ny, y, sample_count, ctypes.c_uint64(seed & (2**64 - 1)),
         raw_data.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
         image.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return h


def render_shard_device(scene, nx, ny, spp_begin, spp_count, seed, shard, nshard, accum_ptr, stream=None, ctx=None):
    """rt_render_shard_device: one shard's tiles into a compact device accumulator (shard_pixels order)."""
    h = upload(scene, ctx)
    call("rt_render_shard_device", h, nx, ny, spp_begin, spp_count, ctypes.c_uint64(seed & (2**64 - 1)), shard,
         nshard, ctypes.c_void_p(accum_ptr), ctypes.c_void_p(stream or 0))
    return h


def hit_rays(scene, rays, ctx=None):
    """rt_hit_rays: rays = (n, 7) float64 (origin, direction, time); returns
    (t, material id) arrays, material -1 for a miss."""
    h = upload(scene, ctx)
    r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 7)
    n = r.shape[0]
    t = np.zeros(n)
    m = np.zeros(n, dtype=np.int32)
    call("rt_hit_rays", h, n, r.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
         t.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), m.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return t, m


def resolve_u8(accum, nx, ny, sample_count):
    """rt_resolve_u8 (main.scm:481-491) on the host."""
    a = np.ascontiguousarray(accum, dtype=np.float64).ravel()
    out = np.zeros(nx * ny * 3, dtype=np.uint8)
    call("rt_resolve_u8", a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), nx, ny, int(sample_count),
         out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return out


def resolve_u8_device(accum_ptr, nx, ny, sample_count, out_ptr, stream=None, ctx=None):
    """rt_resolve_u8_device (main.scm:481-491) on device buffers: nx*ny*3 doubles -> bytes."""
    ctx = ctx or default_context()
    call("rt_resolve_u8_device", ctx.handle, ctypes.c_void_p(accum_ptr), nx, ny, int(sample_count),
         ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream or 0))


def curve_depth_probe(cps, eps8, ctx=None):
    """rt_curve_depth_probe: the curve kernels' depth estimate (bez_maxd) for ray-space control points
    cps (n, 12) and 8 eps (n,); returns int32 depths."""
    ctx = ctx or default_context()
    c = np.ascontiguousarray(cps, dtype=np.float64).reshape(-1, 12)
    e = np.ascontiguousarray(eps8, dtype=np.float64).ravel()
    if e.size != c.shape[0]:
        raise ValueError("one eps8 per curve")
    out = np.zeros(c.shape[0], dtype=np.int32)
    call("rt_curve_depth_probe", ctx.handle, c.shape[0], c.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
         e.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def comm_unique_id():
    """rt_comm_unique_id: a new communicator id (RT_COMM_ID_BYTES bytes), made by rank 0."""
    buf = (ctypes.c_uint8 * _lib.RT_COMM_ID_BYTES)()
    call("rt_comm_unique_id", buf)
    return bytes(buf)


class Comm:
    """rt_comm_create / rt_gather_shards / rt_comm_destroy: the frame-end gather of a multi-GPU frame
    (one process per GPU) over RCCL, behind the C ABI."""

    def __init__(self, unique_id, rank, world, ctx=None):
        if len(unique_id) != _lib.RT_COMM_ID_BYTES:
            raise ValueError("a communicator id has %d bytes" % _lib.RT_COMM_ID_BYTES)
        self.ctx = ctx or default_context()
        self.rank, self.world = rank, world
        buf = (ctypes.c_uint8 * _lib.RT_COMM_ID_BYTES).from_buffer_copy(bytes(unique_id))
        h = ctypes.c_int(0)
        call("rt_comm_create", self.ctx.handle, buf, rank, world, ctypes.byref(h))
        self.handle = h.value

    def gather_shards(self, nx, ny, accum_compact_ptr, frame_ptr, stream=None):
        """rt_gather_shards (collective): every rank's compact accumulator into rank 0's frame."""
        call("rt_gather_shards", self.handle, nx, ny, ctypes.c_void_p(accum_compact_ptr),
             ctypes.c_void_p(frame_ptr or 0), ctypes.c_void_p(stream or 0))

    def close(self):
        if getattr(self, "handle", None):
            call("rt_comm_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_pixels(nx, ny, shard, nshard):
    """rt_shard_pixels: the image pixels (j = y*nx + x) shard `shard` renders."""
    n = ctypes.c_int64(0)
    call("rt_shard_pixels", nx, ny, shard, nshard, None, ctypes.byref(n))
    out = np.zeros(n.value, dtype=np.uint32)
    call("rt_shard_pixels", nx, ny, shard, nshard, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
         ctypes.byref(n))
    return out


def gather_layout(nx, ny, world):
    """rt_gather_layout (host only): per rank its shard's pixel count and the offset of its pixels in the
    ranks' concatenated pixel lists; rank 0 receives rank r's compact accumulator at doubles
    3 * (offset[r] - count[0]) of its receive buffer."""
    cnt = np.zeros(world, dtype=np.int64)
    off = np.zeros(world, dtype=np.int64)
    call("rt_gather_layout", nx, ny, world, cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
         off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    return cnt, off


def gather_shards_local(nx, ny, shard_ptrs, frame_ptr, ctx=None, stream=None):
    """rt_gather_shards_local: every shard's compact accumulator (device pointers, shard r in entry r) on
    this context's device into the frame — rt_gather_shards' receive layout and placement without RCCL."""
    ctx = ctx or default_context()
    arr = (ctypes.c_void_p * len(shard_ptrs))(*[ctypes.c_void_p(p) for p in shard_ptrs])
    call("rt_gather_shards_local", ctx.handle, nx, ny, len(shard_ptrs), arr, ctypes.c_void_p(frame_ptr),
         ctypes.c_void_p(stream or 0))
