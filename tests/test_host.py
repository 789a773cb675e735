"""Host-side logic that needs no GPU: the C ABI exports, scene construction
(the reference's scene definitions), descriptor emission, the tile partition
used for multi-GPU sharding, resolve / PPM output."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from rtamd import _lib, scenes
from rtamd import scene as g
from rtamd.rng import HostStream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "rt.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    decl = _header_functions()
    assert len(decl) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [d for d in decl if d not in exported]
    assert not missing, missing
    assert sorted(_lib.EXPORTED) == decl            # the ctypes binding covers the whole ABI


def test_library_loads_and_reports_errors_without_gpu():
    L = _lib.lib()
    assert L.rt_abi_version() == 7
    h = ctypes.c_int(0)
    assert L.rt_scene_begin(424242, ctypes.byref(h)) != 0
    assert b"invalid context" in L.rt_last_error()
    # render-schedule options are per context: an unknown handle is refused before any device call
    assert L.rt_context_set_option(424242, 1, 2) != 0
    assert b"invalid context" in L.rt_last_error()
    v = ctypes.c_int64(7)
    assert L.rt_context_get_option(424242, 1, ctypes.byref(v)) != 0 and v.value == 7
    with pytest.raises(_lib.RtError):
        _lib.call("rt_shard_pixels", 4, 4, 5, 2, None, ctypes.byref(ctypes.c_int64()))


def test_new_abi_entry_points_refuse_bad_handles_without_gpu():
    """ABI 6 / 7 entry points check their handles and arguments before any device or RCCL call."""
    L = _lib.lib()
    h = ctypes.c_int(0)
    uid = (ctypes.c_uint8 * _lib.RT_COMM_ID_BYTES)()
    assert L.rt_comm_create(424242, uid, 0, 1, ctypes.byref(h)) != 0
    assert b"invalid context" in L.rt_last_error()
    assert L.rt_comm_create(424242, uid, 2, 2, ctypes.byref(h)) != 0
    assert b"rank" in L.rt_last_error()
    assert L.rt_gather_shards(424242, 4, 4, None, None, None) != 0
    assert b"invalid communicator" in L.rt_last_error()
    assert L.rt_comm_destroy(424242) != 0
    assert L.rt_curve_depth_probe(424242, 1, None, None, None) != 0
    assert b"invalid context" in L.rt_last_error()
    assert L.rt_context_set_option(424242, _lib.RT_OPTIONS["exact_libm"], 1) != 0
    # ABI 7 (round 6): the host-only layout and the one-device gather
    cnt = (ctypes.c_int64 * 4)()
    off = (ctypes.c_int64 * 4)()
    assert L.rt_gather_layout(0, 4, 2, cnt, off) != 0
    assert b"positive" in L.rt_last_error()
    assert L.rt_gather_layout(4, 4, 0, cnt, off) != 0
    assert b"world" in L.rt_last_error()
    assert L.rt_gather_layout(4, 4, 2, None, off) != 0
    assert L.rt_gather_layout(1 << 16, 1 << 16, 2, cnt, off) != 0
    assert b"too large" in L.rt_last_error()
    bufs = (ctypes.c_void_p * 2)()
    assert L.rt_gather_shards_local(424242, 4, 4, 2, ctypes.cast(bufs, ctypes.c_void_p), ctypes.c_void_p(16), None) != 0
    assert b"invalid context" in L.rt_last_error()
    assert L.rt_gather_shards_local(424242, 4, 4, 2, None, ctypes.c_void_p(16), None) != 0
    assert b"null" in L.rt_last_error()


def test_random_scene_structure():
    sc = scenes.random_scene(200, 100)
    objs = sc.obj_list
    # push! order reversed (main.scm:36-88): metal (4,1,0) first, ground last
    assert objs[0].kind == "sphere" and objs[0].args[0] == (4.0, 1.0, 0.0) and objs[0].args[2].kind == "metal"
    assert objs[1].args[0] == (-4.0, 1.0, 0.0) and objs[2].args[2].kind == "dielectric"
    assert objs[-1].args[0] == (0.0, -1000.0, 0.0) and objs[-1].args[1] == 1000.0
    small = objs[3:-1]
    assert 150 <= len(small) <= 225
    for o in small:
        c = o.args[0]
        assert c[1] == 0.2
        assert ((c[0] - 4) ** 2 + (c[2]) ** 2) ** 0.5 > 0.9     # skip test main.scm:49
        if o.kind == "moving_sphere":
            assert o.args[2] == 0.0 and o.args[3] == 1.0 and o.args[4] == 0.2
            assert 0.0 <= o.args[1][1] - 0.2 <= 0.5
            assert o.args[5].kind == "lambertian"
        else:
            assert o.args[1] == 0.2 and o.args[2].kind in ("metal", "dielectric")
    # deterministic in the host seed, different for another
    again = scenes.random_scene(200, 100).obj_list
    assert [o.args[0] for o in again] == [o.args[0] for o in objs]
    other = scenes.random_scene(200, 100, seed=1).obj_list
    assert [o.args[0] for o in other] != [o.args[0] for o in objs]


def test_random_scene_draw_order():
    """First grid cell: choose-mat, then centre x, then centre z (main.scm:45-48)."""
    rr = HostStream(scenes.SCENE_SEED)
    choose, cx, cz = rr(), rr(), rr()
    center = (-5 + 0.9 * cx, 0.2, -5 + 0.9 * cz)
    small_last = scenes.random_scene(10, 10).obj_list[-2]      # first pushed small sphere
    assert small_last.args[0] == center
    assert small_last.kind == ("moving_sphere" if choose < 0.8 else "sphere")


class Recorder:
    """A builder that records the descriptor stream (scene.emit)."""

    def __init__(self):
        self.calls = []

    def __getattr__(self, name):
        def f(*a):
            self.calls.append((name, a))
            return len(self.calls) - 1
        return f


def test_emit_shares_objects_and_orders_children_first():
    sc = scenes.cornell_box(64, 64)
    r = Recorder()
    g.emit(sc, r)
    names = [c[0] for c in r.calls]
    assert names.count("material_lambertian") == 3 and names.count("material_diffuse_light") == 1
    assert names.count("box") == 2 and names.count("rotate_y") == 2 and names.count("translate") == 2
    assert names[-4:] == ["list", "set_camera", "set_sky", "commit"]
    # every referenced id was produced earlier
    for i, (name, args) in enumerate(r.calls):
        for a in args:
            if isinstance(a, int) and name not in ("rect", "set_sky"):
                assert a < i


def test_emit_requires_perlin_tables():
    sc = scenes.test_scene2(8, 8)
    sc.perlin = None
    with pytest.raises(ValueError):
        g.emit(sc, Recorder())


def test_constructor_type_checks():
    with pytest.raises(TypeError):
        g.make_sphere((0, 0, 0), 1, "not a material")
    with pytest.raises(TypeError):
        g.make_scene([], None, lambda r: None)


def _tile_stride(n):
    return next(k for k in (3, 5, 7, 11, 13) if n % k)


@pytest.mark.parametrize("nx,ny,n", [(1920, 1080, 8), (33, 17, 3), (16, 16, 2), (5, 3, 4), (1024, 1024, 6),
                                     (1920, 1080, 3), (400, 300, 15)])
def test_shard_partition_is_exact(nx, ny, n):
    from rtamd import gpu
    parts = [gpu.shard_pixels(nx, ny, r, n) for r in range(n)]
    allpix = np.concatenate(parts)
    assert allpix.size == nx * ny
    assert np.array_equal(np.sort(allpix), np.arange(nx * ny, dtype=np.uint32))
    # tile (tx, ty) -> shard (tx + k ty) % n, k the smallest odd prime not dividing n (16x16 tiles, row-major)
    k = _tile_stride(n)
    for r, p in enumerate(parts):
        x, y = p % nx, p // nx
        assert np.all((k * (y // 16) + x // 16) % n == r)
    # round-6 advice: with a stride coprime to n every shard gets tiles of every column residue (the stride 3
    # at n = 3 gave shard r the columns tx = r mod 3 only, whole-column stripes again)
    tx, ty = (nx + 15) // 16, (ny + 15) // 16
    if ty >= n and tx >= n:
        for r, p in enumerate(parts):
            cols = np.unique((p % nx) // 16)
            assert cols.size == tx, (r, cols.size, tx)


@pytest.mark.parametrize("nx,ny", [(1920, 1080), (1024, 1024), (200, 120), (33, 17)])
def test_gather_layout_counts_and_offsets(nx, ny):
    """rt_gather_layout — the receive layout rt_gather_shards (RCCL) and rt_gather_shards_local share — for
    N = 2..8 at the C2 / C5 (1920x1080) and C4 (1024x1024) frame sizes: per rank the shard's pixel count
    (= rt_shard_pixels'), offsets the prefix sums, rank 0's receive buffer holding ranks 1..N-1 back to back
    at 3 (off[r] - count[0]) doubles, and the concatenated lists a permutation of the frame's pixels."""
    from rtamd import gpu
    for n in range(1, 9):
        cnt, off = gpu.gather_layout(nx, ny, n)
        want = np.array([gpu.shard_pixels(nx, ny, r, n).size for r in range(n)])
        assert np.array_equal(cnt, want), (n, cnt, want)
        assert off[0] == 0 and np.array_equal(off[1:], np.cumsum(cnt)[:-1])
        assert cnt.sum() == nx * ny
        recv = 3 * (off - cnt[0])                       # doubles, where rank r's shard lands on rank 0
        assert recv[1] == 0 if n > 1 else True
        for r in range(1, n - 1):
            assert recv[r] + 3 * cnt[r] == recv[r + 1]
        cat = np.concatenate([gpu.shard_pixels(nx, ny, r, n) for r in range(n)])
        assert np.array_equal(np.sort(cat), np.arange(nx * ny, dtype=np.uint32))
        if n > 1 and nx * ny > 16 * 16 * n:
            assert cnt.max() - cnt.min() <= 2 * 16 * 16 * max(1, (nx + 15) // 16 // n + 1)


def test_env_hooks_are_documented():
    """The library reads only the test / fault hooks INTEGRATION.md lists (round 6 pruned the losing split
    curve extend's switches and RTAMD_FUSE_BATCH; RTAMD_DEBUG_DEPTH only in the RT_STATS build)."""
    csrc = os.path.join(ROOT, "scheme-raytrace_amd", "csrc")
    names = set()
    for f in ("rt_api.cpp", "rt_kernels.hip"):
        names |= set(re.findall(r'getenv\("(RTAMD_[A-Z0-9_]+)"\)', open(os.path.join(csrc, f)).read()))
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("Test hooks that remain environment variables"):doc.index("Errors: every entry point")]
    listed = set(re.findall(r"`(RTAMD_[A-Z0-9_]+)`", sec.split("Round 6")[0]))
    assert names - {"RTAMD_DEBUG_DEPTH"} == listed, (sorted(names), sorted(listed))
    for gone in ("RTAMD_CURVE_SPLIT", "RTAMD_CURVE_K", "RTAMD_FUSE_BATCH", "RTAMD_CURVE_DEBUG"):
        assert gone not in names


def test_resolve_matches_reference_formula(oracle_mod):
    from rtamd import gpu
    rs = np.random.RandomState(3)
    acc = rs.uniform(0, 5, size=7 * 5 * 3)
    acc[:5] = [0.0, 4.0, 4.0000001, 1e-9, 100.0]
    want = np.array([int(np.floor(255.99 * min(1.0, np.sqrt(a / 4)))) for a in acc], dtype=np.uint8)
    assert np.array_equal(gpu.resolve_u8(acc, 7, 5, 4), want)
    assert np.array_equal(oracle_mod.resolve_u8(acc, 4), want)


def test_ppm_writer_flips_rows(tmp_path):
    from rtamd.render import write_ppm
    img = np.arange(2 * 3 * 3, dtype=np.uint8)        # nx=2, ny=3, y-up rows
    p = tmp_path / "t.ppm"
    write_ppm(str(p), img, 2, 3)
    lines = p.read_text().splitlines()
    assert lines[0] == "P3" and lines[1] == " 2 3" and lines[2] == "255"   # main.scm:442
    assert lines[3] == "12 13 14"                     # top row first = y = ny-1 (main.scm:445)
    assert lines[-1] == "3 4 5"


def test_medium_order_segments():
    """Media split the object list: a constant medium listed before other
    objects is committed without error and keeps its list position (the
    GPU-side order is checked against the oracle in test_gpu_parity)."""
    from rtamd import scene as g
    from rtamd.camera import make_camera
    white = g.make_lambertian(g.constant_texture((0.73, 0.73, 0.73)))
    box = g.make_box((0, 0, 0), (1, 1, 1), white)
    sc = g.make_scene([g.make_constant_medium(box, 0.5, g.constant_texture((1, 1, 1))),
                       g.make_sphere((0, 0, -3), 1, white)],
                      make_camera((0, 0, 3), (0, 0, 0), (0, 1, 0), 40, 1, 0, 1, 0, 1), g.sky_color)
    assert [o.kind for o in sc.obj_list] == ["medium", "sphere"]
    with pytest.raises(ValueError):
        g.make_constant_medium(box, 0.0, g.constant_texture((1, 1, 1)))


def test_curve_width_must_be_positive():
    """make-bezier accepts any width in the reference, but for width <= 0 its depth estimate is the log of
    a number <= 0 (bezier.scm:179-192): Gauche's log gives a complex number (or -inf) and ceiling->exact
    raises on the first ray that tests the curve.  The host API and the C ABI refuse such widths up front."""
    from rtamd import gpu  # noqa: F401
    red = g.make_lambertian(g.constant_texture((0.65, 0.05, 0.05)))
    for w in (0.0, -0.5, float("inf"), float("nan")):
        with pytest.raises(ValueError):
            g.make_bezier((0, 0, 0), (1, 0, 0), (2, 0, 0), (3, 0, 0), w, red)
        with pytest.raises(ValueError):
            g.bezier_array(np.zeros((2, 12)), w, red)


def _build_c_example(tmp_path):
    import subprocess
    exe = tmp_path / "cornell"
    rtamd_dir = os.path.join(ROOT, "scheme-raytrace_amd", "rtamd")
    subprocess.run(["gcc", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "examples", "cornell.c"), "-L", rtamd_dir,
                    "-l:librtamd.so", "-L", "/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath," + rtamd_dir, "-o", str(exe)],
                   check=True)
    return exe


def test_c_example_builds_against_the_abi(tmp_path):
    """examples/cornell.c uses only include/rt.h and links librtamd.so."""
    import subprocess
    exe = _build_c_example(tmp_path)
    out = subprocess.run([str(exe), "--abi"], check=True, capture_output=True, text=True).stdout
    assert out.strip() == "rt_abi_version 7"


def test_load_points_and_points_to_bezier(tmp_path):
    """load-points (points.scm:10-19): one "x,y,z" per line scaled by
    magnitude, integers and decimals; points->bezier (points.scm:28-43): one
    segment per interior pair, control points (p1, p1 + (p2-p0)/6, p2 -
    (p3-p1)/6, p2)."""
    from rtamd import points, vec as v
    f = tmp_path / "pts.csv"
    f.write_text("0,0,0\n1,2,3\n2.5,-1,0.5\n4,0,-2\n5,1,1\n")
    pts = points.load_points(str(f), 10)
    assert len(pts) == 5
    assert tuple(pts[1]) == (10, 20, 30) and tuple(pts[2]) == (25.0, -10, 5.0)
    bz = points.points_to_bezier(pts)
    assert len(bz) == len(pts) - 3
    p0, p1, p2, p3 = pts[0], pts[1], pts[2], pts[3]
    want = [p1, v.sum(p1, v.scale(v.diff(p2, p0), 1 / 6)), v.diff(p2, v.scale(v.diff(p3, p1), 1 / 6)), p2]
    for a, b in zip(bz[0], want):
        assert tuple(a) == tuple(b)
    assert tuple(bz[-1][0]) == tuple(pts[2]) and tuple(bz[-1][3]) == tuple(pts[3])
