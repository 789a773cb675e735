"""GPU tests of the production schedule and the row / shard entry points.

The small parity renders in test_gpu_parity.py fit under the tail threshold
(max(32768, B/256) paths, rt_api.cpp tail_threshold) and so run entirely in
the tail kernel k_finish.  The tests here size the work so the wavefront
kernels the benchmark times — k_camera, k_extend_lds, the per-material
k_shade queues, sharded compaction, several sample chunks on two render
lanes — do it, at high sample indices, and compare with the oracle (the C
f64 restatement of the reference) or bitwise with other schedules.
"""
import os

import numpy as np
import pytest

from conftest import host_threads
from rtamd import gpu, scenes

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4
SEED = 0x5EED0002


def _wavefront_only(ctx):
    ctx.set_option("tail_off", 1)


def _compare(a, b, n):
    d = np.abs(a / n - b / n)
    px = d.reshape(-1, 3).max(axis=1)
    return float(np.sqrt(np.mean(d ** 2))), float(d.max()), int((px > 1e-9).sum()), px.size


@pytest.fixture(scope="module")
def c2_band(gpu_ctx, oracle_mod):
    """Config C2 (cover scene, 1920x1080) rows 528..543, passes 1000..1023,
    through the production schedule: 8 chunks of 3 passes (92 160 paths each,
    above the tail threshold) on 2 lanes.  The rows cross the horizon, where
    grazing bounces off the ground concentrate the device library's sin / cos
    ulps (test_horizon_rows_exact_libm).  Returns the GPU accumulator, the
    oracle's, and the render statistics."""
    import torch
    nx, ny, y0, rows, s0, n = 1920, 1080, 528, 16, 1000, 24
    scene = scenes.random_scene(nx, ny)
    with gpu_ctx.options(max_paths=3 * rows * nx, lanes=2):
        acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
        h = gpu.render_rows_device(scene, nx, ny, y0, rows, s0, n, SEED, acc.data_ptr())
        st = gpu.stats(h)
        got = acc.cpu().numpy()
    ref = np.zeros(nx * ny * 3)
    lo, hi = y0 * nx, (y0 + rows) * nx
    oracle_mod.build_scene(scene).render(nx, ny, s0, n, SEED, ref, lo, hi, nthreads=host_threads())
    return dict(nx=nx, ny=ny, y0=y0, rows=rows, s0=s0, n=n, scene=scene, got=got, ref=ref, stats=st, lo=lo, hi=hi)


def test_production_band_vs_oracle(c2_band):
    b = c2_band
    st = b["stats"]
    assert st.chunks >= 4 and st.lanes == 2, (st.chunks, st.lanes)
    assert st.extend_rays > st.paths          # the wavefront kernels traced camera and scattered rays
    lo, hi = b["lo"], b["hi"]
    rms, dmax, nbad, npx = _compare(b["got"][3 * lo:3 * hi], b["ref"][3 * lo:3 * hi], b["n"])
    print("C2 band rows %d..%d passes %d..%d: rms=%.3e max=%.3e pixels>1e-9: %d/%d chunks=%d lanes=%d"
          % (b["y0"], b["y0"] + b["rows"] - 1, b["s0"], b["s0"] + b["n"] - 1, rms, dmax, nbad, npx, st.chunks,
             st.lanes))
    assert rms <= RMS_TOL
    assert nbad <= max(2, npx // 200)
    # nothing outside the band was touched
    assert not b["got"][:3 * lo].any() and not b["got"][3 * hi:].any()


def test_production_band_wavefront_to_depth_cap_bitwise(c2_band, sched):
    """The same band with the tail kernel off (every depth in the wavefront,
    one lane, other chunking): bit for bit the production result."""
    import torch
    b = c2_band
    _wavefront_only(sched)
    sched.set_option("lanes", 1)
    sched.set_option("max_paths", 5 * b["rows"] * b["nx"])
    acc = torch.zeros(b["nx"] * b["ny"] * 3, dtype=torch.float64, device="cuda")
    h = gpu.render_rows_device(b["scene"], b["nx"], b["ny"], b["y0"], b["rows"], b["s0"], b["n"], SEED,
                               acc.data_ptr())
    assert gpu.stats(h).finish_paths == 0
    assert np.array_equal(acc.cpu().numpy(), b["got"])


# Configs C3 / C4 (and C4 with the f2 mixture) at their stated frame sizes, on
# a band at the top sample indices of their frames, through the production
# schedule: chunks of `chunk` passes (above the tail threshold) on two render
# lanes, so k_camera / k_extend_lds (or k_extend<F>) and the per-material
# k_shade queues do the wide iterations and k_finish only the tail.
#   name: (nx, ny, y0, rows, first pass, passes, passes per chunk)
BANDS = {
    "cover_marble": (1920, 1080, 400, 16, 1000, 24, 3),       # C3: marble ground (Perlin tables in LDS)
    "cornell": (1024, 1024, 480, 64, 4088, 8, 2),             # C4: cornell-box, 4096-spp frame
    "cornell_mixture": (1024, 1024, 480, 64, 4088, 8, 2),     # C4 + f2 light / cosine mixture
}


@pytest.mark.parametrize("name", sorted(BANDS))
def test_config_band_production_vs_oracle(sched, oracle_mod, name):
    import torch
    nx, ny, y0, rows, s0, n, per_chunk = BANDS[name]
    scene = scenes.SCENES[name](nx, ny)
    sched.set_option("max_paths", per_chunk * rows * nx)
    sched.set_option("lanes", 2)
    acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    h = gpu.render_rows_device(scene, nx, ny, y0, rows, s0, n, SEED, acc.data_ptr())
    st = gpu.stats(h)
    got = acc.cpu().numpy()
    ref = np.zeros(nx * ny * 3)
    lo, hi = y0 * nx, (y0 + rows) * nx
    _, segs = oracle_mod.build_scene(scene).render(nx, ny, s0, n, SEED, ref, lo, hi, nthreads=host_threads())
    rms, dmax, nbad, npx = _compare(got[3 * lo:3 * hi], ref[3 * lo:3 * hi], n)
    print("%s band rows %d..%d passes %d..%d: rms=%.3e max=%.3e pixels>1e-9: %d/%d segments gpu %d oracle %d "
          "(wavefront %d, tail paths %d of %d) chunks=%d lanes=%d"
          % (name, y0, y0 + rows - 1, s0, s0 + n - 1, rms, dmax, nbad, npx, st.segments, segs, st.extend_rays,
             st.finish_paths, st.paths, st.chunks, st.lanes))
    assert st.chunks >= 4 and st.lanes == 2, (st.chunks, st.lanes)
    # the wavefront kernels traced every camera ray and the wide scattered iterations; the tail kernel only
    # took each chunk's last few paths
    assert st.extend_rays > st.paths and st.finish_paths < st.paths
    assert rms <= RMS_TOL
    assert nbad <= max(2, npx // 200)
    assert not got[:3 * lo].any() and not got[3 * hi:].any()


@pytest.mark.parametrize("name", ["cover", "cover_marble"])
def test_horizon_rows_exact_libm(sched, oracle_mod, name):
    """C2 / C3 frame rows 536..543 (the horizon band of the 1920x1080 frame, where the bench's parity_frame
    rows sit), passes 0..255, production schedule (8 chunks on 2 lanes).  With RT_OPT_EXACT_LIBM = exact
    the bounce directions' sin / cos are the C library's bit for bit, and the image must equal the oracle's
    to the last bits: 0 pixels off by more than 1e-9.  The default mode (round 6: exact in scenes with
    noise / marble textures, so C3's count is 0; the device library's sin / cos in the cover scene) may
    move at most 0.5 % of the pixels by more than 1e-9."""
    import torch
    nx, ny, y0, rows, n = 1920, 1080, 536, 8, 256
    scene = scenes.SCENES[name](nx, ny)
    lo, hi = y0 * nx, (y0 + rows) * nx
    ref = np.zeros(nx * ny * 3)
    oracle_mod.build_scene(scene).render(nx, ny, 0, n, SEED, ref, lo, hi, nthreads=host_threads())
    sched.set_option("max_paths", 32 * rows * nx)
    sched.set_option("lanes", 2)
    res = {}
    for mode in ("exact", "auto"):
        sched.set_option("exact_libm", mode)
        acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        h = gpu.render_rows_device(scene, nx, ny, y0, rows, 0, n, SEED, acc.data_ptr())
        st = gpu.stats(h)
        assert st.chunks >= 4 and st.lanes == 2 and st.extend_rays > st.paths
        res[mode] = _compare(acc.cpu().numpy()[3 * lo:3 * hi], ref[3 * lo:3 * hi], n)
        print("%s rows %d..%d passes 0..%d, exact_libm=%s: rms=%.3e max=%.3e pixels>1e-9: %d/%d"
              % (name, y0, y0 + rows - 1, n - 1, mode, *res[mode]))
    rms, dmax, nbad, npx = res["exact"]
    assert nbad == 0 and rms <= 1e-12, res["exact"]
    assert res["auto"][0] <= RMS_TOL and res["auto"][2] <= npx // 200, res["auto"]
    if name == "cover_marble":
        assert res["auto"][2] == 0, res["auto"]


def test_exact_libm_option_values(sched):
    """RT_OPT_EXACT_LIBM takes auto / exact / device (0 / 1 / 2) and refuses anything else; the
    schedule options do not touch it."""
    from rtamd._lib import RtError
    assert sched.get_option("exact_libm") == 0
    for mode, v in (("exact", 1), ("device", 2), ("auto", 0)):
        sched.set_option("exact_libm", mode)
        assert sched.get_option("exact_libm") == v
    with pytest.raises(RtError, match="RT_OPT_EXACT_LIBM"):
        sched.set_option("exact_libm", 3)


def test_trace_line_row_by_row_equals_trace_all(gpu_ctx):
    """trace-line (main.scm:452-469) over every row, pass by pass, and the
    animate loop (main.scm:533-544) equal trace-all's passes bit for bit."""
    from rtamd.render import Renderer
    nx, ny = 48, 27
    scene = scenes.random_scene(nx, ny)
    a = Renderer(nx, ny, seed=SEED)
    b = Renderer(nx, ny, seed=SEED)
    c = Renderer(nx, ny, seed=SEED)
    for k in (1, 2, 3):
        img_a = a.trace_all(scene, k)
        for y in range(ny):
            img_b = b.trace_line(scene, y, k)
        assert np.array_equal(a.raw_data, b.raw_data)
        assert np.array_equal(img_a, img_b)
    for _ in range(2 * (ny + 1)):            # two full sweeps of the GLUT loop
        c.animate(scene)
    d = Renderer(nx, ny, seed=SEED)
    d.trace_all(scene, 1)
    d.trace_all(scene, 2)
    assert np.array_equal(c.raw_data, d.raw_data)
    assert c.anim_sample_count == 3 and c.current_y == 0


def test_rows_match_frame_bitwise(sched):
    """Row bands (rt_render_rows) through the wavefront reassemble the
    full-frame render bit for bit."""
    _wavefront_only(sched)
    nx, ny, spp = 64, 36, 4
    scene = scenes.random_scene(nx, ny)
    full = np.zeros(nx * ny * 3)
    gpu.render_host(scene, nx, ny, 0, spp, SEED, full)
    parts = np.zeros(nx * ny * 3)
    for y0, yn in ((0, 7), (7, 20), (27, 9)):
        gpu.render_rows_host(scene, nx, ny, y0, yn, 0, spp, SEED, parts)
    assert np.array_equal(full, parts)


def test_compact_shards_match_frame(sched):
    """rt_render_shard_device (a rank's compact accumulator, as bench.py's
    multi-GPU path uses) scattered by rt_shard_pixels equals the frame."""
    import torch
    from rtamd import dist as rdist
    _wavefront_only(sched)
    nx, ny, spp, world = 70, 45, 3, 3
    scene = scenes.random_scene(nx, ny)
    full = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    gpu.render_device(scene, nx, ny, 0, spp, SEED, full.data_ptr())
    frame = torch.zeros_like(full)
    for r in range(world):
        local = torch.zeros(rdist.local_size(nx, ny, r, world), dtype=torch.float64, device="cuda")
        gpu.render_shard_device(scene, nx, ny, 0, spp, SEED, r, world, local.data_ptr())
        idx = torch.from_numpy(rdist.shard_pixels(nx, ny, world)[r]).cuda()
        frame.view(-1, 3).index_copy_(0, idx, local.view(-1, 3))
    torch.cuda.synchronize()
    assert torch.equal(full, frame)


def test_row_and_shard_errors(gpu_ctx):
    import torch
    from rtamd._lib import RtError
    nx, ny = 16, 8
    scene = scenes.random_scene(nx, ny)
    acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    with pytest.raises(RtError):
        gpu.render_rows_device(scene, nx, ny, 4, 5, 0, 1, SEED, acc.data_ptr())     # rows past the image
    with pytest.raises(RtError):
        gpu.render_rows_device(scene, nx, ny, -1, 2, 0, 1, SEED, acc.data_ptr())
    with pytest.raises(ValueError):
        gpu.trace_line(scene, nx, ny, 0, 1, SEED, np.zeros(nx * ny * 3), np.zeros(3, dtype=np.uint8))
    from rtamd.render import Renderer
    with pytest.raises(ValueError):
        Renderer(nx, ny).trace_line(scene, ny, 1)
    # the failed calls left nothing behind: a good render still works
    gpu.render_rows_device(scene, nx, ny, 0, ny, 0, 1, SEED, acc.data_ptr())
    torch.cuda.synchronize()
    assert torch.isfinite(acc).all() and acc.abs().sum() > 0


def _noise_scene(nx, ny):
    """t:noise-texture (texture.scm:25-28) on the ground and a sphere, a
    marble sphere, a light: no reference scene uses noise-texture, so this
    one exercises its GPU branch against the oracle."""
    from rtamd import scene as g, vec as v
    from rtamd.camera import make_camera
    from rtamd import perlin
    tables = perlin.from_seed(scenes.PERLIN_SEED)
    objs = [g.make_sphere(v.vec3(0, -1000, 0), 1000, g.make_lambertian(g.noise_texture(4))),
            g.make_sphere(v.vec3(0, 2, 0), 2, g.make_lambertian(g.noise_texture(0.7))),
            g.make_sphere(v.vec3(4, 1.2, 1), 1.2, g.make_metal(g.noise_texture(2.5), 0.2)),
            g.make_sphere(v.vec3(-4, 1.2, 0), 1.2, g.make_lambertian(g.marble_texture(1.5))),
            g.make_xy_rect(3, 5, 1, 3, -2, g.make_diffuse_light(g.constant_texture(v.vec3(4, 4, 4))))]
    cam = make_camera((13, 2, 3), (0, 0, 0), (0, 1, 0), 20, nx / ny, 0, 10, 0, 1)
    return g.make_scene(objs, cam, g.sky_color, perlin=tables)


@pytest.mark.parametrize("wavefront", [False, True])
def test_noise_texture_vs_oracle(sched, oracle_mod, wavefront):
    nx, ny, spp = 64, 36, 8
    if wavefront:
        _wavefront_only(sched)
    sc = _noise_scene(nx, ny)
    acc = np.zeros(nx * ny * 3)
    gpu.render_host(sc, nx, ny, 0, spp, SEED, acc)
    ref, _ = oracle_mod.build_scene(sc).render(nx, ny, 0, spp, SEED, nthreads=host_threads())
    rms, dmax, nbad, npx = _compare(acc, ref, spp)
    print("noise texture (wavefront=%s): rms=%.3e max=%.3e pixels>1e-9: %d/%d" % (wavefront, rms, dmax, nbad, npx))
    assert np.isfinite(acc).all() and acc.sum() > 0
    assert rms <= RMS_TOL
    assert nbad <= max(2, npx // 200)


@pytest.mark.parametrize("wavefront", [False, True])
def test_sampler_cap_raises_fault_not_hang(sched, monkeypatch, wavefront):
    """Every device loop that waits on random data has an attempt cap a valid
    stream cannot reach (rt_kernels.hip kRejectCap = 4096, P(reject) <= 0.48).
    RTAMD_REJECT_CAP=0 lowers the cap so the real samplers — random-in-unit-disk
    in the camera (util.scm:17-23, k_camera / k_finish) and random-in-unit-sphere
    in metal scatter (util.scm:9-15, k_shade / k_finish) — hit it on their first
    rejected draw: the render must return with rt_last_error naming the fault,
    not hang, and the next render (default cap) must be clean and unchanged."""
    import torch
    from rtamd._lib import RtError
    nx, ny, spp = 96, 54, 8
    if wavefront:
        _wavefront_only(sched)
    scene = scenes.random_scene(nx, ny)
    good = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    gpu.render_device(scene, nx, ny, 0, spp, SEED, good.data_ptr())
    torch.cuda.synchronize()
    acc = torch.zeros_like(good)
    monkeypatch.setenv("RTAMD_REJECT_CAP", "0")
    with pytest.raises(RtError, match="rejection sampler"):
        gpu.render_device(scene, nx, ny, 0, spp, SEED, acc.data_ptr())
    monkeypatch.delenv("RTAMD_REJECT_CAP")
    acc.zero_()
    gpu.render_device(scene, nx, ny, 0, spp, SEED, acc.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(acc, good)


def test_pools_shared_per_context_and_released(gpu_ctx, monkeypatch):
    """The render lanes' path pools belong to the context: two scenes render
    on one context in turn, rt_context_release_pools frees the pools, and the
    next renders (pools allocated again) are bit for bit the same."""
    import torch
    from rtamd.gpu import Context
    ctx = Context(0)
    try:
        nx, ny, spp = 96, 54, 8
        a, b = scenes.random_scene(nx, ny), scenes.cornell_box(nx, ny)
        outs = []
        for _ in range(2):
            for sc in (a, b):
                acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
                gpu.render_device(sc, nx, ny, 0, spp, SEED, acc.data_ptr(), ctx=ctx)
                torch.cuda.synchronize()
                outs.append(acc.cpu().numpy())
            ctx.release_pools()
        assert np.array_equal(outs[0], outs[2]) and np.array_equal(outs[1], outs[3])
        assert not np.array_equal(outs[0], outs[1])
    finally:
        ctx.close()


def test_raising_lanes_resizes_pools():
    """The path pools are sized at a render so that the lanes together take at most 65 % of the free
    device memory.  Raising RT_OPT_LANES afterwards (2 -> 4) must size them again for four lanes (round-4
    advice: each extra lane used to allocate another pool of the two-lane size, ~110 % of the budget),
    and the image must not change."""
    import torch
    from rtamd.gpu import Context
    ctx = Context(0)
    try:
        nx, ny, spp = 1920, 1080, 600             # > 4 chunks of the largest pools, so four lanes run
        sc = scenes.random_scene(nx, ny)
        out = []
        for lanes in (2, 4):
            ctx.set_option("lanes", lanes)
            acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
            h = gpu.render_device(sc, nx, ny, 0, spp, SEED, acc.data_ptr(), ctx=ctx)
            st = gpu.stats(h)
            torch.cuda.synchronize()
            print("lanes %d: chunks %d, lanes used %d" % (lanes, st.chunks, st.lanes))
            assert st.lanes == lanes
            out.append(acc)
        assert torch.equal(out[0], out[1])
    finally:
        ctx.close()


@pytest.mark.parametrize("switch", ["RTAMD_NO_EXTEND_LDS", "RTAMD_NO_CAMERA_LDS", "RTAMD_FINISH_GENERIC", "RTAMD_NO_SOLO"])
def test_kernel_variants_bitwise(sched, monkeypatch, switch):
    """The cover scene's specialised kernels (k_extend_lds, k_camera, the SOLO
    tail, the SOLO direct-leaf walk) against the general ones (k_extend<F>,
    k_raygen + k_extend, the group-loop tail, leaf records): the same image
    bit for bit."""
    nx, ny, spp = 64, 36, 3
    if switch != "RTAMD_FINISH_GENERIC":
        _wavefront_only(sched)
    a = np.zeros(nx * ny * 3)
    gpu.render_host(scenes.random_scene(nx, ny), nx, ny, 0, spp, SEED, a)
    monkeypatch.setenv(switch, "1")
    b = np.zeros(nx * ny * 3)
    gpu.render_host(scenes.random_scene(nx, ny), nx, ny, 0, spp, SEED, b)
    assert np.isfinite(a).all()
    assert np.array_equal(a, b)
