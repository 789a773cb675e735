"""GPU tests of the curve path (bezier.scm:13-223) at configuration C5's scale.

* C5 itself — 2^20 curves in a BVH (geometry.scm:294-371 as test-bezier and
  cornell-bezier use it) at 1920x1080 — on a band of rows through the curve
  cloud, at the top sample indices of the 256-spp frame, on the production
  schedule (several chunks on two render lanes: k_camera / k_extend_curves /
  k_shade for the wide iterations, k_finish for the tail), against the oracle
  (whose OBJ_BVH is a tree with the flat list's semantics,
  tests/test_oracle_bvh.py).
* Flat curves — converge's depth estimate negative, so the root is a leaf
  (bezier.scm:130,189-193) — pooled into the wavefront curve kernel's batched
  subdivision (stage B over >= RT_BEZ_HOLD survivors), counted by
  rt_stats.curve_flat_pooled: the case whose negative leaf level faulted C5 in
  round 2 before the level was clamped at 0.
* A curve needing more subdivision levels than the walk supports fails the
  render with the curve fault (the reference has no depth limit).
"""
import os

import numpy as np
import pytest

from conftest import host_threads
from rtamd import gpu, scenes
from rtamd import scene as g
from rtamd import vec as v
from rtamd._lib import RtError

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4
SEED = 0x5EED0002


def _compare(a, b, n):
    d = np.abs(a / n - b / n)
    px = d.reshape(-1, 3).max(axis=1)
    return float(np.sqrt(np.mean(d ** 2))), float(d.max()), int((px > 1e-9).sum()), px.size


def _opts(ctx, **kv):
    for k, val in kv.items():
        ctx.set_option(k, val)


def test_c5_band_production_vs_oracle(sched, oracle_mod):
    """C5 rows 524..555 (the middle of the frame, through the curve cloud),
    passes 252..255 of the 256-spp frame: 4 chunks of one pass (61 440 paths,
    above the tail threshold) on 2 lanes."""
    import torch
    nx, ny, y0, rows, s0, n = 1920, 1080, 524, 32, 252, 4
    sc = scenes.cornell_curves(nx, ny)
    _opts(sched, max_paths=rows * nx, lanes=2)
    acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    h = gpu.render_rows_device(sc, nx, ny, y0, rows, s0, n, SEED, acc.data_ptr())
    st = gpu.stats(h)
    got = acc.cpu().numpy()
    assert st.chunks >= 4 and st.lanes == 2, (st.chunks, st.lanes)
    # depth 0 in its own launch, then the fused curve extend (every deeper segment in one launch per chunk:
    # no tail kernel) unless RTAMD_CURVE_FUSE=0
    assert st.extend_rays > st.paths
    assert st.curve_pooled_batches > 0
    lo, hi = y0 * nx, (y0 + rows) * nx
    ref = np.zeros(nx * ny * 3)
    o = oracle_mod.build_scene(sc)
    _, segs = o.render(nx, ny, s0, n, SEED, ref, lo, hi, nthreads=host_threads())
    rms, dmax, nbad, npx = _compare(got[3 * lo:3 * hi], ref[3 * lo:3 * hi], n)
    print("C5 band rows %d..%d passes %d..%d: rms=%.3e max=%.3e pixels>1e-9: %d/%d segments gpu %d oracle %d "
          "chunks=%d lanes=%d pooled batches=%d"
          % (y0, y0 + rows - 1, s0, s0 + n - 1, rms, dmax, nbad, npx, st.segments, segs, st.chunks, st.lanes,
             st.curve_pooled_batches))
    assert st.segments == segs                  # every closest-hit query, counted on both sides
    assert rms <= RMS_TOL
    assert nbad <= 2
    assert not got[:3 * lo].any() and not got[3 * hi:].any()


def _flat_curve_scene(nx, ny, m=20000, width=3.0):
    """The Cornell frame with m short curves (extent ~0.5) in front of the
    camera: half straight (l0 is rounding only, converge's depth estimate
    ~ -20), half bent by ~1e-3 (depth -2..-4): every root is a leaf.  With
    200 000 curves of width 6 the ribbons overlap so often that grazing
    bounces decide most paths: until round 4 a 1-ulp difference of the
    device's sin / cos from the C library's (a lambertian bounce direction,
    util.scm:37-44) changed 0.7 % of that scene's pixels; the device now
    computes libm's own bits (rt_libm.h)."""
    rs = np.random.default_rng(0x5EED0105)
    white = g.make_lambertian(g.constant_texture(v.vec3(0.73, 0.73, 0.73)))
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    light = g.make_diffuse_light(g.constant_texture(v.vec3(4, 4, 4)))
    base = rs.uniform(150.0, 400.0, size=(m, 1, 3))
    t = np.linspace(0.0, 0.5, 4).reshape(1, 4, 1) * rs.normal(size=(m, 1, 3))
    bend = 1e-3 * rs.normal(size=(m, 4, 3))
    bend[: m // 2] = 0.0
    objs = [g.flip_normals(g.make_yz_rect(0, 555, 0, 555, 555, white)),
            g.make_yz_rect(0, 555, 0, 555, 0, red),
            g.flip_normals(g.make_xz_rect(213, 343, 227, 332, 554, light)),
            g.make_xz_rect(0, 555, 0, 555, 0, white),
            g.make_bvh_node([g.bezier_array((base + t + bend).reshape(m, 12), width, white)], 0, 0)]
    return g.make_scene(objs, scenes.cornell_camera_for(nx, ny), g.sky_color)


@pytest.mark.parametrize("m,width", [(20000, 3.0), (200000, 6.0)])
def test_flat_curves_in_pooled_batches_vs_oracle(sched, oracle_mod, m, width):
    """Flat curves reach the pooled stage B of k_extend_curves (counted on the
    device), the render raises no fault, and the image matches the oracle:
    at most 2 of 16 384 pixels above 1e-9 (a flipped sample moves its pixel by
    ~1e-2 / spp), in the sparse cloud and in the dense one."""
    nx, ny, spp = 128, 128, 64
    sc = _flat_curve_scene(nx, ny, m, width)
    _opts(sched, tail_off=1, lanes=1)
    acc = np.zeros(nx * ny * 3)
    h = gpu.render_host(sc, nx, ny, 0, spp, SEED, acc)
    st = gpu.stats(h)
    print("flat curves (%d, width %g): pooled batches %d, flat survivors walked in them %d, segments %d"
          % (m, width, st.curve_pooled_batches, st.curve_flat_pooled, st.segments))
    assert st.finish_paths == 0
    assert st.curve_pooled_batches > 0 and st.curve_flat_pooled > 0
    ref, segs = oracle_mod.build_scene(sc).render(nx, ny, 0, spp, SEED, nthreads=host_threads())
    rms, dmax, nbad, npx = _compare(acc, ref, spp)
    print("flat curves (%d, width %g) vs oracle: rms=%.3e max=%.3e pixels>1e-9: %d/%d segments gpu %d oracle %d"
          % (m, width, rms, dmax, nbad, npx, st.segments, segs))
    assert rms <= RMS_TOL
    assert nbad <= 2
    # the same render through the tail kernel's per-lane curve test: bit for bit
    _opts(sched, tail_off=0, tail_paths=100000000)
    b = np.zeros(nx * ny * 3)
    gpu.render_host(sc, nx, ny, 0, spp, SEED, b)
    assert np.array_equal(acc, b)


@pytest.mark.parametrize("wavefront", [False, True])
def test_curve_deeper_than_walk_faults(sched, wavefront):
    """A curve of width 1e-13 spanning ~150 units needs ~27 subdivision levels
    (bezier.scm:180-193); the walk supports 24, so the render fails with the
    curve fault instead of a silently clamped image, and the next render of a
    normal scene is unaffected."""
    if wavefront:
        _opts(sched, tail_off=1)
    nx, ny, spp = 48, 48, 1
    white = g.make_lambertian(g.constant_texture(v.vec3(0.73, 0.73, 0.73)))
    curve = g.make_bezier(v.vec3(200, 200, 250), v.vec3(260, 380, 260), v.vec3(320, 150, 280), v.vec3(370, 330, 300),
                          1e-13, white)
    sc = g.make_scene([g.make_xz_rect(0, 555, 0, 555, 0, white), curve], scenes.cornell_camera_for(nx, ny),
                      g.sky_color)
    acc = np.zeros(nx * ny * 3)
    with pytest.raises(RtError, match="curve walk"):
        gpu.render_host(sc, nx, ny, 0, spp, SEED, acc)
    ok = np.zeros(nx * ny * 3)
    gpu.render_host(scenes.cornell_bezier(nx, ny), nx, ny, 0, spp, SEED, ok)
    assert np.isfinite(ok).all()


def test_duplicate_curves_tie_to_the_later_curve(sched, oracle_mod):
    """Curves duplicated exactly (same control points, other materials) in a
    BVH: every tie in z goes to the later curve of the list, as a flat
    hit-obj-list's scan keeps a curve at z <= t-max (geometry.scm:41-46,
    bezier.scm:164).  This is the project's convention for BVHs, shared by the
    oracle: the reference's own BVH breaks ties by tree shape
    (geometry.scm:252-254, 360-365, a random split axis), and no reference
    output covers exact ties.  rt_hit_rays against the oracle's hit_world,
    material by material; the render against the oracle too."""
    rs = np.random.default_rng(0x5EED0106)
    mats = [g.make_lambertian(g.constant_texture(v.vec3(0.2 + 0.2 * k, 0.5, 0.3))) for k in range(3)]
    cps = rs.uniform(100.0, 450.0, size=(300, 12))
    objs = [g.make_xz_rect(0, 555, 0, 555, 0, mats[0]),
            g.make_bvh_node([g.bezier_array(cps, 8.0, mats[0]), g.bezier_array(cps[::2].copy(), 8.0, mats[1]),
                             g.bezier_array(cps[::3].copy(), 8.0, mats[2])], 0, 0)]
    nx, ny = 48, 48
    sc = g.make_scene(objs, scenes.cornell_camera_for(nx, ny), g.sky_color)
    o = oracle_mod.build_scene(sc)
    cam = np.array(sc.camera.slots())
    n = 4096
    s_, t_ = rs.uniform(0, 1, n), rs.uniform(0, 1, n)
    rays = np.zeros((n, 7))
    rays[:, 0:3] = cam[9:12]
    rays[:, 3:6] = cam[0:3] + s_[:, None] * cam[3:6] + t_[:, None] * cam[6:9] - cam[9:12]
    rays[n // 2:, 3:6] /= np.linalg.norm(rays[n // 2:, 3:6], axis=1)[:, None]   # unit directions too
    t, m = gpu.hit_rays(sc, rays)
    counts = np.zeros(4, dtype=int)
    for k in range(n):
        h = o.hit_world(rays[k, 0:3], rays[k, 3:6], 0.0)
        et, em = (h[0], int(h[7])) if h else (0.0, -1)
        assert (et, em) == (t[k], m[k]), (k, et, em, t[k], m[k])
        counts[em + 1] += 1
    print("duplicate curves: misses / floor-or-first / second / third copies hit:", counts)
    assert counts[2] > 0 and counts[3] > 0        # ties resolved to the later copies
    _opts(sched, tail_off=1)
    acc = np.zeros(nx * ny * 3)
    gpu.render_host(sc, nx, ny, 0, 4, SEED, acc)
    ref, _ = o.render(nx, ny, 0, 4, SEED, nthreads=host_threads())
    rms, dmax, nbad, npx = _compare(acc, ref, 4)
    print("duplicate curves render: rms=%.3e max=%.3e pixels>1e-9: %d/%d" % (rms, dmax, nbad, npx))
    assert rms <= RMS_TOL and nbad <= 2


def test_few_curves_among_spheres_large_launch(sched, oracle_mod, monkeypatch):
    """Two curves in the cover scene's world BVH (random-scene, main.scm:31-88,
    with its spheres), 960x540x16 spp in one chunk: 8.3M paths, thousands
    of rays per wave of the persistent curve kernel.  Candidates are rare, so a
    lane that queued one waits many loop iterations for a batch while the
    other lanes keep claiming rays; the per-ray iteration cap counts only the
    lane's own work, so a valid render raises no fault (round-2 advice: the
    cap once counted the waiting too and scaled with the launch, not the
    scene).  The image equals the per-ray curve kernel's bit for bit, and a
    band of it matches the oracle."""
    from rtamd.rng import HostStream
    nx, ny, spp = 960, 540, 16
    objs = scenes.random_scene_objects(HostStream(scenes.SCENE_SEED))
    gold = g.make_metal(g.constant_texture(v.vec3(0.8, 0.6, 0.2)), 0.05)
    red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
    objs.append(g.make_bezier(v.vec3(-6, 0.3, -2), v.vec3(-2, 2.5, 1), v.vec3(2, -0.5, 2), v.vec3(6, 1.5, -1),
                              0.15, gold))
    objs.append(g.make_bezier(v.vec3(-3, 2.0, 3), v.vec3(0, 0.5, -3), v.vec3(3, 3.0, 1), v.vec3(5, 0.8, 2), 0.1, red))
    sc = g.make_scene(objs, scenes.camera_for(nx, ny), g.sky_color)
    _opts(sched, tail_off=1, lanes=1, max_paths=nx * ny * spp)
    acc = np.zeros(nx * ny * 3)
    h = gpu.render_host(sc, nx, ny, 0, spp, SEED, acc)
    st = gpu.stats(h)
    assert st.chunks == 1 and st.finish_paths == 0, (st.chunks, st.finish_paths)
    monkeypatch.setenv("RTAMD_CURVE_BLOCKS", "0")                  # the per-ray curve kernel
    b = np.zeros(nx * ny * 3)
    gpu.render_host(sc, nx, ny, 0, spp, SEED, b)
    assert np.isfinite(acc).all() and np.array_equal(acc, b), np.abs(acc - b).max()
    y0, rows = 250, 8
    lo, hi = y0 * nx, (y0 + rows) * nx
    ref = np.zeros(nx * ny * 3)
    oracle_mod.build_scene(sc).render(nx, ny, 0, spp, SEED, ref, lo, hi, nthreads=host_threads())
    rms, dmax, nbad, npx = _compare(acc[3 * lo:3 * hi], ref[3 * lo:3 * hi], spp)
    print("few curves among spheres: segments %d, rows %d..%d vs oracle rms=%.3e max=%.3e pixels>1e-9: %d/%d"
          % (st.segments, y0, y0 + rows - 1, rms, dmax, nbad, npx))
    # round 4 let one pixel through at 3e-4: sample 5 of pixel 247288 reflects off the gold curve over and
    # over (|dir| grows each time), and its segment 70 starts 1e9 from the scene, where the f32 slab ends
    # erred past the box margin and the walk culled the curve (tools/dbg/few_curves_probe.py).  The curve
    # scenes' box rays carry per-axis slack for the origin's rounding now (BoxRayW): no pixel may differ.
    assert rms <= RMS_TOL and nbad == 0


def test_curve_walk_stack_overflow_bitwise(sched, monkeypatch):
    """The curve walk pushes up to three children per node; commit_scene bounds
    its stack (rt_scene_info.curve_stack), and entries past the LDS column go
    to the per-lane overflow area in HBM (one region per render lane).  With
    the LDS column cut to one entry (RTAMD_CURVE_LDS_STACK=1) every deeper push
    takes that path, on two render lanes, fused over the depths and one launch
    per depth: the image must not change by a bit."""
    nx, ny, spp = 96, 64, 4
    _opts(sched, tail_off=1, lanes=2, max_paths=nx * ny)
    base = np.zeros(nx * ny * 3)
    h = gpu.render_host(scenes.cornell_curves(nx, ny, n_curves=1 << 14), nx, ny, 0, spp, SEED, base)
    info, st = gpu.scene_info(h), gpu.stats(h)
    assert info["curve_stack"] > 4 and st.lanes == 2 and st.finish_paths == 0
    monkeypatch.setenv("RTAMD_CURVE_LDS_STACK", "1")
    low = np.zeros_like(base)
    gpu.render_host(scenes.cornell_curves(nx, ny, n_curves=1 << 14), nx, ny, 0, spp, SEED, low)
    print("curve walk stack: bound %d, LDS entries 1 vs %d" % (info["curve_stack"], info["tree_depth"]))
    assert np.array_equal(base, low)
    # the same with one curve-kernel launch per depth
    monkeypatch.setenv("RTAMD_CURVE_FUSE", "0")
    other = np.zeros_like(base)
    gpu.render_host(scenes.cornell_curves(nx, ny, n_curves=1 << 14), nx, ny, 0, spp, SEED, other)
    assert np.array_equal(base, other)


def test_curve_ray_cap_faults_without_hang(sched, monkeypatch):
    """k_extend_curves bounds the iterations a lane works on one ray; a lane
    that hits the bound raises the path fault and stays out of the refill, so
    candidates it queued earlier can never be credited to a new ray (round-3
    advice: a refilled lane then waited forever on W.done).  The cap is lowered
    (RTAMD_CURVE_RAY_CAP, a device variable) so rays of a 16K-curve cloud hit
    it mid-walk with candidates queued: the render must fail with the path
    fault within the test's time limit, and the next render must be clean and
    bit-identical to one before."""
    nx, ny, spp = 96, 64, 2
    _opts(sched, tail_off=1, lanes=1)
    sc = scenes.cornell_curves(nx, ny, n_curves=1 << 14)
    good = np.zeros(nx * ny * 3)
    gpu.render_host(sc, nx, ny, 0, spp, SEED, good)
    for cap in (3, 12):
        monkeypatch.setenv("RTAMD_CURVE_RAY_CAP", str(cap))
        acc = np.zeros(nx * ny * 3)
        with pytest.raises(RtError, match="persistent kernel's path or ray"):
            gpu.render_host(sc, nx, ny, 0, spp, SEED, acc)
    monkeypatch.delenv("RTAMD_CURVE_RAY_CAP")
    again = np.zeros(nx * ny * 3)
    gpu.render_host(sc, nx, ny, 0, spp, SEED, again)
    assert np.array_equal(good, again)


def test_curve_hit_appends_spill_between_shards(sched, monkeypatch):
    """k_extend_curves appends a wave's finished rays to one queue shard (blockIdx * 4 + wave) & 7, while
    its waves claim rays dynamically, so a shard's share is not bounded by n / 8 (round-4 advice).  With
    one block (4 waves: shards 0..3 take every hit) and the shard slack cut to 256 entries
    (RTAMD_SHARD_SLACK), each used shard receives ~n/4 > n/8 + 256 hits: the appends must spill into the
    next shards instead of faulting, and the image must equal the default launch's bit for bit."""
    nx, ny, spp = 96, 64, 4
    sc = scenes.cornell_curves(nx, ny, n_curves=1 << 12)
    _opts(sched, tail_off=1, lanes=1, max_paths=nx * ny * spp)
    a = np.zeros(nx * ny * 3)
    gpu.render_host(sc, nx, ny, 0, spp, SEED, a)
    monkeypatch.setenv("RTAMD_SHARD_SLACK", "256")
    monkeypatch.setenv("RTAMD_CURVE_BLOCKS", "1")
    b = np.zeros(nx * ny * 3)
    h = gpu.render_host(sc, nx, ny, 0, spp, SEED, b)
    st = gpu.stats(h)
    print("one curve block, slack 256: paths %d, hits at depth 0 %d" % (st.paths, st.shade_hits_d0))
    assert st.shade_hits_d0 > st.paths // 4 + 8 * 256      # more hits than four unspilled shards could hold
    assert np.isfinite(a).all() and np.array_equal(a, b)
