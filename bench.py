#!/usr/bin/env python3
"""Benchmark: Mrays/s on the RTIOW cover scene at 1920x1080x1024spp (config C2).

A "step" = one full frame: every pixel of the 1920x1080 frame gets `--spp`
camera samples (1024 by default) traced through the wavefront
(raygen -> [extend -> shade/compact]* -> accumulate), i.e. the whole C2
workload.  A ray = one ray segment (one closest-hit query issued by the
integrator).  `value` = total segments / wall time over
the timed steps (max over ranks), inputs resident in HBM.

Multi-GPU (torch.distributed.run, one process per GPU): the frame is split
into interleaved 16x16 tiles (tile (tx, ty) -> rank (tx + k ty) % N, k = 3, or 5 when 3 | N); each rank renders its
tiles into a compact accumulator of its own pixels (rt_render_shard_device)
and rank 0 gathers the shards over RCCL / xGMI at frame end and scatters them
into the frame (rtamd.dist.gather_frame; the pixels are disjoint, so the
frame is bit-identical to one GPU's).  Total work per step is fixed:
"scaling": "strong".

Each step also resolves the frame to bytes on the device (rt_resolve_u8_device,
main.scm:481-491), after the gather when N > 1.

Parity (the metric's "per-pixel RMS vs ref"), at every N, after the timed
steps on rank 0: (1) `parity`: the oracle renders a 64-row band at the top
sample indices (at N=1 this is also the timed cpu_baseline) and the GPU renders
the same band and passes with the production schedule; (2) `parity_frame`:
rows of the last timed frame itself (gathered from every rank when N > 1)
against the oracle's render of those rows with every pass.

Roofline: `roofline` is the closest-hit kernels' own HBM fraction (one render
lane, HIP events on the lane's stream; with two lanes in the timed region it
comes from one extra untimed single-lane frame, and the overlapped figure is
`roofline_two_lane`); `roofline_frame` is the whole path's algorithmic bytes
per frame over ms_per_step.  PMC-derived `traffic` / `valu` / `valu_issue`
come from profiles/pmc/<scene>_*.json only when those carry this rt_kernels.hip's hash.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "scheme-raytrace_amd"))

METRIC = "Mrays/sec at 1920x1080x1024spp RTIOW cover scene; per-pixel RMS vs ref"   # BASELINE.json (C2)
SCENE_NAME = {"cover": "RTIOW cover scene", "cover_marble": "Perlin-textured + moving spheres cover scene",
              "cornell": "Cornell box scene", "cornell_mixture": "Cornell box scene with pdf.scm mixture sampling",
              "curves": "2^20 Bezier curves scene"}


def metric_for(scene, nx, ny, spp):
    """The metric string for this run's configuration (BASELINE.json's for C2)."""
    return "Mrays/sec at %dx%dx%dspp %s; per-pixel RMS vs ref" % (nx, ny, spp, SCENE_NAME.get(scene, scene + " scene"))
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
F64_VALU_PEAK_TFLOPS = 78.6    # MI355X FP64 vector spec (FMA = 2 flops)
# Algorithmic HBM bytes of the extend kernels: every segment
# reads its ray record o, d (6 x f64 = 48 B; k_camera writes it instead); a
# hit writes its queue record t (8) + leaf id (4) + slot (4) = 16 B; a miss
# instead reads throughput + work id (28 B) and writes the sample colour
# (24 B) = 52 B, i.e. 36 B more.  Per path add the camera ray's time and draw
# counter (12 B, depth-0 state) and one miss (each path ends in the sky except
# the few absorbed / depth-capped ones: an upper bound within ~1%).
EXTEND_BYTES_PER_SEGMENT = 48 + 16
EXTEND_BYTES_PER_PATH = 12 + (52 - 16)


def extend_kernels(scene, info):
    """The kernels whose launches the extend events bracket (roofline*.kernel)."""
    if scene == "curves":
        return "k_extend_curves (persistent, every depth)"
    if info.get("camera_lds_bytes"):
        return "k_camera (depth 0) + k_extend_lds"
    return "k_extend_lds" if info.get("extend_lds_bytes") else "k_extend"


def extend_bytes(segments, paths):
    return EXTEND_BYTES_PER_SEGMENT * segments + EXTEND_BYTES_PER_PATH * paths


# Algorithmic HBM bytes of the wavefront shade phase (the per-material k_shade
# launches of an iteration): a shaded hit reads its queue record (16: t, leaf,
# slot) and ray record (48), plus the camera ray's time and draw counter (12)
# at depth 0 or the path record (32) deeper; a survivor writes ray + path
# records (80), a path that ends at the hit writes its sample colour (24).
def shade_bytes(hits_d0, hits, survivors):
    return (76 * hits_d0 + 96 * hits + 80 * survivors + 24 * (hits_d0 + hits - survivors))


def shade_roofline(ms_shade, launches, hits_d0, hits, survivors, note, scene, frame=None):
    """The shade phase (one iteration's per-material k_shade launches, HIP
    events around them) against the HBM roofline."""
    if not launches or ms_shade <= 0 or not (hits_d0 + hits):
        return None
    b = shade_bytes(hits_d0, hits, survivors)
    ach = b / (ms_shade * 1e-3) / 1e9
    hpl = (hits_d0 + hits) / launches
    pm, _ = load_pmc("shade", scene, frame)     # PMC HBM bytes per hit (tools/profile_round.sh) x hits per launch
    traffic = round(pm["bytes_per_hit"] * hpl) if pm and pm.get("bytes_per_hit") else None
    return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": traffic,
            "kernel": "k_shade<material> (one iteration's launches)",
            "bytes_per_launch": round(b / launches), "hits_per_launch": round(hpl),
            "avg_launch_ms": round(ms_shade / launches, 4), "note": note}


def scene_device(info):
    """rt_get_scene_info plus the LDS kernels' occupancy: resident blocks of
    512 threads per CU -> waves per SIMD (4 SIMDs per CU)."""
    out = dict(info)
    cus = max(1, info["cus"])
    for k in ("extend", "camera"):
        blocks = info["%s_lds_blocks" % k]
        out["%s_waves_per_simd" % k] = round(blocks / cus * 512 / 64 / 4, 2) if blocks else None
    return out


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--spp", type=int, default=1024)
    p.add_argument("--nx", type=int, default=1920)
    p.add_argument("--ny", type=int, default=1080)
    p.add_argument("--scene", default="cover")
    p.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0002)
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true",
                   help="skip the CPU baseline and with it the band parity check (both need the oracle)")
    p.add_argument("--no-profile-events", action="store_true")
    p.add_argument("--no-isolated", action="store_true", help="skip the single-lane profiling frame")
    p.add_argument("--lanes", type=int, default=0, help="render lanes (RT_OPT_LANES); 0 = the library's choice")
    p.add_argument("--exact-libm", default="auto", choices=["auto", "exact", "device"],
                   help="RT_OPT_EXACT_LIBM for the timed frames (bounce directions' sin / cos)")
    p.add_argument("--shard-balance", default="",
                   help="comma-separated shard counts (e.g. 2,4,8): render each tile shard of the frame alone on "
                        "this GPU, print its time and segments (max / mean) and exit; no timed bench line")
    return p.parse_args()


def host_cpu():
    """The GPU box's host CPU as this process sees it: model, nproc, the
    affinity set, the cgroup CPU quota and OMP_NUM_THREADS (the box gives a
    one-GPU job a 16-CPU share of a much larger machine)."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = os.cpu_count()
    try:
        with open("/proc/cpuinfo") as f:
            info["model"] = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "unknown")
    except OSError:
        info["model"] = "unknown"
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["cgroup_cpus"] = quota
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    share = info["affinity"] or 1
    if quota:
        share = min(share, max(1, int(quota)))
    if info["omp_num_threads"] and info["omp_num_threads"].isdigit():
        share = min(share, int(info["omp_num_threads"]))
    info["threads_used"] = max(1, share)
    return info


def band_rows(ny):
    rows = min(64, ny)
    return max(0, ny // 3 - rows // 2), rows


def oracle_band(o, scene, nx, ny, spp, seed, budget_s, T):
    """The oracle on rows y0..y0+63 at the top sample indices (passes spp-P ..
    spp-1, P sized to ~budget_s on T threads).  Returns (ref, segments,
    seconds, per-row-pass seconds)."""
    import numpy as np
    y0, rows = band_rows(ny)
    lo, hi = y0 * nx, (y0 + rows) * nx
    # calibrate: one pass over 8 rows (after a zero-pixel call that builds the oracle's trees)
    cal = np.zeros(nx * ny * 3)
    o.render(nx, ny, spp - 1, 1, seed, cal, lo, lo, T)
    t = time.perf_counter()
    o.render(nx, ny, spp - 1, 1, seed, cal, lo, min(hi, lo + 8 * nx), T)
    per_row_pass = (time.perf_counter() - t) / min(8, rows)
    P = int(max(1, min(spp, budget_s / max(1e-9, per_row_pass * rows))))
    acc = np.zeros(nx * ny * 3)
    t = time.perf_counter()
    _, segs = o.render(nx, ny, spp - P, P, seed, acc, lo, hi, T)
    t_all = time.perf_counter() - t
    return {"acc": acc, "y0": y0, "rows": rows, "spp_begin": spp - P, "passes": P}, segs, t_all, per_row_pass


def cpu_baseline(o, scene, nx, ny, spp, seed, budget_s, host):
    """The oracle (C f64 restatement, OpenMP over pixels) timed on the host:
    (1) on the process's whole CPU share, on a 64-row band of the frame at the
        top sample indices (oracle_band); its accumulator is also the parity
        reference for the GPU's band;
    (2) on one thread, rows of the same band at pass spp-1 (~budget_s/3);
    (3) config C1 (cover scene 200x100x8 spp) in full, all threads and one.
    Returns (cpu_baseline dict, band reference, per-row-pass seconds)."""
    import numpy as np
    from rtamd import scenes
    T = host["threads_used"]
    ref, segs, t_all, per_row_pass = oracle_band(o, scene, nx, ny, spp, seed, budget_s, T)
    y0, rows, P = ref["y0"], ref["rows"], ref["passes"]
    lo = y0 * nx
    # one thread: the band row by row, pass spp-1 then spp-2 ..., until ~budget/3
    one = np.zeros(nx * ny * 3)
    t1, segs1, done = 0.0, 0, 0
    while t1 < budget_s / 3 and done < rows * spp:
        r, k = done % rows, done // rows
        t = time.perf_counter()
        _, sg = o.render(nx, ny, spp - 1 - k, 1, seed, one, lo + r * nx, lo + (r + 1) * nx, 1)
        t1 += time.perf_counter() - t
        segs1 += sg
        done += 1
    # C1 in full (200x100, 8 passes, seed 0x5EED0001)
    import oracle  # cpu_baseline leg only
    c1 = oracle.build_scene(scenes.random_scene(200, 100))
    c1_rates = {}
    for th in (T, 1):
        a = np.zeros(200 * 100 * 3)
        t = time.perf_counter()
        _, sg = c1.render(200, 100, 0, 8, 0x5EED0001, a, 0, -1, th)
        c1_rates[th] = (sg / (time.perf_counter() - t) / 1e6, sg)
    out = {"value": round(segs / t_all / 1e6, 3), "unit": "Mrays/s", "cores": T, "kind": "port",
           "sample": "oracle/rt_oracle.c (C f64 restatement of the Scheme hot path, OpenMP, %d threads) on rows "
                     "%d..%d of the %dx%d frame, passes %d..%d (%d segments, %.1f s); Gauche, the reference's "
                     "runtime, is not installed on the box" % (T, y0, y0 + rows - 1, nx, ny, spp - P, spp - 1, segs,
                                                                 t_all),
           "single_thread": {"value": round(segs1 / t1 / 1e6, 4), "unit": "Mrays/s", "cores": 1,
                             "sample": "%d row-passes of the band (rows %d..%d, passes from %d down; %d segments, "
                                       "%.1f s)" % (done, y0, y0 + rows - 1, spp - 1, segs1, t1)},
           "c1_full": {"config": "C1: cover scene 200x100x8 spp, seed 0x5EED0001, whole frame",
                       "threads": {str(T): round(c1_rates[T][0], 3), "1": round(c1_rates[1][0], 4)},
                       "unit": "Mrays/s", "segments": c1_rates[1][1]},
           "host": host}
    return out, ref, per_row_pass


def frame_rows_parity(o, frame_np, nx, ny, spp, seed, per_row_pass, budget_s, T):
    """Rows of the benchmarked frame itself (rank 0's, after the gather when
    N > 1: every rank's tiles cross a row) against the oracle's render of the
    same rows with every pass 0..spp-1.  Rows: as many as ~budget_s of oracle
    time allows (1..8), centred in the frame."""
    import numpy as np
    rows = int(max(1, min(8, budget_s / max(1e-9, per_row_pass * spp))))
    y0 = max(0, ny // 2 - rows // 2)
    lo, hi = y0 * nx, (y0 + rows) * nx
    ref = np.zeros(nx * ny * 3)
    t = time.perf_counter()
    o.render(nx, ny, 0, spp, seed, ref, lo, hi, T)
    dt = time.perf_counter() - t
    got = frame_np[3 * lo:3 * hi] / spp
    exp = ref[3 * lo:3 * hi] / spp
    d = np.abs(got - exp)
    rms = float(np.sqrt(np.mean(d ** 2)))
    return {"rms_vs_oracle": rms, "max_abs": float(d.max()),
            "pixels_gt_1e-9": int((d.reshape(-1, 3).max(axis=1) > 1e-9).sum()), "pixels": int(d.size // 3),
            "tolerance_rms": 1e-4, "pass": bool(rms <= 1e-4), "rows": "%d..%d" % (y0, y0 + rows - 1),
            "passes": "0..%d" % (spp - 1), "oracle_s": round(dt, 1),
            "note": "rows of the last timed frame (the gathered frame on rank 0) vs the oracle, all passes",
            "_ref": ref[3 * lo:3 * hi]}


def frame_rows_parity_mode(pf, scene, nx, ny, spp, seed, h, ctx, mode):
    """parity_frame's rows again with RT_OPT_EXACT_LIBM = mode (rt_render_rows_device, every pass, the
    production schedule), against the same oracle render (pf["_ref"])."""
    import numpy as np
    import torch
    from rtamd import gpu
    y0, y1 = (int(x) for x in pf["rows"].split(".."))
    ref = pf.pop("_ref")
    acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    with ctx.options(exact_libm=gpu._lib.RT_LIBM[mode]):
        gpu.render_rows_device(scene, nx, ny, y0, y1 - y0 + 1, 0, spp, seed, acc.data_ptr(), ctx=ctx)
    torch.cuda.synchronize()
    lo, hi = 3 * y0 * nx, 3 * (y1 + 1) * nx
    d = np.abs(acc.cpu().numpy()[lo:hi] / spp - ref / spp)
    rms = float(np.sqrt(np.mean(d ** 2)))
    return {"exact_libm": mode, "rms_vs_oracle": rms, "max_abs": float(d.max()),
            "pixels_gt_1e-9": int((d.reshape(-1, 3).max(axis=1) > 1e-9).sum()), "pixels": int(d.size // 3),
            "tolerance_rms": 1e-4, "pass": bool(rms <= 1e-4), "rows": pf["rows"], "passes": pf["passes"],
            "note": "parity_frame's rows rendered again (rt_render_rows_device, production schedule) with "
                    "RT_OPT_EXACT_LIBM = %s, against the same oracle render" % mode}


def gpu_band_parity(scene, nx, ny, seed, ref, h, ctx):
    """Render the cpu_baseline band (same rows, same top-of-frame passes) on
    the GPU with the production schedule — rt_render_rows_device, the default
    chunk policy (>= 4 chunks) and two render lanes, so k_camera, k_extend_lds
    and the k_shade kernels do the work — and compare with the oracle's
    accumulator.  Parity metric: per-pixel linear-RGB RMS of sum/passes."""
    import numpy as np
    import torch
    from rtamd import gpu
    acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    gpu.render_rows_device(scene, nx, ny, ref["y0"], ref["rows"], ref["spp_begin"], ref["passes"], seed,
                           acc.data_ptr(), ctx=ctx)
    st = gpu.stats(h)
    torch.cuda.synchronize()
    lo, hi = 3 * ref["y0"] * nx, 3 * (ref["y0"] + ref["rows"]) * nx
    P = ref["passes"]
    got = acc.cpu().numpy()[lo:hi] / P
    exp = ref["acc"][lo:hi] / P
    d = np.abs(got - exp)
    rms = float(np.sqrt(np.mean(d ** 2)))
    return {"rms_vs_oracle": rms, "max_abs": float(d.max()),
            "pixels_gt_1e-9": int((d.reshape(-1, 3).max(axis=1) > 1e-9).sum()),
            "pixels": int(d.size // 3), "tolerance_rms": 1e-4, "pass": bool(rms <= 1e-4),
            "rows": "%d..%d" % (ref["y0"], ref["y0"] + ref["rows"] - 1),
            "passes": "%d..%d" % (ref["spp_begin"], ref["spp_begin"] + P - 1),
            "gpu_schedule": {"chunks": int(st.chunks), "lanes": int(st.lanes), "paths": int(st.paths),
                             "wavefront_segments": int(st.extend_rays), "tail_paths": int(st.finish_paths)},
            "note": "oracle = oracle/rt_oracle.c on the host, GPU = rt_render_rows_device (production schedule)"}


def shard_balance(a, scene, h, ctx, nx, ny, spp, counts):
    """--shard-balance: the multi-GPU frame's tile shards (rt_render_shard_device, tile (tx, ty) -> shard (tx + k ty) % N)
    rendered one at a time on this GPU, each timed alone, against the whole frame rendered the same way.
    max / mean of the shard times bounds N-GPU strong-scaling efficiency (the frame waits for its slowest
    rank); T_frame / max(T_shard) is the speedup the partition allows before the gather."""
    import torch
    from rtamd import dist as rdist
    from rtamd import gpu
    stream = torch.cuda.current_stream().cuda_stream

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t, gpu.stats(h)

    frame = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    for _ in range(max(1, a.warmup)):
        timed(lambda: gpu.render_device(scene, nx, ny, 0, spp, a.seed, frame.data_ptr(), stream=stream, ctx=ctx))
    t_frame, st = timed(lambda: gpu.render_device(scene, nx, ny, 0, spp, a.seed, frame.data_ptr(), stream=stream,
                                                  ctx=ctx))
    out = {"mode": "shard_balance", "config": "%s: %s %dx%dx%dspp" % (SCENE_CONFIG.get(a.scene, "extra"), a.scene, nx,
                                                                      ny, spp),
           "frame_ms": round(t_frame * 1e3, 2), "frame_segments": int(st.segments), "partitions": {}}
    for n in counts:
        rows = []
        for r in range(n):
            shard = torch.zeros(rdist.local_size(nx, ny, r, n), dtype=torch.float64, device="cuda")
            t, st = timed(lambda: gpu.render_shard_device(scene, nx, ny, 0, spp, a.seed, r, n, shard.data_ptr(),
                                                          stream=stream, ctx=ctx))
            rows.append({"shard": r, "pixels": shard.numel() // 3, "ms": round(t * 1e3, 2),
                         "segments": int(st.segments)})
            print("bench: shard-balance N=%d shard %d: %.1f ms" % (n, r, t * 1e3), file=sys.stderr, flush=True)
        ms = [x["ms"] for x in rows]
        sg = [x["segments"] for x in rows]
        mean_ms, mean_sg = sum(ms) / n, sum(sg) / n
        out["partitions"][str(n)] = {
            "shards": rows, "ms_max_over_mean": round(max(ms) / mean_ms, 4),
            "segments_max_over_mean": round(max(sg) / mean_sg, 4),
            "predicted_speedup": round(t_frame * 1e3 / max(ms), 3),
            "predicted_efficiency": round(t_frame * 1e3 / max(ms) / n, 4),
            "note": "one GPU renders each shard alone: efficiency = T_frame / (N max T_shard), before the gather"}
    print(json.dumps(out), flush=True)


SCENE_CONFIG = {"cover": "C2", "cover_marble": "C3", "cornell": "C4", "cornell_mixture": "C4-mixture", "curves": "C5"}
SCENE_DATA = {
    "cover": "RTIOW cover scene (random-scene, main.scm:31-89 + repairs R1/R3) generated from host seed 0x5EED0001",
    "cover_marble": "cover scene with a marble ground (C3), host seed 0x5EED0001, Perlin seed 0x5EED0003",
    "cornell": "cornell-box (main.scm:330-351)",
    "cornell_mixture": "cornell-box with pdf.scm light/cosine mixture sampling toward the ceiling light (extension f2)",
    "curves": "2^20 curves from seeded random polylines via points->bezier (numpy seed 0x5EED0005) in a BVH "
              "inside the cornell-bezier frame (main.scm:353-373)",
}


def kernel_sha16():
    """Hash of the kernel source the PMC summaries under profiles/ must carry
    (tools/pmc_report.py stamps them) for bench.py to use their counters."""
    import hashlib
    with open(os.path.join(ROOT, "scheme-raytrace_amd", "csrc", "rt_kernels.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def pmc_path(kind, scene):
    """Where tools/pmc_report.py files a scene's PMC summary (kind: extend / shade)."""
    return os.path.join(ROOT, "profiles", "pmc", "%s_%s.json" % (scene, kind))


def load_pmc(kind, scene, frame=None):
    """The scene's PMC summary (profiles/pmc/<scene>_<kind>.json) if it was measured on this scene with
    these kernels and (round 6) at this frame size and sample count (`frame` = "NXxNYxSPPspp": the schedule —
    chunks, per-depth or fused curve launches — follows them), else None.  Returns (summary, path)."""
    path = pmc_path(kind, scene)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        pm = json.load(f)
    if pm.get("scene") != scene or pm.get("kernel_sha16") != kernel_sha16():
        return None, None
    if frame is not None and (" %s," % frame) not in str(pm.get("config", "")):
        return None, None
    return pm, os.path.relpath(path, ROOT)


def extend_roofline(segs, tail_segs, paths, launches, ms_ext, pm, kernels, note):
    """The closest-hit kernels' HBM roofline: algorithmic bytes per launch over
    the average launch duration (HIP events on the lane's stream)."""
    if not launches or ms_ext <= 0:
        return None
    wf_segs = segs - tail_segs
    rays_per_launch = wf_segs / launches
    avg_ms = ms_ext / launches
    bytes_per_launch = extend_bytes(wf_segs, paths) / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": round(pm["bytes_per_segment"] * rays_per_launch) if pm else None,
            "kernel": kernels, "bytes_per_launch": round(bytes_per_launch),
            "rays_per_launch": round(rays_per_launch), "avg_launch_ms": round(avg_ms, 4), "launches": launches,
            "note": note}


# Algorithmic HBM bytes of the rest of the frame (roofline_frame): a tail
# path (k_finish) reads its ray + path records once (80 B) and writes its
# sample (24 B); the accumulate reads every sample (24 B) and reads + writes
# each pixel's running sum once per chunk (48 B); the resolve reads the sum
# (24 B) and writes the bytes (3 B) per pixel.
TAIL_BYTES_PER_PATH = 80 + 24


def frame_bytes(segs, tail_segs, paths, sh_d0, sh, sh_surv, finish_paths, npix, chunks):
    return {"extend": extend_bytes(segs - tail_segs, paths), "shade": shade_bytes(sh_d0, sh, sh_surv),
            "tail": TAIL_BYTES_PER_PATH * finish_paths, "accumulate": 24 * paths + 48 * npix * chunks,
            "resolve": 27 * npix}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist

    from rtamd import dist as rdist
    from rtamd import gpu, scenes
    from rtamd._lib import call

    # RCCL ("nccl") over xGMI, one GPU per rank.  RTAMD_DIST_BACKEND=gloo rehearses the
    # multi-process flow on fewer GPUs than ranks (ranks share devices, the gather goes
    # through host memory); it is never the measured configuration.
    backend = os.environ.get("RTAMD_DIST_BACKEND", "nccl")
    device = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    torch.cuda.set_device(device)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    nx, ny, spp = a.nx, a.ny, a.spp
    t_scene = time.perf_counter()
    scene = scenes.SCENES[a.scene](nx, ny)          # the host's scene constructors (the Scheme side's work)
    t_scene = time.perf_counter() - t_scene
    ctx = gpu.default_context(device)
    if a.lanes:
        ctx.set_option("lanes", a.lanes)
    ctx.set_option("exact_libm", a.exact_libm)
    t_commit = time.perf_counter()
    h = gpu.upload(scene, ctx)                      # one-time scene commit (not in the timed steps; reported)
    t_commit = time.perf_counter() - t_commit
    info0 = gpu.scene_info(h)
    scene_commit = {
        "scene_build_ms": round(t_scene * 1e3, 1),
        "commit_total_ms": round(t_commit * 1e3, 1),
        "constructors_ms": round(t_commit * 1e3 - info0["commit_ms"], 1),
        "commit_build_ms": round(info0["commit_ms"] - info0["commit_upload_ms"], 1),
        "commit_upload_ms": round(info0["commit_upload_ms"], 1),
        "commit_sah_ms": round(info0["commit_sah_ms"], 1), "commit_threads": int(info0["commit_threads"]),
        "note": "one-time per scene, outside the timed steps (SURVEY §8(d) d1): scene_build = the host's scene "
                "constructors (rtamd.scenes, e.g. points->bezier for C5); constructors = their rt_add_* calls "
                "through the C ABI; commit_build = rt_scene_commit's flattening and BVH builds (SAH sweep, "
                "BVH4 collapse); commit_upload = its device allocations and copies"}
    call("rt_set_profiling", h, 0 if a.no_profile_events else 1)
    if a.shard_balance:
        shard_balance(a, scene, h, ctx, nx, ny, spp, [int(x) for x in a.shard_balance.split(",") if x])
        return
    # world == 1: the frame accumulator; world > 1: this rank's compact shard (its tiles only), gathered
    # onto rank 0 over RCCL at frame end (rtamd.dist.gather_frame).  Rank 0 resolves the frame to bytes
    # (main.scm:481-491) inside the step.
    frame = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda") if world == 1 or rank == 0 else None
    shard = torch.zeros(rdist.local_size(nx, ny, rank, world), dtype=torch.float64, device="cuda") \
        if world > 1 else None
    image = torch.zeros(nx * ny * 3, dtype=torch.uint8, device="cuda") if frame is not None else None

    def step():
        t0 = time.perf_counter()
        stream = torch.cuda.current_stream().cuda_stream
        if world == 1:
            frame.zero_()
            gpu.render_device(scene, nx, ny, 0, spp, a.seed, frame.data_ptr(), stream=stream, ctx=ctx)
        else:
            shard.zero_()
            gpu.render_shard_device(scene, nx, ny, 0, spp, a.seed, rank, world, shard.data_ptr(), stream=stream,
                                    ctx=ctx)
        t1 = time.perf_counter()                    # the render call returns with its streams drained
        if world > 1:
            rdist.gather_frame(shard, nx, ny, rank, world, out=frame)
        if frame is not None:
            gpu.resolve_u8_device(frame.data_ptr(), nx, ny, spp, image.data_ptr(), stream=stream, ctx=ctx)
        torch.cuda.synchronize()
        return gpu.stats(h), t1 - t0, time.perf_counter() - t1

    def progress(msg):                 # a line per frame: long configurations (C5) take a minute per frame
        if rank == 0:
            print("bench: %s (%.1f s)" % (msg, time.perf_counter() - t_start), file=sys.stderr, flush=True)

    t_start = time.perf_counter()
    for w in range(a.warmup):
        step()
        progress("warmup frame %d/%d" % (w + 1, a.warmup))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    segs = paths = 0
    ms_ext = ms_shade = ms_fin = 0.0
    launches = 0
    tail_segs = finish_paths = chunks = 0
    sh_d0 = sh = sh_surv = 0
    t_render = t_gather = 0.0
    lanes = 0
    for k in range(a.steps):
        s, tr, tg = step()
        progress("timed frame %d/%d" % (k + 1, a.steps))
        t_render += tr
        t_gather += tg
        segs += s.segments
        paths += s.paths
        ms_ext += s.ms_extend
        ms_shade += s.ms_shade
        launches += s.extend_launches
        ms_fin += s.ms_finish
        tail_segs += s.segments - s.extend_rays
        finish_paths += s.finish_paths
        chunks += s.chunks
        lanes = s.lanes
        sh_d0 += s.shade_hits_d0
        sh += s.shade_hits
        sh_surv += s.shade_survivors
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    last_frame = frame.cpu().numpy() if frame is not None else None
    # The timed frames keep two render lanes in flight (one for curve scenes): a kernel's
    # event-bracketed duration there includes the other lane's concurrent kernels.  One more
    # (untimed) frame with a single lane gives each kernel its own duration; with one lane
    # already, the timed region's events are the kernels' own.
    iso = None
    if not a.no_profile_events and not a.no_isolated and lanes > 1:
        with ctx.options(lanes=1):
            iso = step()[0]
        progress("single-lane profiling frame")
    red_dev = "cpu" if backend == "gloo" else "cuda"
    tot = torch.tensor([segs, paths], dtype=torch.float64, device=red_dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    per_rank = torch.tensor([t_render, t_gather], dtype=torch.float64, device=red_dev)
    ranks = [per_rank.clone() for _ in range(world)]
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_gather(ranks, per_rank)
    segs_all, paths_all = float(tot[0]), float(tot[1])
    elapsed = float(tmax[0])
    if rank == 0:
        value = segs_all / elapsed / 1e6
        ext_kernels = extend_kernels(a.scene, gpu.scene_info(h))
        frame = "%dx%dx%dspp" % (nx, ny, spp)
        pm, pm_src = load_pmc("extend", a.scene, frame)    # PMC counters of these kernels (tools/profile_round.sh)
        two_lane = None
        if iso is not None:
            roof = extend_roofline(iso.segments, iso.segments - iso.extend_rays, iso.paths,
                                   iso.extend_launches, iso.ms_extend, pm, ext_kernels,
                                   "single render lane: one extra untimed frame right after the timed ones "
                                   "(HIP events on the lane's stream, nothing concurrent)")
            two_lane = extend_roofline(segs, tail_segs, paths, launches, ms_ext, pm, ext_kernels,
                                       "timed region, %d render lanes overlapped: launch durations include the "
                                       "other lane's kernels" % lanes)
        else:
            roof = extend_roofline(segs, tail_segs, paths, launches, ms_ext, pm, ext_kernels,
                                   "timed region, one render lane (HIP events on the lane's stream)")
        valu = valu_issue = None
        if pm and roof and pm.get("valu_busy") is not None:
            # share of SIMD cycles issuing VALU over the extend kernels (rocprofv3 VALUBusy, one bench frame):
            # the issue-side roofline of these VALU / latency-bound kernels
            valu_issue = {"bound": "valu_issue", "achieved": round(pm["valu_busy"] / 100.0, 4), "peak": 1.0,
                          "unit": "fraction of SIMD cycles issuing VALU",
                          "frac": round(pm["valu_busy"] / 100.0, 4),
                          "lane_utilization": round(pm["valu_lane_utilization"] / 100.0, 4),
                          "lds_busy": round(pm["lds_busy"] / 100.0, 4),
                          "lds_bank_conflict_ratio": round(pm["lds_bank_conflict_ratio"], 4),
                          "wait_share": round(pm["wait_share"], 4),
                          "valu_instr_per_segment": round(pm["valu_instr_per_segment"], 2),
                          "source": "%s (%s, kernels %s)" % (pm_src, pm.get("config", ""), pm["kernel_sha16"])}
        if pm and roof and pm.get("f64_flops_per_segment"):
            tf = pm["f64_flops_per_segment"] * roof["rays_per_launch"] / (roof["avg_launch_ms"] * 1e-3) / 1e12
            valu = {"bound": "valu_f64", "achieved": round(tf, 3), "peak": F64_VALU_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(tf / F64_VALU_PEAK_TFLOPS, 4),
                    "f64_flops_per_segment": round(pm["f64_flops_per_segment"], 1),
                    "note": "issued f64 lane-ops from SQ_INSTS_VALU_{ADD,MUL,FMA(x2),TRANS}_F64 x 64"}
        # the whole path's algorithmic bytes per frame over the frame time: north_star's path-level figure
        fb = frame_bytes(segs, tail_segs, paths, sh_d0, sh, sh_surv, finish_paths, nx * ny, chunks)
        fb_step = {k: v / a.steps for k, v in fb.items()}
        frame_ach = sum(fb.values()) / elapsed / 1e9 if world == 1 else None
        roof_frame = None
        if frame_ach is not None:
            roof_frame = {"bound": "hbm", "achieved": round(frame_ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(frame_ach / HBM_PEAK_GBS, 5),
                          "bytes_per_step": {k: round(v) for k, v in fb_step.items()},
                          "note": "algorithmic bytes of every kernel of the frame (extend + shade + tail + "
                                  "accumulate + resolve) / ms_per_step"}
        render_s = [float(r[0]) / a.steps for r in ranks]
        gather_s = [float(r[1]) / a.steps for r in ranks]
        out = {
            "metric": metric_for(a.scene, nx, ny, spp), "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: %s; path RNG seed %#x" % (SCENE_DATA.get(a.scene, a.scene + " scene"), a.seed),
            "config": {"workload": "%s: %s scene %dx%dx%dspp, one full frame per step (render + %sresolve)"
                                   % (SCENE_CONFIG.get(a.scene, "extra"), a.scene, nx, ny, spp,
                                      "gather + " if world > 1 else ""),
                       "scene": a.scene, "nx": nx, "ny": ny, "spp": spp,
                       "parallelism": ("tile-shard%d" % world if world > 1 else "single") +
                                      ("" if world == 1 or backend == "nccl" else " (%s rehearsal)" % backend)},
            "roofline": roof, "roofline_two_lane": two_lane, "roofline_frame": roof_frame,
            "valu": valu, "valu_issue": valu_issue,
            "roofline_shade": (shade_roofline(iso.ms_shade, iso.extend_launches, iso.shade_hits_d0, iso.shade_hits,
                                              iso.shade_survivors, "single render lane frame, as roofline", a.scene,
                                              frame)
                               if iso is not None else
                               shade_roofline(ms_shade, launches, sh_d0, sh, sh_surv, "timed region, one render lane",
                                              a.scene, frame)),
            "pmc_source": ("%s (kernels %s)" % (pm_src, pm["kernel_sha16"])) if pm else
                          "none: no PMC summary for these kernels (traffic / valu / valu_issue need "
                          "tools/profile_round.sh on this kernel source at this frame)",
            "scene_device": scene_device(gpu.scene_info(h)),
            "scene_commit": scene_commit,
            "exact_libm": a.exact_libm,
            "render_lanes": lanes,
            "per_rank_ms_per_step": {"render_min": round(min(render_s) * 1e3, 3),
                                     "render_max": round(max(render_s) * 1e3, 3),
                                     "gather_and_resolve_max": round(max(gather_s) * 1e3, 3),
                                     "note": "render = the rank's render call (its streams drained); then the "
                                             "gather to rank 0 (N > 1) and rank 0's resolve_u8"},
            "samples_per_s": round(paths_all / elapsed, 1),
            "segments_per_path": round(segs_all / max(1.0, paths_all), 4),
            "ms_extend_per_step": round(ms_ext / a.steps, 3), "ms_shade_per_step": round(ms_shade / a.steps, 3),
            "ms_finish_per_step": round(ms_fin / a.steps, 3),
            "extend_rays_per_step": round((segs - tail_segs) / a.steps), "paths_per_step": round(paths / a.steps),
            "tail_segments_per_step": round(tail_segs / a.steps),
            "shade_hits_d0_per_step": round(sh_d0 / a.steps), "shade_hits_per_step": round(sh / a.steps),
            "shade_survivors_per_step": round(sh_surv / a.steps),
        }
        out["cpu_baseline"] = None
        out["parity"] = None
        out["parity_frame"] = None
        if not a.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle  # the checker and the CPU baseline only, after the timed region
            host = host_cpu()
            T = host["threads_used"]
            o = oracle.build_scene(scene)
            if world == 1:
                out["cpu_baseline"], ref, per_row_pass = cpu_baseline(o, scene, nx, ny, spp, a.seed,
                                                                      a.cpu_baseline_seconds, host)
            else:                           # the CPU baseline is an N = 1 figure; the parity legs run at every N
                ref, _, _, per_row_pass = oracle_band(o, scene, nx, ny, spp, a.seed, a.cpu_baseline_seconds, T)
            par = gpu_band_parity(scene, nx, ny, a.seed, ref, h, ctx)
            out["parity"] = par
            for k in ("rms_vs_oracle", "max_abs", "pixels_gt_1e-9"):
                out[k] = par[k]
            out["parity_frame"] = frame_rows_parity(o, last_frame, nx, ny, spp, a.seed, per_row_pass,
                                                    a.cpu_baseline_seconds, T)
            # the same rows with the other libm mode (RT_OPT_EXACT_LIBM): exact = the C library's sin / cos
            other = "device" if a.exact_libm == "exact" or (a.exact_libm == "auto" and a.scene == "curves") \
                else "exact"
            out["parity_frame_" + other] = frame_rows_parity_mode(out["parity_frame"], scene, nx, ny, spp, a.seed,
                                                                  h, ctx, other)
            out["parity_frame"]["exact_libm"] = a.exact_libm
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
