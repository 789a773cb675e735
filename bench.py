#!/usr/bin/env python3
"""Benchmark: Mrays/s on the RTIOW cover scene at 1920x1080x1024spp (config C2).

A "step" = one full frame: every pixel of the 1920x1080 frame gets `--spp`
camera samples (1024 by default) traced through the wavefront
(raygen -> [extend -> shade/compact]* -> accumulate), i.e. the whole C2
workload.  A ray = one ray segment (one closest-hit query issued by the
integrator).  `value` = total segments / wall time over
the timed steps (max over ranks), inputs resident in HBM.

Multi-GPU (torch.distributed.run, one process per GPU): the frame is split
into interleaved 16x16 tiles (tile t -> rank t % N); each rank renders its
tiles into a compact accumulator of its own pixels (rt_render_shard_device)
and rank 0 gathers the shards over RCCL / xGMI at frame end and scatters them
into the frame (rtamd.dist.gather_frame; the pixels are disjoint, so the
frame is bit-identical to one GPU's).  Total work per step is fixed:
"scaling": "strong".

Parity (the metric's "per-pixel RMS vs ref"): after the timed steps rank 0
times the oracle on a 64-row band of the frame at the top sample indices
(cpu_baseline) and renders the same band and passes on the GPU with the
production schedule; rms_vs_oracle / max_abs / pixels_gt_1e-9 compare them.
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


def shade_roofline(st, note, scene):
    if not st or not st.extend_launches or st.ms_shade <= 0 or not (st.shade_hits_d0 + st.shade_hits):
        return None
    b = shade_bytes(st.shade_hits_d0, st.shade_hits, st.shade_survivors)
    ach = b / (st.ms_shade * 1e-3) / 1e9
    hpl = (st.shade_hits_d0 + st.shade_hits) / st.extend_launches
    traffic = None                      # PMC HBM bytes per hit (tools/profile_round.sh) x hits per launch
    pmc = os.path.join(ROOT, "profiles", "pmc_shade.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            pm = json.load(f)
        if pm.get("scene") == scene and pm.get("bytes_per_hit"):
            traffic = round(pm["bytes_per_hit"] * hpl)
    return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": traffic,
            "kernel": "k_shade<material> (one iteration's launches)",
            "bytes_per_launch": round(b / st.extend_launches), "hits_per_launch": round(hpl),
            "avg_launch_ms": round(st.ms_shade / st.extend_launches, 4), "note": note}


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


def cpu_baseline(scene, nx, ny, spp, seed, budget_s):
    """The oracle (C f64 restatement, OpenMP over pixels) timed on the host:
    (1) on the process's whole CPU share, on a 64-row band of the frame at the
        top sample indices (passes spp-P .. spp-1, P sized to ~budget_s); its
        accumulator is also the parity reference for the GPU's band;
    (2) on one thread, rows of the same band at pass spp-1 (~budget_s/3);
    (3) config C1 (cover scene 200x100x8 spp) in full, all threads and one.
    Returns (cpu_baseline dict, band reference)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle  # cpu_baseline leg only
    from rtamd import scenes
    host = host_cpu()
    T = host["threads_used"]
    o = oracle.build_scene(scene)
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
    return out, {"acc": acc, "y0": y0, "rows": rows, "spp_begin": spp - P, "passes": P}


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


SCENE_CONFIG = {"cover": "C2", "cover_marble": "C3", "cornell": "C4", "cornell_mixture": "C4-mixture", "curves": "C5"}
SCENE_DATA = {
    "cover": "RTIOW cover scene (random-scene, main.scm:31-89 + repairs R1/R3) generated from host seed 0x5EED0001",
    "cover_marble": "cover scene with a marble ground (C3), host seed 0x5EED0001, Perlin seed 0x5EED0003",
    "cornell": "cornell-box (main.scm:330-351)",
    "cornell_mixture": "cornell-box with pdf.scm light/cosine mixture sampling toward the ceiling light (extension f2)",
    "curves": "2^20 curves from seeded random polylines via points->bezier (numpy seed 0x5EED0005) in a BVH "
              "inside the cornell-bezier frame (main.scm:353-373)",
}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    nx, ny, spp = a.nx, a.ny, a.spp
    scene = scenes.SCENES[a.scene](nx, ny)
    ctx = gpu.default_context(local)
    h = gpu.upload(scene, ctx)                      # one-time scene upload (not timed)
    call("rt_set_profiling", h, 0 if a.no_profile_events else 1)
    # world == 1: the frame accumulator; world > 1: this rank's compact shard (its tiles only), gathered
    # onto rank 0 over RCCL at frame end (rtamd.dist.gather_frame)
    frame = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda") if world == 1 or rank == 0 else None
    local = torch.zeros(rdist.local_size(nx, ny, rank, world), dtype=torch.float64, device="cuda") \
        if world > 1 else None

    def step():
        (frame if world == 1 else local).zero_()
        rdist.render_frame(scene, nx, ny, 0, spp, a.seed, rank, world, local=local, frame=frame, ctx=ctx)
        return gpu.stats(h)

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
    tail_segs = 0
    sh_d0 = sh = sh_surv = 0
    for k in range(a.steps):
        s = step()
        progress("timed frame %d/%d" % (k + 1, a.steps))
        segs += s.segments
        paths += s.paths
        ms_ext += s.ms_extend
        ms_shade += s.ms_shade
        launches += s.extend_launches
        ms_fin += s.ms_finish
        tail_segs += s.segments - s.extend_rays
        sh_d0 += s.shade_hits_d0
        sh += s.shade_hits
        sh_surv += s.shade_survivors
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # One more (untimed) frame with a single render lane: the overlapped lanes
    # of the timed steps run two chunks' kernels concurrently, so a kernel's
    # event-bracketed duration there includes its neighbour's work.  This
    # frame gives each kernel's duration with the chip to itself.
    iso = None
    if not a.no_profile_events and not a.no_isolated:
        os.environ["RTAMD_LANES"] = "1"
        try:
            iso = step()
        finally:
            del os.environ["RTAMD_LANES"]
        progress("single-lane profiling frame")
    red_dev = "cpu" if backend == "gloo" else "cuda"
    tot = torch.tensor([segs, paths], dtype=torch.float64, device=red_dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    segs_all, paths_all = float(tot[0]), float(tot[1])
    elapsed = float(tmax[0])
    if rank == 0:
        value = segs_all / elapsed / 1e6
        roof = None
        valu = None
        valu_issue = None
        roof_iso = None
        ext_kernels = extend_kernels(a.scene, gpu.scene_info(h))
        pm = None                       # PMC bytes / issue counters of the extend kernels (tools/profile_round.sh)
        pmc = os.path.join(ROOT, "profiles", "pmc_extend.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                pm = json.load(f)
            if pm.get("scene") != a.scene or not pm.get("bytes_per_segment"):
                pm = None
        if iso is not None and iso.extend_launches and iso.ms_extend > 0:
            bpl = extend_bytes(iso.extend_rays, iso.paths) / iso.extend_launches
            ams = iso.ms_extend / iso.extend_launches
            ach = bpl / (ams * 1e-3) / 1e9
            roof_iso = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 5), "kernel": ext_kernels,
                        "bytes_per_launch": round(bpl), "rays_per_launch": round(iso.extend_rays / iso.extend_launches),
                        "avg_launch_ms": round(ams, 4),
                        "traffic": round(pm["bytes_per_segment"] * iso.extend_rays / iso.extend_launches) if pm else None,
                        "note": "one extra untimed frame with a single render lane (no concurrent kernels)"}
        if launches and ms_ext > 0:
            # wavefront extend launches only (the depth tail runs in k_finish)
            wf_segs = segs - tail_segs
            rays_per_launch = wf_segs / launches
            avg_ms = ms_ext / launches
            bytes_per_launch = extend_bytes(wf_segs, paths) / launches
            achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
            traffic = None
            if pm:
                traffic = round(pm["bytes_per_segment"] * rays_per_launch)
            roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "kernel": ext_kernels, "bytes_per_launch": round(bytes_per_launch),
                    "rays_per_launch": round(rays_per_launch), "avg_launch_ms": round(avg_ms, 4),
                    "note": "timed region; render lanes overlap, so launch durations include concurrent kernels"}
            if pm and pm.get("valu_busy") is not None:
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
                              "source": "profiles/pmc_extend.json (%s)" % pm.get("config", "")}
            if pm and pm.get("f64_flops_per_segment"):
                tf = pm["f64_flops_per_segment"] * rays_per_launch / (avg_ms * 1e-3) / 1e12
                valu = {"bound": "valu_f64", "achieved": round(tf, 3), "peak": F64_VALU_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(tf / F64_VALU_PEAK_TFLOPS, 4),
                        "f64_flops_per_segment": round(pm["f64_flops_per_segment"], 1),
                        "note": "issued f64 lane-ops from SQ_INSTS_VALU_{ADD,MUL,FMA(x2),TRANS}_F64 x 64"}
        out = {
            "metric": metric_for(a.scene, nx, ny, spp), "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: %s; path RNG seed %#x" % (SCENE_DATA.get(a.scene, a.scene + " scene"), a.seed),
            "config": {"workload": "%s: %s scene %dx%dx%dspp, one full frame per step"
                                   % (SCENE_CONFIG.get(a.scene, "extra"), a.scene, nx, ny, spp),
                       "scene": a.scene, "nx": nx, "ny": ny, "spp": spp,
                       "parallelism": ("tile-shard%d" % world if world > 1 else "single") +
                                      ("" if world == 1 or backend == "nccl" else " (%s rehearsal)" % backend)},
            "roofline": roof, "roofline_isolated": roof_iso, "valu": valu, "valu_issue": valu_issue,
            "roofline_shade_isolated": shade_roofline(iso, "single render lane frame, as roofline_isolated", a.scene),
            "scene_device": scene_device(gpu.scene_info(h)),
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
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"], ref = cpu_baseline(scene, nx, ny, spp, a.seed, a.cpu_baseline_seconds)
            par = gpu_band_parity(scene, nx, ny, a.seed, ref, h, ctx)
            out["parity"] = par
            for k in ("rms_vs_oracle", "max_abs", "pixels_gt_1e-9"):
                out[k] = par[k]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
