#!/usr/bin/env python3
"""Benchmark: Mrays/s on the RTIOW cover scene at 1920x1080x1024spp (config C2).

A "step" = one full frame: every pixel of the 1920x1080 frame gets `--spp`
camera samples (1024 by default) traced through the wavefront
(raygen -> [extend -> shade/compact]* -> accumulate), i.e. the whole C2
workload.  A ray = one ray segment (one closest-hit query issued by the
integrator).  `value` = total segments / wall time over
the timed steps (max over ranks), inputs resident in HBM.

Multi-GPU (torch.distributed.run, one process per GPU): the frame is split
into interleaved 16x16 tiles (tile t -> rank t % N, rt_render_device's
shard arguments), each rank renders its tiles into a full-frame f64
accumulator, and the per-rank accumulators are gathered onto rank 0 at frame
end with one RCCL reduce over xGMI (tiles are disjoint, every other pixel is
0.0, so the sum is the exact union).  Total work per step is fixed:
"scaling": "strong".
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "scheme-raytrace_amd"))

METRIC = "Mrays/sec at 1920x1080x1024spp RTIOW cover scene; per-pixel RMS vs ref"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
F64_VALU_PEAK_TFLOPS = 78.6    # MI355X FP64 vector spec (FMA = 2 flops)
# Algorithmic HBM bytes of the extend kernels: every segment
# reads its ray record o, d (6 x f64 = 48 B); a hit writes t (8) + leaf id (4)
# + its queue entry (4) = 16 B; a miss instead reads throughput + work id
# (28 B) and writes the sample colour (24 B) = 52 B, i.e. 36 B more.  Per
# path add the camera ray's time (8 B, depth-0 state) and one miss (each path
# ends in the sky except the few absorbed / depth-capped ones: an upper bound
# within ~1%).
EXTEND_BYTES_PER_SEGMENT = 48 + 16
EXTEND_BYTES_PER_PATH = 8 + (52 - 16)


def extend_bytes(segments, paths):
    return EXTEND_BYTES_PER_SEGMENT * segments + EXTEND_BYTES_PER_PATH * paths


# Algorithmic HBM bytes of the wavefront shade phase (the per-material k_shade
# launches of an iteration): a shaded hit reads its queue entry (4), hit record
# (16) and ray record (48), plus the camera ray's time and draw counter (12)
# at depth 0 or the path record (32) deeper; a survivor writes ray + path
# records (80), a path that ends at the hit writes its sample colour (24).
def shade_bytes(hits_d0, hits, survivors):
    return (80 * hits_d0 + 100 * hits + 80 * survivors + 24 * (hits_d0 + hits - survivors))


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
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-profile-events", action="store_true")
    p.add_argument("--no-isolated", action="store_true", help="skip the single-lane profiling frame")
    return p.parse_args()


def cpu_baseline(scene, nx, ny, seed, budget_s):
    """Time the oracle (C f64 restatement, OpenMP over pixels) on a bounded
    sample of the same workload: a 64-row band of the C2 frame, one spp per
    call, repeated with successive sample indices until ~budget_s of work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle  # cpu_baseline leg only
    threads = max(1, min(16, os.cpu_count() or 1))
    o = oracle.build_scene(scene)
    acc = np.zeros(nx * ny * 3)
    rows = min(64, ny)
    y0 = max(0, ny // 3 - rows // 2)
    lo, hi = y0 * nx, (y0 + rows) * nx
    t_used, segs_total, passes = 0.0, 0, 0
    while t_used < budget_s:
        t = time.perf_counter()
        _, segs = o.render(nx, ny, passes, 1, seed, acc, lo, hi, threads)
        t_used += time.perf_counter() - t
        segs_total += segs
        passes += 1
    rate = segs_total / t_used / 1e6
    return {"value": round(rate, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": "oracle/rt_oracle.c (C f64 restatement of the Scheme hot path, OpenMP, %d threads) on rows "
                      "%d..%d of the %dx%d C2 frame, %d spp (%d segments, %.1f s); Gauche, the reference's "
                      "runtime, is not installed on the box" % (threads, y0, y0 + rows, nx, ny, passes, segs_total,
                                                                 t_used)}


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

    from rtamd import gpu, scenes
    from rtamd._lib import call

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    nx, ny, spp = a.nx, a.ny, a.spp
    scene = scenes.SCENES[a.scene](nx, ny)
    ctx = gpu.default_context(local)
    h = gpu.upload(scene, ctx)                      # one-time scene upload (not timed)
    call("rt_set_profiling", h, 0 if a.no_profile_events else 1)
    accum = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    lib_stream = None                               # librtamd's own stream (events live there)

    def step():
        accum.zero_()
        torch.cuda.synchronize()
        gpu.render_device(scene, nx, ny, 0, spp, a.seed, accum.data_ptr(), shard=rank, nshard=world,
                          stream=lib_stream, ctx=ctx)
        s = gpu.stats(h)
        if world > 1:
            dist.reduce(accum, dst=0, op=dist.ReduceOp.SUM)   # RCCL gather of disjoint tiles
        return s

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    segs = paths = 0
    ms_ext = ms_shade = ms_fin = 0.0
    launches = 0
    tail_segs = 0
    sh_d0 = sh = sh_surv = 0
    for _ in range(a.steps):
        s = step()
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
    tot = torch.tensor([segs, paths], dtype=torch.float64, device="cuda")
    tmax = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    segs_all, paths_all = float(tot[0]), float(tot[1])
    elapsed = float(tmax[0])
    if rank == 0:
        value = segs_all / elapsed / 1e6
        roof = None
        valu = None
        roof_iso = None
        if iso is not None and iso.extend_launches and iso.ms_extend > 0:
            bpl = extend_bytes(iso.extend_rays, iso.paths) / iso.extend_launches
            ams = iso.ms_extend / iso.extend_launches
            ach = bpl / (ams * 1e-3) / 1e9
            roof_iso = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 5), "kernel": "k_extend + k_extend_lds",
                        "bytes_per_launch": round(bpl), "rays_per_launch": round(iso.extend_rays / iso.extend_launches),
                        "avg_launch_ms": round(ams, 4),
                        "note": "one extra untimed frame with a single render lane (no concurrent kernels)"}
        if launches and ms_ext > 0:
            # wavefront extend launches only (the depth tail runs in k_finish)
            wf_segs = segs - tail_segs
            rays_per_launch = wf_segs / launches
            avg_ms = ms_ext / launches
            bytes_per_launch = extend_bytes(wf_segs, paths) / launches
            achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
            traffic = None
            pm = None
            pmc = os.path.join(ROOT, "profiles", "pmc_extend.json")
            if os.path.exists(pmc):
                with open(pmc) as f:
                    pm = json.load(f)
                if pm.get("scene") != a.scene or not pm.get("bytes_per_segment"):
                    pm = None
            if pm:
                traffic = round(pm["bytes_per_segment"] * rays_per_launch)
            roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "kernel": "k_extend + k_extend_lds", "bytes_per_launch": round(bytes_per_launch),
                    "rays_per_launch": round(rays_per_launch), "avg_launch_ms": round(avg_ms, 4),
                    "note": "timed region; render lanes overlap, so launch durations include concurrent kernels"}
            if pm and pm.get("f64_flops_per_segment"):
                tf = pm["f64_flops_per_segment"] * rays_per_launch / (avg_ms * 1e-3) / 1e12
                valu = {"bound": "valu_f64", "achieved": round(tf, 3), "peak": F64_VALU_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(tf / F64_VALU_PEAK_TFLOPS, 4),
                        "f64_flops_per_segment": round(pm["f64_flops_per_segment"], 1),
                        "note": "issued f64 lane-ops from SQ_INSTS_VALU_{ADD,MUL,FMA(x2),TRANS}_F64 x 64"}
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: %s; path RNG seed %#x" % (SCENE_DATA.get(a.scene, a.scene + " scene"), a.seed),
            "config": {"workload": "%s: %s scene %dx%dx%dspp, one full frame per step"
                                   % (SCENE_CONFIG.get(a.scene, "extra"), a.scene, nx, ny, spp),
                       "scene": a.scene, "nx": nx, "ny": ny, "spp": spp,
                       "parallelism": "tile-shard%d" % world if world > 1 else "single"},
            "roofline": roof, "roofline_isolated": roof_iso, "valu": valu,
            "roofline_shade_isolated": shade_roofline(iso, "single render lane frame, as roofline_isolated", a.scene),
            "samples_per_s": round(paths_all / elapsed, 1),
            "segments_per_path": round(segs_all / max(1.0, paths_all), 4),
            "ms_extend_per_step": round(ms_ext / a.steps, 3), "ms_shade_per_step": round(ms_shade / a.steps, 3),
            "ms_finish_per_step": round(ms_fin / a.steps, 3),
            "extend_rays_per_step": round((segs - tail_segs) / a.steps), "paths_per_step": round(paths / a.steps),
            "tail_segments_per_step": round(tail_segs / a.steps),
            "shade_hits_d0_per_step": round(sh_d0 / a.steps), "shade_hits_per_step": round(sh / a.steps),
            "shade_survivors_per_step": round(sh_surv / a.steps),
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, nx, ny, a.seed, a.cpu_baseline_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
