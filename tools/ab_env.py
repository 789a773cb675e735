#!/usr/bin/env python3
"""A/B timing of librtamd knobs that are read at scene commit or per render
(RTAMD_* environment variables), in one process on one GPU.

usage: python tools/ab_env.py [--scene cover] [--spp 256] [--rounds 3] [--lanes 2] \
           base: "no_solo:RTAMD_NO_SOLO=1" ...
Each variant gets its own freshly committed scene; variants are timed in
interleaved rounds (one full frame each) so box drift hits them alike.
Prints one JSON line per variant: Mrays/s (median), per-kernel ms, scene info.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scheme-raytrace_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="cover")
    p.add_argument("--nx", type=int, default=1920)
    p.add_argument("--ny", type=int, default=1080)
    p.add_argument("--spp", type=int, default=256)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--lanes", default=None, help="render lanes (RT_OPT_LANES) for every variant")
    p.add_argument("variants", nargs="+", help="name:ENV=V,opt.tail_div=256 (name: alone = defaults)")
    a = p.parse_args()
    import torch
    from rtamd import gpu, scenes
    from rtamd._lib import call
    ctx = gpu.default_context(0)
    if a.lanes:
        ctx.set_option("lanes", int(a.lanes))
    vs = []
    for spec in a.variants:
        name, _, envs = spec.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        vs.append((name, env))
    handles, sc_objs = {}, {}
    acc = torch.zeros(a.nx * a.ny * 3, dtype=torch.float64, device="cuda")

    def with_env(env, fn):
        # keys "opt.<name>" are context options (rt_context_set_option), the rest environment variables
        opts = {k[4:]: int(v) for k, v in env.items() if k.startswith("opt.")}
        envs = {k: v for k, v in env.items() if not k.startswith("opt.")}
        old = {k: os.environ.get(k) for k in envs}
        os.environ.update(envs)
        for k, v in opts.items():
            ctx.set_option(k, v)
        try:
            return fn()
        finally:
            for k in opts:
                ctx.set_option(k, 0)
            if a.lanes:
                ctx.set_option("lanes", int(a.lanes))
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    for name, env in vs:
        sc = scenes.SCENES[a.scene](a.nx, a.ny)
        h = with_env(env, lambda: gpu.upload(sc, ctx))
        call("rt_set_profiling", h, 1)
        handles[name], sc_objs[name] = h, sc
        with_env(env, lambda: gpu.render_device(sc, a.nx, a.ny, 0, a.spp, 0x5EED0002, acc.data_ptr(), ctx=ctx))
    res = {name: [] for name, _ in vs}
    for r in range(a.rounds):
        for name, env in vs:
            sc = sc_objs[name]
            acc.zero_()
            torch.cuda.synchronize()
            t = time.perf_counter()
            with_env(env, lambda: gpu.render_device(sc, a.nx, a.ny, 0, a.spp, 0x5EED0002, acc.data_ptr(), ctx=ctx))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            st = gpu.stats(handles[name])
            res[name].append((st.segments / dt / 1e6, dt, st.ms_extend, st.ms_shade, st.ms_finish,
                              st.extend_launches, float(acc.sum())))
        print("round %d done" % r, file=sys.stderr, flush=True)
    for name, env in vs:
        rows = res[name]
        print(json.dumps({
            "variant": name, "env": env, "mrays": round(statistics.median(x[0] for x in rows), 1),
            "all": [round(x[0], 1) for x in rows], "ms_frame": round(statistics.median(x[1] for x in rows) * 1e3, 2),
            "ms_extend": round(statistics.median(x[2] for x in rows), 2),
            "ms_shade": round(statistics.median(x[3] for x in rows), 2),
            "ms_finish": round(statistics.median(x[4] for x in rows), 2),
            "launches": rows[0][5], "checksum": rows[0][6], "info": gpu.scene_info(handles[name])}), flush=True)


if __name__ == "__main__":
    main()
