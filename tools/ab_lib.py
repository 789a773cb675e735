#!/usr/bin/env python3
"""A/B timing of two (or more) builds of librtamd.so on one GPU, with an image
checksum per variant (the variants must render the same image bit for bit).

usage: python tools/ab_lib.py --scene curves --spp 4 --rounds 2 base:path/to/librtamd_base.so new:path/to/librtamd.so \
           leaf1:path/to/librtamd.so:RTAMD_BVH_LEAF=1
Each (variant, round) is a separate process (RTAMD_LIB selects the library),
rounds interleaved so box drift hits the variants alike.  Prints a line per
run and a JSON summary (median Mrays/s, per-kernel ms of the last run)."""
import argparse
import hashlib
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, os.path.join(ROOT, "scheme-raytrace_amd"))
    import time
    import torch
    from rtamd import gpu, scenes
    from rtamd._lib import call
    sc = scenes.SCENES[a.scene](a.nx, a.ny)
    h = gpu.upload(sc)
    call("rt_set_profiling", h, 1)
    acc = torch.zeros(a.nx * a.ny * 3, dtype=torch.float64, device="cuda")
    gpu.render_device(sc, a.nx, a.ny, 0, a.spp, a.seed, acc.data_ptr())   # warm-up (sizes the path pools)
    acc.zero_()
    torch.cuda.synchronize()
    t = time.perf_counter()
    gpu.render_device(sc, a.nx, a.ny, 0, a.spp, a.seed, acc.data_ptr())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    st = gpu.stats(h)
    img = acc.cpu().numpy()
    digest = hashlib.sha1(img.tobytes()).hexdigest()[:16]
    if a.out:
        import numpy as np
        np.save(a.out, img)
    print(json.dumps({"mrays": st.segments / dt / 1e6, "ms": dt * 1e3, "segments": st.segments, "sha": digest,
                      "ms_extend": st.ms_extend, "ms_shade": st.ms_shade, "ms_finish": st.ms_finish}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="cover")
    p.add_argument("--nx", type=int, default=1920)
    p.add_argument("--ny", type=int, default=1080)
    p.add_argument("--spp", type=int, default=256)
    p.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0002)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--child", action="store_true")
    p.add_argument("--out", default=None, help="(child) save the accumulator here (.npy)")
    p.add_argument("variants", nargs="*")
    a = p.parse_args()
    if a.child:
        return child(a)
    res = {}
    for r in range(a.rounds):
        for spec in a.variants:
            name, _, rest = spec.partition(":")
            lib, _, envs = rest.partition(":")
            env = dict(os.environ, RTAMD_LIB=os.path.abspath(lib))
            env.update(dict(kv.split("=", 1) for kv in envs.split(",") if kv))
            img_path = "/tmp/ab_lib_%s.npy" % name
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--scene", a.scene, "--nx",
                                  str(a.nx), "--ny", str(a.ny), "--spp", str(a.spp), "--seed", str(a.seed),
                                  "--out", img_path],
                                 env=env, capture_output=True, text=True, timeout=900)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            if out.returncode != 0 or not line:
                print("variant %s failed:\n%s" % (name, out.stderr[-3000:]), flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            res.setdefault(name, []).append(d)
            print("round %d %-10s %9.2f Mrays/s  %9.1f ms  sha %s  extend %.1f shade %.1f finish %.1f"
                  % (r, name, d["mrays"], d["ms"], d["sha"], d["ms_extend"], d["ms_shade"], d["ms_finish"]), flush=True)
    summ = {n: {"median_mrays": statistics.median(x["mrays"] for x in v), "sha": sorted({x["sha"] for x in v})}
            for n, v in res.items()}
    import numpy as np
    names = [spec.partition(":")[0] for spec in a.variants]
    ref = np.load("/tmp/ab_lib_%s.npy" % names[0]) / a.spp
    for n in names[1:]:
        d = np.abs(np.load("/tmp/ab_lib_%s.npy" % n) / a.spp - ref)
        summ[n]["rms_vs_" + names[0]] = float(np.sqrt(np.mean(d ** 2)))
        summ[n]["pixels_gt_1e-9"] = int((d.reshape(-1, 3).max(axis=1) > 1e-9).sum())
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
