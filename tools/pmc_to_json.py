#!/usr/bin/env python3
"""Turn rocprofv3 --pmc passes over the extend kernels (k_extend, k_extend_lds)
into profiles/pmc_extend.json: HBM bytes and f64 lane-ops per ray segment.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in
KiB; FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read
(the ray records are read with 16-B loads), so it is doubled; WRITE_SIZE is
taken as is.  The segment count is the extend_rays the profiled bench run
itself reports (its JSON line): k_extend_lds is a persistent kernel, so grid
sizes are not ray counts.

usage: pmc_to_json.py FETCH.csv WRITE.csv BENCH.log SCENE OUT.json [SQ_F64.csv]
"""
import csv
import json
import sys

KERNELS = ("k_extend",)          # matches k_extend<F> and k_extend_lds


def total(path, counter):
    tot = 0.0
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and any(k in r["Kernel_Name"] for k in KERNELS):
            tot += float(r["Counter_Value"])
    return tot


def rays_of(bench_log):
    line = [x for x in open(bench_log).read().splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    return d["extend_rays_per_step"] * d["steps"]


def sq_f64(path, rays):
    tot = {}
    for r in csv.DictReader(open(path)):
        if any(k in r["Kernel_Name"] for k in KERNELS):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ops = (tot.get("SQ_INSTS_VALU_ADD_F64", 0) + tot.get("SQ_INSTS_VALU_MUL_F64", 0)
           + 2 * tot.get("SQ_INSTS_VALU_FMA_F64", 0) + tot.get("SQ_INSTS_VALU_TRANS_F64", 0)) * 64
    return ops / rays, {k: v / rays * 64 for k, v in tot.items()}


def main():
    fetch_csv, write_csv, bench_log, scene, out = sys.argv[1:6]
    rays = rays_of(bench_log)
    fb = total(fetch_csv, "FETCH_SIZE") * 1024.0
    wb = total(write_csv, "WRITE_SIZE") * 1024.0
    res = {
        "kernel": "k_extend + k_extend_lds", "scene": scene, "segments": rays,
        "fetch_bytes_per_segment_raw": fb / rays, "fetch_bytes_per_segment": 2.0 * fb / rays,
        "write_bytes_per_segment": wb / rays,
        "bytes_per_segment": 2.0 * fb / rays + wb / rays,
        "algorithmic_bytes_per_segment": "64 + 36 per path-ending miss (bench.py extend_bytes)",
        "note": "FETCH_SIZE doubled (gfx950 wide-read under-count: ray records are 16-B loads)",
    }
    if len(sys.argv) > 6:
        res["f64_flops_per_segment"], res["sq_per_lane_segment"] = sq_f64(sys.argv[6], rays)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
