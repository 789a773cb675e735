#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over k_extend into
profiles/pmc_extend.json: HBM bytes per ray segment.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in
KiB; FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read,
so it is doubled; WRITE_SIZE is taken as is.  Rays per launch = the launch's
Grid_Size (threads, = live paths rounded up to the 256-thread block).

usage: pmc_to_json.py FETCH.csv WRITE.csv SCENE OUT.json [SQ_F64.csv]

The optional SQ pass (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64) gives issued
f64 lane-ops per segment: (ADD + MUL + 2*FMA + TRANS) * 64 / rays.
"""
import csv
import json
import sys


def load(path, counter):
    tot, grid = 0.0, 0
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "k_extend" not in r["Kernel_Name"]:
            continue
        tot += float(r["Counter_Value"]) * 1024.0
        grid += int(r["Grid_Size"])
    return tot, grid


def sq_f64(path):
    tot, grids = {}, {}
    for r in csv.DictReader(open(path)):
        if "k_extend" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        grids[r["Dispatch_Id"]] = int(r["Grid_Size"])
    rays = sum(grids.values())
    ops = (tot.get("SQ_INSTS_VALU_ADD_F64", 0) + tot.get("SQ_INSTS_VALU_MUL_F64", 0)
           + 2 * tot.get("SQ_INSTS_VALU_FMA_F64", 0) + tot.get("SQ_INSTS_VALU_TRANS_F64", 0)) * 64
    return ops / rays, {k: v / rays * 64 for k, v in tot.items()}


def main():
    fetch_csv, write_csv, scene, out = sys.argv[1:5]
    fb, fg = load(fetch_csv, "FETCH_SIZE")
    wb, wg = load(write_csv, "WRITE_SIZE")
    res = {
        "kernel": "k_extend", "scene": scene,
        "fetch_bytes_per_segment_raw": fb / fg, "fetch_bytes_per_segment": 2.0 * fb / fg,
        "write_bytes_per_segment": wb / wg,
        "bytes_per_segment": 2.0 * fb / fg + wb / wg,
        "algorithmic_bytes_per_segment": "72 + 36 per path-ending miss (bench.py extend_bytes)",
        "launches_rays": [fg, wg],
        "note": "FETCH_SIZE doubled (gfx950 wide-read under-count); loads here are 8 B/lane SoA f64, "
                "a width the guide leaves uncalibrated",
    }
    if len(sys.argv) > 5:
        res["f64_flops_per_segment"], res["sq_per_wave_segment"] = sq_f64(sys.argv[5])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
