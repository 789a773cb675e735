#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the shade kernels
(k_shade<material>) into profiles/pmc_shade.json: HBM bytes per shaded hit,
next to the algorithmic bytes per hit (bench.py shade_bytes) of the same run.

Same gfx950 corrections as tools/pmc_to_json.py: the counters are in KiB and
FETCH_SIZE, which reports half of the bytes of the 16-B record loads, is
doubled.  The hit counts come from the profiled bench run's own JSON line.

usage: pmc_shade_json.py FETCH.csv WRITE.csv BENCH.log SCENE OUT.json
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def total(path, counter):
    tot = 0.0
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and "k_shade" in r["Kernel_Name"]:
            tot += float(r["Counter_Value"])
    return tot


def main():
    from bench import shade_bytes
    fetch_csv, write_csv, bench_log, scene, out = sys.argv[1:6]
    d = json.loads([x for x in open(bench_log).read().splitlines() if x.startswith("{")][-1])
    steps = d["steps"]
    h0, h, sv = (d["shade_hits_d0_per_step"] * steps, d["shade_hits_per_step"] * steps,
                 d["shade_survivors_per_step"] * steps)
    hits = h0 + h
    fb = total(fetch_csv, "FETCH_SIZE") * 1024.0
    wb = total(write_csv, "WRITE_SIZE") * 1024.0
    res = {
        "kernel": "k_shade<material>", "scene": scene, "hits": hits,
        "fetch_bytes_per_hit_raw": fb / hits, "fetch_bytes_per_hit": 2.0 * fb / hits,
        "write_bytes_per_hit": wb / hits, "bytes_per_hit": (2.0 * fb + wb) / hits,
        "algorithmic_bytes_per_hit": shade_bytes(h0, h, sv) / hits,
        "note": "FETCH_SIZE doubled (gfx950 wide-read under-count: records are 16-B loads); leaf-record "
                "staging into LDS (scene data, L2-resident) is not algorithmic but is in the counters",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
