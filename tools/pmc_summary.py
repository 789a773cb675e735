#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per counter, the sum over dispatches, and
per-segment ratios (rays = sum of Grid_Size of the kernel's dispatches)."""
import csv
import sys
from collections import defaultdict


def load(path):
    tot = defaultdict(float)
    grids = {}
    for r in csv.DictReader(open(path)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        grids[r["Dispatch_Id"]] = int(r["Grid_Size"])
    return tot, sum(grids.values())


if __name__ == "__main__":
    for path in sys.argv[1:]:
        tot, rays = load(path)
        print(path, "rays=%d" % rays)
        for k in sorted(tot):
            print("  %-28s %16.4g  per-wave-segment(x64/ray): %10.1f" % (k, tot[k], tot[k] / rays * 64))
