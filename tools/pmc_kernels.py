#!/usr/bin/env python3
"""Per-kernel PMC summary from rocprofv3 counter CSVs (any number of passes).

usage: tools/pmc_kernels.py DIR [DIR...]
Prints, per kernel: dispatches, waves, per-wave SQ counts, VALU busy
(ACTIVE_INST_VALU x 4 / BUSY_CYCLES-normalised), fetch / write MB.
"""
import collections
import csv
import glob
import os
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rtamd::", "")
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((p, r["Dispatch_Id"]))
    for k, d in sorted(agg.items()):
        w = d.get("SQ_WAVES", 0) or 1
        out = {c: round(v / w, 1) for c, v in d.items() if c.startswith("SQ_") and c != "SQ_WAVES"}
        print("%-22s waves %9d" % (k, d.get("SQ_WAVES", 0)))
        print("   per wave:", out)
        mb = {c: round(v / 1024, 1) for c, v in d.items() if c in ("FETCH_SIZE", "WRITE_SIZE")}
        tc = {c: v for c, v in d.items() if c.startswith("TC")}
        print("   MB:", mb, " TC:", {c: "%.3g" % v for c, v in tc.items()})


if __name__ == "__main__":
    main()
