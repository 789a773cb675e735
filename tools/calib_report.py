#!/usr/bin/env python3
"""Counter factors of tools/calib_fetch.hip: per pattern, each counter's bytes
over the pattern's algorithmic bytes.  usage: calib_report.py DIR PROG_LOG OUT.json
DIR holds one rocprofv3 --pmc run per subdirectory (fetch/, write/, req/)."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, log, out = sys.argv[1:4]
    algo = {}
    for line in open(log):
        if line.startswith("{"):
            r = json.loads(line)
            algo[r["pattern"]] = r["algo_bytes"]
    vals = collections.defaultdict(dict)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k not in algo:
                continue
            vals[k][r["Counter_Name"]] = vals[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    res = {}
    for k, a in algo.items():
        v = vals.get(k, {})
        row = {"algo_bytes": a}
        if "FETCH_SIZE" in v:
            row["FETCH_SIZE_over_algo"] = round(v["FETCH_SIZE"] * 1024 / a, 4)   # FETCH_SIZE is in KB
        if "WRITE_SIZE" in v:
            row["WRITE_SIZE_over_algo"] = round(v["WRITE_SIZE"] * 1024 / a, 4)
        r32, r64, r128 = (v.get("TCC_EA0_RDREQ_32B_sum"), v.get("TCC_EA0_RDREQ_64B_sum"),
                          v.get("TCC_EA0_RDREQ_128B_sum"))
        if v.get("TCC_EA0_RDREQ_sum") is not None:
            row["rdreq"] = v["TCC_EA0_RDREQ_sum"]
            row["rdreq_32B"], row["rdreq_64B"], row["rdreq_128B"] = r32, r64, r128
        res[k] = row
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
