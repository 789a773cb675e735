#!/usr/bin/env python3
"""Per-kernel PMC report of one bench frame (tools/profile_round.sh passes).

usage: pmc_report.py PROFILE_DIR BENCH_LOG OUT.json

PROFILE_DIR holds the rocprofv3 counter passes fetch/ write/ sq1/ sq2/ (one
frame each, same configuration) and the kernel-trace runs kt1/ (one render
lane) and kt2/ (two).  BENCH_LOG is one profiled run's log (its JSON line
gives the frame's item counts: segments, paths, shaded hits).

Per kernel family it writes: dispatches, device time per frame (kernel
trace), HBM bytes (FETCH_SIZE doubled, the gfx950 correction for 16-B
loads, MI355X_MICROARCH.md §HBM; WRITE_SIZE as is) per item, VALU busy
(share of SIMD cycles issuing VALU: VALUBusy), VALU lane utilisation
(VALUUtilization: active lanes per issued VALU instruction, i.e.
divergence), LDS busy (LdsUtil) and bank-conflict ratio, share of wave
cycles waiting (SQ_WAIT_ANY / wave cycles), occupancy, and per item VALU /
SALU / LDS instructions and f64 lane-ops.  Derived percentages are averaged
over dispatches weighted by GRBM_GUI_ACTIVE (each dispatch's busy cycles).

It also writes profiles/pmc/<scene>_extend.json and <scene>_shade.json, which
bench.py reads for roofline.traffic and the valu / valu_issue objects.
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def family(name):
    n = name.split("(")[0].replace("void ", "").replace("rtamd::", "")
    if n.startswith("k_shade"):
        mat = n[n.index("<") + 1:].split(",")[0] if "<" in n else "?"
        return "k_shade<%s>" % {"0": "lambertian", "1": "metal", "2": "dielectric", "3": "light"}.get(mat, mat)
    for k in ("k_extend_lds", "k_extend_curves", "k_extend", "k_camera", "k_finish", "k_raygen", "k_accumulate",
              "k_resolve_u8"):
        if n.startswith(k):
            return k
    return n[:40]


def read_counters(d):
    """{family: {counter: [(dispatch, value), ...]}} over every csv under d."""
    out = collections.defaultdict(lambda: collections.defaultdict(dict))
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            key = (p, r["Dispatch_Id"])
            out[family(r["Kernel_Name"])][r["Counter_Name"]][key] = \
                out[family(r["Kernel_Name"])][r["Counter_Name"]].get(key, 0.0) + float(r["Counter_Value"])
    return out


def kernel_ms(d):
    """{family: (calls, total ms)} from a kernel-trace stats csv under d."""
    res = collections.defaultdict(lambda: [0, 0.0])
    for p in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            f = family(r["Name"])
            res[f][0] += int(r["Calls"])
            res[f][1] += float(r["TotalDurationNs"]) / 1e6
    return {k: (v[0], round(v[1], 3)) for k, v in res.items()}


def main():
    pdir, bench_log, out_path = sys.argv[1:4]
    from bench import EXTEND_BYTES_PER_PATH, EXTEND_BYTES_PER_SEGMENT, shade_bytes
    # the bench line (its start can share a log line with stderr output written around it)
    d = json.loads([x[x.index('{"metric"'):] for x in open(bench_log).read().splitlines() if '{"metric"' in x][-1])
    steps = d["steps"]
    segs_wf = d["extend_rays_per_step"] * steps
    paths = d["paths_per_step"] * steps
    h0, h, sv = (d["shade_hits_d0_per_step"] * steps, d["shade_hits_per_step"] * steps,
                 d["shade_survivors_per_step"] * steps)
    tail = d["tail_segments_per_step"] * steps
    items = {"k_camera": paths, "k_extend_lds": segs_wf - paths, "k_extend": segs_wf, "k_finish": tail,
             "shade": h0 + h}
    fams = collections.defaultdict(dict)
    for sub in ("fetch", "write", "sq1", "sq2"):
        for fam, ctrs in read_counters(os.path.join(pdir, sub)).items():
            for c, disp in ctrs.items():
                fams[fam].setdefault(c, {}).update(disp)      # keys carry the pass's csv path
    ms1, ms2 = kernel_ms(os.path.join(pdir, "kt1")), kernel_ms(os.path.join(pdir, "kt2"))

    def tot(f, c):
        return sum(fams[f].get(c, {}).values())

    def wavg(f, metric):
        """GRBM_GUI_ACTIVE-weighted mean of a per-dispatch derived metric (same pass)."""
        vals, gui = fams[f].get(metric, {}), fams[f].get("GRBM_GUI_ACTIVE", {})
        num = den = 0.0
        for k, v in vals.items():
            w = gui.get(k, 0.0)
            num += v * w
            den += w
        return num / den if den else None

    report = {"config": d["config"]["workload"], "scene": d["config"]["scene"], "items_per_frame": items,
              "kernels": {}}
    for f in sorted(fams):
        n_items = items.get("shade" if f.startswith("k_shade") else f)
        r = {"dispatches": len(fams[f].get("FETCH_SIZE", {})) or len(fams[f].get("SQ_WAVES", {})),
             "ms_one_lane": ms1.get(f, (0, None))[1], "ms_two_lanes": ms2.get(f, (0, None))[1],
             "fetch_MB": round(2 * tot(f, "FETCH_SIZE") / 1024, 1), "write_MB": round(tot(f, "WRITE_SIZE") / 1024, 1)}
        for m in ("VALUBusy", "VALUUtilization", "LdsUtil", "LdsBankConflict", "OccupancyPercent"):
            v = wavg(f, m)
            r[m] = round(v, 3) if v is not None else None
        wc = tot(f, "SQ_WAVE_CYCLES")
        r["wait_share"] = round(tot(f, "SQ_WAIT_ANY") / wc, 3) if wc else None
        if n_items:
            r["items"] = n_items
            r["hbm_bytes_per_item"] = round((2 * tot(f, "FETCH_SIZE") + tot(f, "WRITE_SIZE")) * 1024 / n_items, 2)
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                r[c.lower().replace("sq_insts_", "") + "_instr_per_item"] = round(tot(f, c) / n_items, 3)
            f64 = (tot(f, "SQ_INSTS_VALU_ADD_F64") + tot(f, "SQ_INSTS_VALU_MUL_F64") +
                   2 * tot(f, "SQ_INSTS_VALU_FMA_F64") + tot(f, "SQ_INSTS_VALU_TRANS_F64")) * 64
            r["f64_lane_ops_per_item"] = round(f64 / n_items, 2)
        report["kernels"][f] = r

    # the extend phase (k_camera at depth 0, k_extend_lds / k_extend deeper): bench.py's roofline.traffic
    ext = [f for f in ("k_camera", "k_extend_lds", "k_extend", "k_extend_curves") if f in fams]
    fb = sum(tot(f, "FETCH_SIZE") for f in ext) * 1024
    wb = sum(tot(f, "WRITE_SIZE") for f in ext) * 1024
    f64 = sum((tot(f, "SQ_INSTS_VALU_ADD_F64") + tot(f, "SQ_INSTS_VALU_MUL_F64") + 2 * tot(f, "SQ_INSTS_VALU_FMA_F64")
               + tot(f, "SQ_INSTS_VALU_TRANS_F64")) * 64 for f in ext)
    gui = {f: fams[f].get("GRBM_GUI_ACTIVE", {}) for f in ext}

    def ext_avg(metric):
        num = den = 0.0
        for f in ext:
            for k, v in fams[f].get(metric, {}).items():
                num += v * gui[f].get(k, 0.0)
                den += gui[f].get(k, 0.0)
        return num / den if den else None

    alg = EXTEND_BYTES_PER_SEGMENT * segs_wf + EXTEND_BYTES_PER_PATH * paths
    pmc_ext = {"kernel": " + ".join(ext), "scene": report["scene"], "config": report["config"], "segments": segs_wf,
               "fetch_bytes_per_segment": 2 * fb / segs_wf, "write_bytes_per_segment": wb / segs_wf,
               "bytes_per_segment": (2 * fb + wb) / segs_wf, "algorithmic_bytes_per_segment": alg / segs_wf,
               "f64_flops_per_segment": f64 / segs_wf,
               "valu_busy": ext_avg("VALUBusy"), "valu_lane_utilization": ext_avg("VALUUtilization"),
               "lds_busy": ext_avg("LdsUtil"), "lds_bank_conflict_ratio": ext_avg("LdsBankConflict"),
               "wait_share": (sum(tot(f, "SQ_WAIT_ANY") for f in ext) / max(1.0, sum(tot(f, "SQ_WAVE_CYCLES")
                                                                                 for f in ext))),
               "valu_instr_per_segment": sum(tot(f, "SQ_INSTS_VALU") for f in ext) / segs_wf,
               "note": "one frame at the bench configuration; FETCH_SIZE doubled (16-B record loads)"}
    shf = [f for f in fams if f.startswith("k_shade")]
    hits = h0 + h
    sfb = sum(tot(f, "FETCH_SIZE") for f in shf) * 1024
    swb = sum(tot(f, "WRITE_SIZE") for f in shf) * 1024
    pmc_sh = {"kernel": "k_shade<material>", "scene": report["scene"], "config": report["config"], "hits": hits,
              "fetch_bytes_per_hit": 2 * sfb / hits, "write_bytes_per_hit": swb / hits,
              "bytes_per_hit": (2 * sfb + swb) / hits, "algorithmic_bytes_per_hit": shade_bytes(h0, h, sv) / hits,
              "note": "one frame at the bench configuration; FETCH_SIZE doubled (16-B record loads)"}
    report["extend_phase"] = pmc_ext
    report["shade_phase"] = pmc_sh
    # stamp: bench.py uses these counters only while the kernels are the ones they were measured on
    with open(os.path.join(ROOT, "scheme-raytrace_amd", "csrc", "rt_kernels.hip"), "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    for rec in (report, pmc_ext, pmc_sh):
        rec["kernel_sha16"] = sha
    json.dump(report, open(out_path, "w"), indent=1)
    # per scene (bench.py load_pmc: profiles/pmc/<scene>_{extend,shade}.json)
    os.makedirs(os.path.join(ROOT, "profiles", "pmc"), exist_ok=True)
    json.dump(pmc_ext, open(os.path.join(ROOT, "profiles", "pmc", "%s_extend.json" % report["scene"]), "w"), indent=1)
    json.dump(pmc_sh, open(os.path.join(ROOT, "profiles", "pmc", "%s_shade.json" % report["scene"]), "w"), indent=1)
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
