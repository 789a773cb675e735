#!/usr/bin/env python3
"""Per-kernel register / spill / LDS / scratch figures from the device
assembly (make -C scheme-raytrace_amd/csrc asm -> rt_kernels.s).
usage: python tools/kernel_regs.py [rt_kernels.s] [name-filter]"""
import re
import sys


def kernels(path):
    s = open(path).read()
    meta = s[s.index("amdhsa.kernels:"):]
    out = {}
    for blk in re.split(r"\n  - ", meta)[1:]:
        m = re.search(r"^    \.name:\s+(\S+)", blk, re.M)
        if not m:
            continue
        f = {k: int(re.search(r"^    \.%s:\s+(\d+)" % k, blk, re.M).group(1))
             for k in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                       "group_segment_fixed_size", "private_segment_fixed_size")
             if re.search(r"^    \.%s:" % k, blk, re.M)}
        out[m.group(1)] = f
    return out


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else "scheme-raytrace_amd/csrc/rt_kernels.s"
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, f in sorted(kernels(path).items()):
        if flt in name:
            print("%-90s vgpr %3d agpr %3d spill %3d lds %6d scratch %4d" % (
                name[:90], f.get("vgpr_count", 0), f.get("agpr_count", 0), f.get("vgpr_spill_count", 0),
                f.get("group_segment_fixed_size", 0), f.get("private_segment_fixed_size", 0)))
