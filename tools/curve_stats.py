#!/usr/bin/env python3
"""Curve-kernel statistics (stats build only): where k_extend_curves spends
its wave cycles and how busy stage B's lanes are.

Build:  make -C scheme-raytrace_amd/csrc EXTRA=-DRT_STATS OUT=../rtamd/librtamd_stats.so
Run:    RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_stats.so python3 tools/curve_stats.py [spp]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scheme-raytrace_amd"))


def main():
    import numpy as np
    from rtamd import gpu, scenes, _lib
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    nx, ny = 1920, 1080
    lib = ctypes.CDLL(_lib.LIB_PATH)
    b = (ctypes.c_ulonglong * 48)()
    ctx = gpu.default_context(0)
    ctx.set_option("lanes", 1)
    ctx.set_option("tail_off", 1)              # the wavefront curve kernel at every depth
    sc = scenes.cornell_curves(nx, ny)
    acc = np.zeros(nx * ny * 3)
    gpu.render_host(sc, nx, ny, 0, 1, 0x5EED0002, acc)          # upload + warm
    lib.rt_debug_stats(b, 1)
    gpu.render_host(sc, nx, ny, 0, spp, 0x5EED0002, acc)
    lib.rt_debug_stats(b, 1)
    waves = max(1, b[24])
    out = {
        "queries": b[11], "bvh_nodes_per_query": b[12] / max(1, b[11]), "leaves_per_query": b[13] / max(1, b[11]),
        "kernel_waves": b[24], "kernel_clock_per_wave": b[40] / waves,
        "stage_a_share": b[41] / max(1, b[40]), "stage_b_share": b[39] / max(1, b[40]),
        "stage_b_passes": b[31], "survivors": b[38], "survivors_per_pass": b[38] / max(1, b[31]),
        "stage_b_lane_util": b[33] / max(1, 64 * b[32]),
        "steps_per_survivor": b[34] / max(1, b[38]), "rederived_per_survivor": b[35] / max(1, b[38]),
        "rederive_splits_per_survivor": b[36] / max(1, b[38]), "leaf_tests_per_survivor": b[37] / max(1, b[38]),
        "kernel_lane_busy": b[21] / max(1, 64 * b[23]),
        "kernel_lane_bvh_step": b[20] / max(1, 64 * b[23]), "kernel_lane_wait": b[22] / max(1, 64 * b[23]),
        "kernel_iters_per_wave": b[23] / waves, "flushes_per_wave": b[25] / waves,
        "kernel_clock_per_iter": b[40] / max(1, b[23]),
        "step1_finish_share": b[42] / max(1, b[40]), "step2_claim_share": b[43] / max(1, b[40]),
        "step3_bvh_share": b[44] / max(1, b[40]), "stage_b_refill_share": b[45] / max(1, b[40]),
        "stage_b_leaf_share": b[46] / max(1, b[40]), "stage_b_node_share": b[47] / max(1, b[40]),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
