#!/usr/bin/env python3
"""BVH traversal statistics per closest-hit query (stats build only).

Build:  make -C scheme-raytrace_amd/csrc EXTRA=-DRT_STATS OUT=../rtamd/librtamd_stats.so
Run:    RTAMD_LIB=scheme-raytrace_amd/rtamd/librtamd_stats.so python3 tools/trav_stats.py [scene] [spp]
Prints node visits, leaf visits and sphere / moving-sphere tests per query,
for the all-times tree (camera rays) and the time-0 tree (scattered rays).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scheme-raytrace_amd"))


def main():
    import json
    import numpy as np
    from rtamd import gpu, scenes, _lib
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "cover"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    nx, ny = 1920, 1080
    lib = ctypes.CDLL(_lib.LIB_PATH)
    buf = (ctypes.c_ulonglong * 48)()
    out = {}
    for mode in ("bvh0", "no_bvh0"):
        if mode == "no_bvh0":
            os.environ["RTAMD_NO_BVH0"] = "1"
        sc = scenes.SCENES[scene_name](nx, ny)
        acc = np.zeros(nx * ny * 3)
        lib.rt_debug_stats(buf, 1)
        gpu.render_host(sc, nx, ny, 0, spp, 0x5EED0002, acc)
        lib.rt_debug_stats(buf, 1)
        r = {}
        for tag, o in (("all_times", 0), ("time0", 16)):
            n = buf[o]
            w = max(1, buf[o + 7])
            if n:
                r[tag] = {"queries": n, "nodes": buf[o + 1] / n, "leaves": buf[o + 2] / n,
                          "sphere_tests": buf[o + 3] / n, "msphere_tests": buf[o + 4] / n,
                          "lane_inner_iters": buf[o + 5] / n, "lane_outer_iters": buf[o + 6] / n,
                          "wave_max_inner_iters": buf[o + 8] / w, "wave_max_outer_iters": buf[o + 9] / w,
                          "lanes_per_wave": buf[o + 10] / w}
        if buf[11]:
            n = buf[11]
            r["curves"] = {"queries": n, "nodes": buf[12] / n, "leaves": buf[13] / n, "candidates": buf[14] / n,
                           "root_survivors": buf[15] / n, "flushes_per_wave_query": buf[27] * 64.0 / n,
                           "wave_loop_iters": buf[28] / max(1, buf[29]), "lanes_per_wave": buf[30] / max(1, buf[29]),
                           "lane_steps": (buf[12] + buf[13]) / n}
        if buf[24]:
            w = buf[24]
            r["curves_persistent"] = {"waves": w, "wave_iters": buf[23] / w, "lane_steps_per_wave_iter": buf[20] / buf[23] / 64,
                                      "lane_busy_frac": buf[21] / buf[23] / 64, "lane_wait_frac": buf[22] / buf[23] / 64,
                                      "flushes_per_wave": buf[25] / w}
        out[mode] = r
        if scene_name.startswith("curves"):
            break
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
