#!/usr/bin/env python3
"""Time one scene commit (C5's 2^20 curves by default) through the C ABI; with a library built
-DRT_COMMIT_PROFILE (make OUT=../rtamd/librtamd_prof.so EXTRA=-DRT_COMMIT_PROFILE, selected with
RTAMD_LIB) rt_scene_commit prints its phases on stderr.  usage: tools/commit_profile.py [scene]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scheme-raytrace_amd"))
from rtamd import gpu, scenes  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "curves"
t0 = time.perf_counter()
sc = scenes.SCENES[name](1920, 1080)
t1 = time.perf_counter()
h = gpu.upload(sc)
t2 = time.perf_counter()
info = gpu.scene_info(h)
print("scene %s: build %.1f ms, upload (constructors + commit) %.1f ms, commit %.1f ms (sah %.1f on %d threads, "
      "device %.1f)" % (name, (t1 - t0) * 1e3, (t2 - t1) * 1e3, info["commit_ms"], info["commit_sah_ms"],
                        info["commit_threads"], info["commit_upload_ms"]))
