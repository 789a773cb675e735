# GPU debug: the flat-curve scene, per-sample frames under several schedules
import os, sys
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(root, 'scheme-raytrace_amd'), os.path.join(root, 'tests')]
import numpy as np
from rtamd import gpu
from test_gpu_curves import _flat_curve_scene
nx = ny = 128
out = {}
for name, env in [("tail", {"RTAMD_TAIL_PATHS": "100000000"}),
                  ("wave", {"RTAMD_TAIL_PATHS": "0", "RTAMD_TAIL_DIV": "1000000000"}),
                  ("flatlist", {"RTAMD_TAIL_PATHS": "100000000", "RTAMD_BVH_MIN": "1000000000"})]:
    for k in ("RTAMD_TAIL_PATHS", "RTAMD_TAIL_DIV", "RTAMD_BVH_MIN"):
        os.environ.pop(k, None)
    os.environ.update(env)
    sc = _flat_curve_scene(nx, ny)
    for s in range(4):
        a = np.zeros(nx * ny * 3)
        gpu.render_host(sc, nx, ny, s, 1, 0x5EED0002, a)
        out["%s_%d" % (name, s)] = a
    print(name, "done", flush=True)
os.makedirs(os.path.join(root, "gpurun_out", "dbg"), exist_ok=True)
np.savez_compressed(os.path.join(root, "gpurun_out", "dbg", "flat.npz"), **out)
