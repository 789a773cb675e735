# GPU debug: the flat-curve scene, per-sample frames under several schedules
import os, sys
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(root, 'scheme-raytrace_amd'), os.path.join(root, 'tests')]
import numpy as np
from rtamd import gpu
from test_gpu_curves import _flat_curve_scene
nx = ny = 128
out = {}
ctx = gpu.default_context(0)
for name, opts, env in [("tail", {"tail_paths": 100000000}, {}),
                        ("wave", {"tail_off": 1}, {}),
                        ("flatlist", {"tail_paths": 100000000}, {"RTAMD_BVH_MIN": "1000000000"})]:
    os.environ.pop("RTAMD_BVH_MIN", None)
    os.environ.update(env)
    ctx.reset_options()
    for k, val in opts.items():
        ctx.set_option(k, val)
    sc = _flat_curve_scene(nx, ny)
    for s in range(4):
        a = np.zeros(nx * ny * 3)
        gpu.render_host(sc, nx, ny, s, 1, 0x5EED0002, a)
        out["%s_%d" % (name, s)] = a
    print(name, "done", flush=True)
os.makedirs(os.path.join(root, "gpurun_out", "dbg"), exist_ok=True)
np.savez_compressed(os.path.join(root, "gpurun_out", "dbg", "flat.npz"), **out)
