# GPU debug: the oracle's per-segment rays of the flat-curve scene's differing samples through rt_hit_rays
import json, os, sys
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(root, 'scheme-raytrace_amd'), os.path.join(root, 'tests'), os.path.join(root, 'oracle')]
import numpy as np
import oracle
from rtamd import gpu
from test_gpu_curves import _flat_curve_scene
np.set_printoptions(linewidth=220, precision=17)
nx = ny = 128
sc = _flat_curve_scene(nx, ny)
o = oracle.build_scene(sc)
cases = json.load(open(os.path.join(root, 'tools', 'dbg', 'cases.json')))
for j, s in cases:
    tr = o.trace_sample(nx, ny, j % nx, j // nx, 0x5EED0002, s)
    rays = np.concatenate([tr[:, 0:6], np.zeros((len(tr), 1))], axis=1)
    t, m = gpu.hit_rays(sc, rays)
    for k in range(len(tr)):
        ot, om = (tr[k, 7], int(tr[k, 11])) if tr[k, 6] else (0.0, -1)
        if ot != t[k] or om != m[k]:
            print("pixel %d sample %d segment %d: oracle t=%r mat=%d  gpu t=%r mat=%d" % (j, s, k, ot, om, t[k], m[k]))
            print("  ray", repr(list(tr[k, 0:6])))
            break
    else:
        print("pixel %d sample %d: all %d segments agree" % (j, s, len(tr)))
