# GPU debug: localise the samples of test_few_curves_among_spheres_large_launch's band that differ from
# the oracle, then the first segment whose closest hit differs (the oracle's own rays through rt_hit_rays).
# If every segment's hit agrees, the divergence is in a scatter (a libm ulp, a division) and the
# per-segment materials / draw counters are printed for that sample.
import os
import sys

root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(root, 'scheme-raytrace_amd'), os.path.join(root, 'tests'), os.path.join(root, 'oracle')]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from rtamd import gpu, scenes  # noqa: E402
from rtamd import scene as g  # noqa: E402
from rtamd import vec as v  # noqa: E402
from rtamd.rng import HostStream  # noqa: E402

np.set_printoptions(linewidth=220, precision=17)
SEED = 0x5EED0002
nx, ny, spp = 960, 540, 16
y0, rows = int(os.environ.get("Y0", "250")), int(os.environ.get("ROWS", "8"))
objs = scenes.random_scene_objects(HostStream(scenes.SCENE_SEED))
gold = g.make_metal(g.constant_texture(v.vec3(0.8, 0.6, 0.2)), 0.05)
red = g.make_lambertian(g.constant_texture(v.vec3(0.65, 0.05, 0.05)))
objs.append(g.make_bezier(v.vec3(-6, 0.3, -2), v.vec3(-2, 2.5, 1), v.vec3(2, -0.5, 2), v.vec3(6, 1.5, -1), 0.15, gold))
objs.append(g.make_bezier(v.vec3(-3, 2.0, 3), v.vec3(0, 0.5, -3), v.vec3(3, 3.0, 1), v.vec3(5, 0.8, 2), 0.1, red))
sc = g.make_scene(objs, scenes.camera_for(nx, ny), g.sky_color)
o = oracle.build_scene(sc)
lo, hi = y0 * nx, (y0 + rows) * nx
nth = min(16, os.cpu_count() or 1)
found = []
for s in range(spp):
    a = np.zeros(nx * ny * 3)
    gpu.render_rows_host(sc, nx, ny, y0, rows, s, 1, SEED, a)
    r = np.zeros(nx * ny * 3)
    o.render(nx, ny, s, 1, SEED, r, lo, hi, nthreads=nth)
    d = np.abs(a[3 * lo:3 * hi] - r[3 * lo:3 * hi]).reshape(-1, 3).max(axis=1)
    for q in np.nonzero(d > 1e-12)[0]:
        found.append((lo + int(q), s, float(d[q])))
print("differing samples (pixel, sample, max channel diff):", found, flush=True)
for j, s, dd in found[:8]:
    x, y = j % nx, j // nx
    tr = o.trace_sample(nx, ny, x, y, SEED, s)
    rays = np.concatenate([tr[:, 0:6], np.zeros((len(tr), 1))], axis=1)
    ctr0 = int(tr[0, 12])
    rays[0, 6] = oracle.stream(SEED, j, s, ctr0 - 1, 1)[0]     # camera time = the camera's last draw (t0 0, t1 1)
    t, m = gpu.hit_rays(sc, rays)
    print("pixel %d (x %d y %d) sample %d diff %.3e: %d segments, materials %s" %
          (j, x, y, s, dd, len(tr), [int(q) for q in tr[:, 11]]), flush=True)
    for k in range(len(tr)):
        ot, om = (tr[k, 7], int(tr[k, 11])) if tr[k, 6] else (0.0, -1)
        if ot != t[k] or om != m[k]:
            print("  first differing hit at segment %d: oracle t=%r mat=%d  gpu t=%r mat=%d" % (k, ot, om, t[k], m[k]))
            print("  ray", repr(list(rays[k])))
            break
    else:
        print("  every segment's closest hit agrees: the divergence is in a scatter")
        for k in range(len(tr)):
            print("   seg %d o=%r d=%r t=%r mat=%d ctr=%d" % (k, list(tr[k, 0:3]), list(tr[k, 3:6]), tr[k, 7],
                                                              int(tr[k, 11]), int(tr[k, 12])))
