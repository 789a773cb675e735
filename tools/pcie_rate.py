"""The host-buffer boundary's rate: C2 (cover 1920x1080x1024 spp) through rt_render (the
caller's accumulator in host memory: copied to the device and back around the render) against
rt_render_device (the accumulator already in HBM, bench.py's `value`), one frame each after a warmup frame.
Run on the GPU box: python tools/pcie_rate.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scheme-raytrace_amd"))
from rtamd import gpu, scenes  # noqa: E402

nx, ny, spp, seed = 1920, 1080, 1024, 0x5EED0002
sc = scenes.random_scene(nx, ny)
acc_h = np.zeros(nx * ny * 3)
acc_d = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
gpu.render_device(sc, nx, ny, 0, 16, seed, acc_d.data_ptr())          # warmup (pools, LDS sizing)
torch.cuda.synchronize()
res = {}
imgs = {}
for name in ("device", "host", "device", "host"):
    acc_h[:] = 0.0
    acc_d.zero_()
    torch.cuda.synchronize()
    t = time.perf_counter()
    if name == "host":
        gpu.render_host(sc, nx, ny, 0, spp, seed, acc_h)
    else:
        gpu.render_device(sc, nx, ny, 0, spp, seed, acc_d.data_ptr())
        torch.cuda.synchronize()
    dt = time.perf_counter() - t
    res.setdefault(name, []).append(dt)
    segs = gpu.stats(gpu.upload(sc)).segments
    imgs.setdefault(name, []).append(acc_h.copy() if name == "host" else acc_d.cpu().numpy())
    print("%s: %.1f ms, %.0f Mrays/s (ray segments), %d segments" % (name, dt * 1e3, segs / dt / 1e6, segs), flush=True)
pairs = [(imgs["device"][0], imgs["device"][1], "device/device"), (imgs["host"][0], imgs["host"][1], "host/host"),
         (imgs["device"][0], imgs["host"][0], "device/host")]
for x, y, name in pairs:
    d = np.abs(x - y)
    print("%s: equal %s, max diff %.3e, pixels differing %d" % (name, np.array_equal(x, y), d.max(),
                                                                 int((d.reshape(-1, 3).max(axis=1) > 0).sum())))
print("accumulator %.1f MB each way; host-path overhead %.2f ms per frame"
      % (acc_h.nbytes / 1e6, (min(res["host"]) - min(res["device"])) * 1e3))
