"""Does re-allocating the path pools slow the render?  C2 (cover 1920x1080x1024 spp), frames in one process:
two on the first pools, then rounds of rt_context_release_pools + two frames on the re-allocated pools."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scheme-raytrace_amd"))
from rtamd import gpu, scenes  # noqa: E402

nx, ny, spp, seed = 1920, 1080, 1024, 0x5EED0002
sc = scenes.random_scene(nx, ny)
ctx = gpu.default_context()
acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
free0, total = torch.cuda.mem_get_info()
print("device memory: free %.1f GB of %.1f GB" % (free0 / 1e9, total / 1e9), flush=True)
for rnd in range(4):
    if rnd:
        ctx.release_pools()
        torch.cuda.synchronize()
    for f in range(2):
        acc.zero_()
        torch.cuda.synchronize()
        t = time.perf_counter()
        h = gpu.render_device(sc, nx, ny, 0, spp, seed, acc.data_ptr())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        st = gpu.stats(h)
        free, _ = torch.cuda.mem_get_info()
        print("pools %d frame %d: %.1f ms, %.0f Mrays/s, chunks %d, free after %.1f GB" % (
            rnd, f, dt * 1e3, st.segments / dt / 1e6, st.chunks, free / 1e9), flush=True)
