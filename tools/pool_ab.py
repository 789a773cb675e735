"""C2 (cover 1920x1080x1024 spp) at a few path-pool sizes (RT_OPT_MAX_PATHS), variants interleaved; each
size renders one untimed full frame first (a re-allocated pool's first frame waits for the driver to clear the
memory it reuses: tools/realloc_probe.py): [SCENE=curves SPP=256] python tools/pool_ab.py M1 M2 ...
(Mi paths; 0 = automatic)."""
import hashlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scheme-raytrace_amd"))
from rtamd import gpu, scenes  # noqa: E402

nx, ny = int(os.environ.get("NX", 1920)), int(os.environ.get("NY", 1080))
spp, seed = int(os.environ.get("SPP", 1024)), 0x5EED0002
sc = scenes.SCENES[os.environ.get("SCENE", "cover")](nx, ny)
ctx = gpu.default_context()
acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
for rnd in range(int(os.environ.get("ROUNDS", 2))):
    for m in [int(x) for x in sys.argv[1:]]:
        ctx.set_option("max_paths", m << 20)
        gpu.render_device(sc, nx, ny, 0, spp, seed, acc.data_ptr())     # sizes and first-touches the pools
        acc.zero_()
        torch.cuda.synchronize()
        t = time.perf_counter()
        h = gpu.render_device(sc, nx, ny, 0, spp, seed, acc.data_ptr())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        st = gpu.stats(h)
        print("round %d max_paths %dM: %.1f ms, %.0f Mrays/s, chunks %d lanes %d, sha %s" % (
            rnd, m, dt * 1e3, st.segments / dt / 1e6, st.chunks, st.lanes,
            hashlib.sha256(acc.cpu().numpy().tobytes()).hexdigest()[:16]), flush=True)
