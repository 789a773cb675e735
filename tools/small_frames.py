"""Small frames (the progressive loop's one pass per call, main.scm:533-544; a rank's share of a multi-GPU
frame): C2's scene at NX x NY (default 1920x1080) and SPP per frame, timed over a few frames for each tail
threshold (RT_OPT_TAIL_PATHS, 0 = the library's choice) given on the command line.
Run on the GPU box: [SCENE=cornell NX=680 NY=381 FRAMES=3] python tools/small_frames.py SPP T1 T2 ..."""
import hashlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scheme-raytrace_amd"))
from rtamd import gpu, scenes  # noqa: E402

spp = int(sys.argv[1])
tails = sys.argv[2:] or ["0"]           # N: RT_OPT_TAIL_PATHS = N; dN: RT_OPT_TAIL_DIV = N
nx, ny = int(os.environ.get("NX", 1920)), int(os.environ.get("NY", 1080))
seed, frames = 0x5EED0002, int(os.environ.get("FRAMES", 20))
sc = scenes.SCENES[os.environ.get("SCENE", "cover")](nx, ny)
ctx = gpu.default_context()
acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
ref = None
for rnd in range(2):
    for tp in tails:
        if tp.startswith("d"):
            ctx.set_option("tail_paths", 0)
            ctx.set_option("tail_div", int(tp[1:]))
        else:
            ctx.set_option("tail_div", 0)
            ctx.set_option("tail_paths", int(tp))
        gpu.render_device(sc, nx, ny, 0, spp, seed, acc.data_ptr())      # warmup
        torch.cuda.synchronize()
        acc.zero_()
        torch.cuda.synchronize()
        t = time.perf_counter()
        segs = 0
        for f in range(frames):
            h = gpu.render_device(sc, nx, ny, f * spp, spp, seed, acc.data_ptr())
            segs += gpu.stats(h).segments
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / frames
        img = acc.cpu().numpy()
        same = "ref" if ref is None else ("same" if (img == ref).all() else "DIFFERENT")
        if ref is None:
            ref = img
        print("round %d spp %d tail %s: %.3f ms/frame, %.0f Mrays/s (segments), image %s sha %s"
              % (rnd, spp, tp, dt * 1e3, segs / frames / dt / 1e6, same,
                 hashlib.sha256(img.tobytes()).hexdigest()[:16]), flush=True)
