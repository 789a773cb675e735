import faulthandler, sys, os, time
faulthandler.dump_traceback_later(50, exit=True)
sys.path.insert(0, "scheme-raytrace_amd")
import numpy as np, torch
from rtamd import gpu, scenes
for (nx, ny, spp) in [(64, 36, 4), (320, 180, 16), ]:
    t = time.time()
    sc = scenes.SCENES["cover"](nx, ny)
    acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda:0")
    gpu.render_device(sc, nx, ny, 0, spp, 0x5EED0002, acc.data_ptr())
    torch.cuda.synchronize()
    print(nx, ny, spp, "ok %.2fs" % (time.time() - t), float(acc.sum()), flush=True)
