"""The pixel driver: trace-all / trace-line / save-as-ppm (main.scm:439-491).

``Renderer`` owns the reference's globals *size-x*, *size-y*, *raw-data*
(running f64 sum, nx*ny*3, y-up rows) and *image* (u8).  ``trace_all(scene,
sample_count)`` is one pass exactly like the reference's: it adds sample
number ``sample_count`` (1-based) to every pixel and re-resolves the image
with sqrt(sum/sample_count).  ``trace_line(scene, y, sample_count)`` is the
reference's per-row pass (main.scm:452-469) and ``animate(scene)`` its GLUT
display step (main.scm:533-544: one row per call, then the next pass).
``render(scene, spp)`` runs many passes in one GPU call (same result as spp
successive trace_all calls).
"""
import numpy as np

from . import gpu

DEFAULT_SEED = 0x5EED0002


class Renderer:
    def __init__(self, nx, ny, seed=DEFAULT_SEED, ctx=None):
        self.size_x, self.size_y = int(nx), int(ny)
        self.seed = int(seed)
        self.ctx = ctx
        self.raw_data = np.zeros(self.size_x * self.size_y * 3, dtype=np.float64)
        self.image = np.zeros(self.size_x * self.size_y * 3, dtype=np.uint8)
        self.sample_count = 0
        self.current_y = 0            # *current-y* (main.scm:431)
        self.anim_sample_count = 1    # *sample-count* (main.scm:531)

    def trace_all(self, scene, sample_count):
        """main.scm:471-491 — one sample per pixel (pass `sample_count`)."""
        if sample_count < 1:
            raise ValueError("sample-count is 1-based")
        gpu.render_host(scene, self.size_x, self.size_y, sample_count - 1, 1, self.seed, self.raw_data, self.ctx)
        self.image = gpu.resolve_u8(self.raw_data, self.size_x, self.size_y, sample_count)
        self.sample_count = sample_count
        return self.image

    def trace_line(self, scene, y, sample_count):
        """main.scm:452-469 — sample number `sample_count` (1-based) of row y only,
        and row y of the image re-resolved; animate (main.scm:533-544) calls it
        row by row, so a full sweep equals trace_all(scene, sample_count)."""
        if sample_count < 1:
            raise ValueError("sample-count is 1-based")
        if not 0 <= y < self.size_y:
            raise ValueError("row outside the image")
        gpu.trace_line(scene, self.size_x, self.size_y, y, sample_count, self.seed, self.raw_data, self.image,
                       self.ctx)
        return self.image

    def animate(self, scene):
        """One display callback of main.scm:533-544 with *rendering?* on: trace
        the current row; after the last row start the next sample pass."""
        if self.current_y < self.size_y:
            self.trace_line(scene, self.current_y, self.anim_sample_count)
            self.current_y += 1
        else:
            self.anim_sample_count += 1
            self.current_y = 0
        return self.image

    def render(self, scene, spp, spp_begin=None):
        """Passes spp_begin+1 .. spp_begin+spp in one call (default: continue)."""
        if spp_begin is None:
            spp_begin = self.sample_count
        gpu.render_host(scene, self.size_x, self.size_y, spp_begin, spp, self.seed, self.raw_data, self.ctx)
        self.sample_count = spp_begin + spp
        self.image = gpu.resolve_u8(self.raw_data, self.size_x, self.size_y, self.sample_count)
        return self.image

    def save_as_ppm(self, path="test.ppm"):
        """main.scm:439-450 — P3, rows written top-down (flipping y-up rows)."""
        write_ppm(path, self.image, self.size_x, self.size_y)


def write_ppm(path, image, nx, ny):
    img = np.asarray(image, dtype=np.uint8).reshape(ny, nx, 3)
    with open(path, "w") as f:
        f.write("P3\n %d %d\n255\n" % (nx, ny))
        for y in range(ny):
            row = img[ny - y - 1]
            f.write("".join("%d %d %d\n" % (int(p[0]), int(p[1]), int(p[2])) for p in row))
