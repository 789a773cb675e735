#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by EXECUTING THE REFERENCE.

Builder tooling, run only in the build container (it reads the reference's
.scm files from /root/reference; the GPU box never sees them):

    python tests/golden/make_golden.py

It loads the reference (soma-arc/scheme-raytrace) with tests/golden/
minischeme.py, binds srfi-27 `random-real` to the drop-in's counter-based
streams (rtamd.rng: host stream for load / scene-construction draws, the
per-(pixel, sample) path stream while a pixel is traced) and records:

* ref_kat.json   — reference functions on fixed inputs: reflect, refract,
                   schlick (material.scm), random-cosine-direction (util.scm),
                   make-onb-from-w / local (onb.scm), make-camera / get-ray
                   (camera.scm), Perlin tables drawn at module load,
                   noise / turb (perlin.scm), textures, sphere / rect / box
                   hits through the closure protocol (geometry.scm).
* ref_<scene>.json — per-(pixel, sample) colours of `color` (main.scm:100-121)
                   driven exactly as trace-all's per-pixel body
                   (main.scm:476-479, the expression is read from main.scm),
                   plus the running sum and the u8 image (main.scm:480-491).

Repairs, applied as overlays in the `main` module and
nowhere else:
  R1  (g:make-scene obj-list) with one argument (main.scm:89) completes the
      scene with *camera* and sky-color.
  R2  make-metal / make-dielectric results are wrapped to the 4-slot material
      protocol color expects: scatter returns (valid scattered att 1),
      scattering-pdf returns 1, emitted returns #f64(0 0 0).
  R3  *size-x* / *size-y* are set to the fixture's size and the reference's
      own (define *camera* ...) / (define *cornell-camera* ...) forms are
      re-evaluated, so the aspect is nx/ny.
Floats are stored as float.hex() strings (exact).
"""
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "scheme-raytrace_amd"))

import minischeme as ms  # noqa: E402
from rtamd import rng  # noqa: E402
from rtamd.scenes import PERLIN_SEED, SCENE_SEED  # noqa: E402

PATH_SEED = 0x5EED0002

OVERLAY = r"""
(define repair:orig-make-metal m:make-metal)
(define repair:orig-make-dielectric m:make-dielectric)
(define repair:orig-make-scene g:make-scene)
(define (repair:specular mat)
  (vector (lambda (ray hit-rec)
            (receive (valid? scattered attenuation) ((vector-ref mat 0) ray hit-rec)
              (values valid? scattered attenuation 1)))
          (lambda (ray hit-rec scattered) 1)
          (lambda (ray hit-rec u v p) (v:vec3 0 0 0))
          mat))
(define (m:make-metal albedo fuzz) (repair:specular (repair:orig-make-metal albedo fuzz)))
(define (m:make-dielectric ref-idx) (repair:specular (repair:orig-make-dielectric ref-idx)))
(define (g:make-scene obj-list . rest)
  (if (null? rest)
      (repair:orig-make-scene obj-list *camera* sky-color)
      (apply repair:orig-make-scene obj-list rest)))
"""


def H(x):
    if isinstance(x, (list, tuple)):
        return [H(v) for v in x]
    if isinstance(x, bool) or x is None:
        return x
    if isinstance(x, complex):
        return None
    return float(x).hex()


class Ref:
    def __init__(self):
        self.it = ms.Interp(REF)
        # perlin tables are drawn at module load (perlin.scm:32-36)
        self.it.random_real = rng.HostStream(PERLIN_SEED)
        self.perlin = self.it.load_module("perlin")
        self.it.random_real = rng.HostStream(0xC0FFEE)     # main.scm's own load-time scenes (unused)
        self.main = self.it.load_module("main")
        self.forms = ms.read_all(open(os.path.join(REF, "main.scm")).read())
        for f in ms.read_all(OVERLAY):
            self.it.eval(f, self.main)

    def ev(self, src, mod=None):
        out = None
        for f in ms.read_all(src):
            out = self.it.eval(f, mod or self.main)
        return out

    def define_form(self, name):
        for f in self.forms:
            if isinstance(f, ms.Pair) and f.car == "define":
                t = f.cdr.car
                n = t.car if isinstance(t, ms.Pair) else t
                if n == name:
                    return f
        raise KeyError(name)

    def set_size(self, nx, ny):
        self.main.own[ms.sym("*size-x*")] = nx
        self.main.own[ms.sym("*size-y*")] = ny
        for cam in ("*camera*", "*cornell-camera*"):                 # R3
            self.it.eval(self.define_form(cam), self.main)

    def pixel_body(self):
        """trace-all's per-pixel colour expression (main.scm:476-479), read
        from main.scm, wrapped as (lambda (x y scene) ...)."""
        ta = self.define_form("trace-all")
        body = ta.cdr.cdr.car            # (dotimes (y ...) (dotimes (x ...) (let* (...) ...)))
        inner = ms.to_list(body)[2]      # (dotimes (x *size-x*) (let* ...))
        let_star = ms.to_list(inner)[2]
        bindings = ms.to_list(let_star.cdr.car)
        col = [b for b in bindings if b.car == "col"][0]
        expr = col.cdr.car
        lam = ms.from_list([ms.sym("lambda"), ms.from_list([ms.sym("x"), ms.sym("y"), ms.sym("scene")]), expr])
        return self.it.eval(lam, self.main)


def _bezier_rays():
    """Rays aimed at points of the two KAT curves (plus misses): from a camera
    like *camera*, straight down z (the d == 0 branch of get-projection-mat,
    bezier.scm:24-31), with short (|d| < 1) and long directions."""
    def bez(cp, t):
        u = 1 - t
        return [cp[0][k] * u ** 3 + 3 * cp[1][k] * u * u * t + 3 * cp[2][k] * u * t * t + cp[3][k] * t ** 3
                for k in range(3)]
    c1 = [(-1, 0, -1), (-0.8, 1, 1), (0.8, -1, 1), (1, 0, -1)]
    c2 = [(130, 0, 65), (150, 0, 190), (130, 0, 190), (265, 0, 295)]
    out = []
    for t in (0.05, 0.3, 0.5, 0.77, 0.95):
        p = bez(c1, t)
        for o, sc in (((0, 5, 5), 1.0), ((0.3, 2, 6), 0.5), ((-3, 0.5, 1), 2.0)):
            d = [(p[k] - o[k]) * sc for k in range(3)]
            out.append((o, tuple(d), 0.0))
            out.append((o, (d[0] + 0.01, d[1], d[2] - 0.02), 0.0))
        out.append(((p[0], p[1], 4.0), (0.0, 0.0, -1.0), 0.0))          # along -z
        out.append(((p[0] + 0.03, p[1], -4.0), (0.0, 0.0, 1.0), 0.0))   # along +z, offset inside width
        q = bez(c2, t)
        out.append(((278, 278, -800), tuple(q[k] - (278, 278, -800)[k] for k in range(3)), 0.0))
        out.append(((278, 400, 100), tuple(q[k] - (278, 400, 100)[k] for k in range(3)), 0.0))
    out.append(((0, 5, 5), (0, 1, 0), 0.0))                              # miss
    return out


def kat(ref):
    it = ref.it
    out = {}
    mat_mod = it.modules["material"]
    util = it.modules["util"]
    onb = it.modules["onb"]
    cam = it.modules["camera"]
    def vec3(v):
        return ms.F64Vec(float(x) for x in v)

    def call(mod, name, *a):
        return mod.lookup(ms.sym(name))(*a)
    out["reflect"] = [[H(v), H(n), H(call(mat_mod, "reflect", vec3(v), vec3(n)))] for v, n in
                      [((1.0, -1.0, 0.5), (0.0, 1.0, 0.0)), ((0.3, 0.2, -0.9), (0.267, 0.534, 0.801))]]
    rf = []
    for v, n, ni in [((0.6, -0.8, 0.0), (0.0, 1.0, 0.0), 1 / 1.5), ((1.2, -1.6, 0.0), (0.0, 1.0, 0.0), 1 / 1.5),
                     ((0.9, 0.1, 0.0), (0.0, 1.0, 0.0), 1.5), ((0.1, -0.7, 0.3), (0.0, 0.0, 1.0), 1.5)]:
        r = call(mat_mod, "refract", vec3(v), vec3(n), ni)
        rf.append([H(v), H(n), H(ni), bool(r[0]), H(r[1]) if r[0] else None])
    out["refract"] = rf
    out["schlick"] = [[H(c), H(r), H(call(mat_mod, "schlick", c, r))] for c, r in
                      [(0.0, 1.5), (0.25, 1.5), (0.7, 1.5), (1.0, 1.5), (0.9, 1 / 1.5)]]
    cd = []
    for r1, r2 in [(0.125, 0.64), (0.9, 0.01), (0.5, 0.5)]:
        seq = iter([r1, r2])
        it.random_real = lambda s=seq: next(s)
        cd.append([H(r1), H(r2), H(call(util, "random-cosine-direction"))])
    out["cosine_direction"] = cd
    ob = []
    for nrm in [(0.0, 1.0, 0.0), (0.95, 0.1, 0.2), (-0.3, 0.4, 5.0)]:
        b = call(onb, "make-onb-from-w", vec3(nrm))
        ob.append([H(nrm), H(b[0]), H(b[1]), H(b[2])])
    out["onb"] = ob
    # camera + get-ray (camera.scm:63-92) with a scripted random stream
    c = call(cam, "make-camera", vec3((0, 5, 5)), vec3((0, 0, 0)), vec3((0, 1, 0)), 40, ms.div(1920, 1080), 0, 1,
             0, 1)
    out["camera_cover_1920x1080"] = [H(c[k]) for k in range(7)] + [H(c[7]), H(c[8]), H(c[9])]
    c2 = call(cam, "make-camera", vec3((13, 2, 3)), vec3((0, 0, 0)), vec3((0, 1, 0)), 20, ms.div(3, 2), 0.1, 10,
              0, 1)
    out["camera_lens"] = [H(c2[k]) for k in range(7)] + [H(c2[7]), H(c2[8]), H(c2[9])]
    seq = iter([0.9, 0.95, 0.3, 0.6, 0.25])          # disk rejects (0.9,0.95) then accepts, then time
    it.random_real = lambda s=seq: next(s)
    r = call(cam, "get-ray", c2, 0.25, 0.75)
    out["get_ray_lens"] = {"s": H(0.25), "t": H(0.75), "origin": H(r[0]), "dir": H(r[1]), "time": H(r[2])}
    # Perlin tables drawn at load with the host stream PERLIN_SEED
    P = ref.perlin
    out["perlin_seed"] = PERLIN_SEED
    out["perlin_ranvec"] = [H(v) for v in P.own[ms.sym("+ranvec+")]]
    out["perlin_perm"] = [list(P.own[ms.sym(n)]) for n in ("+perm-x+", "+perm-y+", "+perm-z+")]
    noise = P.lookup(ms.sym("noise"))
    turb = P.lookup(ms.sym("turb"))
    pts = [(0.3, 0.7, 1.1), (-2.5, 0.25, 7.75), (123.4, -55.5, 0.001), (0.0, 0.0, 0.0)]
    out["noise"] = [[H(p), H(noise(vec3(p)))] for p in pts]
    out["turb"] = [[H(p), H(turb(vec3(p)))] for p in pts]
    tex = it.modules["texture"]
    marble = call(tex, "marble-texture", 1)
    checker = call(tex, "checker-texture", call(tex, "constant-texture", vec3((0.2, 0.3, 0.1))),
                   call(tex, "constant-texture", vec3((0.9, 0.9, 0.9))))
    out["marble"] = [[H(p), H(marble[0](0, 0, vec3(p)))] for p in pts]
    out["checker"] = [[H(p), H(checker[0](0, 0, vec3(p)))] for p in pts + [(-0.1, 0.2, 0.3), (0.5, -1.7, 2.2)]]
    # closest hits through the closure protocol (geometry.scm)
    hits = {}
    setup = {
        "spheres": "(list (g:make-sphere (v:vec3 0 0 -1) 0.5 (m:make-lambertian (t:constant-texture (v:vec3 1 0 0))))"
                   " (g:make-sphere (v:vec3 0 -100.5 -1) 100 (m:make-lambertian (t:constant-texture (v:vec3 0 1 0))))"
                   " (g:make-sphere (v:vec3 -1 0 -1) -0.45 (m:make-dielectric 1.5))"
                   " (g:make-moving-sphere (v:vec3 1 0 -1) (v:vec3 1 0.5 -1) 0 1 0.3"
                   "   (m:make-lambertian (t:constant-texture (v:vec3 0 0 1)))))",
        "cornell_boxes": "(list (g:translate (g:rotate-y (g:make-box (v:vec3 0 0 0) (v:vec3 165 165 165)"
                         " (m:make-lambertian (t:constant-texture (v:vec3 0.73 0.73 0.73)))) -18) (v:vec3 130 0 65))"
                         " (g:translate (g:rotate-y (g:make-box (v:vec3 0 0 0) (v:vec3 165 330 165)"
                         " (m:make-lambertian (t:constant-texture (v:vec3 0.73 0.73 0.73)))) 15) (v:vec3 265 0 295))"
                         " (g:flip-normals (g:make-xz-rect 213 343 227 332 554"
                         " (m:make-diffuse-light (t:constant-texture (v:vec3 3 3 3))))))",
        "bezier": "(list (b:make-bezier (v:vec3 -1 0 -1) (v:vec3 -0.8 1 1) (v:vec3 0.8 -1 1) (v:vec3 1 0 -1)"
                  " 0.1 (m:make-lambertian (t:constant-texture (v:vec3 0.65 0.05 0.05))))"
                  " (b:make-bezier (v:vec3 130 0 65) (v:vec3 150 0 190) (v:vec3 130 0 190) (v:vec3 265 0 295)"
                  " 10 (m:make-lambertian (t:constant-texture (v:vec3 0.73 0.73 0.73)))))",
    }
    rays = {
        "spheres": [((0, 0, 0), (0, 0, -1), 0.0), ((0, 0, 0), (-1, 0.1, -1), 0.0), ((0, 0, 0), (0.9, 0.05, -1), 0.7),
                    ((0, 0, 0), (0.9, 0.05, -1), 0.0), ((0, 1, 0), (0, -1, 0.001), 0.0), ((-1, 0, -1), (0, 0, 1), 0.0)],
        "cornell_boxes": [((200, 80, -500), (0, 0, 1), 0.0), ((278, 278, -800), (0.05, 0.3, 1), 0.0),
                          ((300, 100, 400), (0.1, -0.2, -1), 0.0), ((278, 500, 278), (0.01, 1, 0.02), 0.0)],
        "bezier": _bezier_rays(),
    }
    hobj = it.modules["geometry"].lookup(ms.sym("hit-obj-list"))
    for name, src in setup.items():
        objs = ref.ev(src)
        res = []
        for o, d, tm in rays[name]:
            ray = [vec3(o), vec3(d), tm]
            h = hobj(objs, ray, 0.001, 999999999999)
            if h[0] is False:
                res.append([H(o), H(d), H(tm), None])
            else:
                rec = h[1]
                res.append([H(o), H(d), H(tm), [H(rec[0]), H(rec[1]), H(rec[2])]])
        hits[name] = res
    out["hits"] = hits
    # points.scm: polyline -> Catmull-Rom Bezier control points
    pts_mod = it.modules["points"]
    poly = [(0.0, 0.0, 0.0), (1.0, 2.0, 0.5), (2.5, 1.0, -1.0), (4.0, 3.0, 0.25), (3.0, 5.5, 2.0), (1.5, 4.0, 3.0)]
    res = call(pts_mod, "points->bezier", [vec3(q) for q in poly])
    out["points_to_bezier"] = {"points": H(poly), "beziers": [[H(list(c)) for c in ms.to_list(b)]
                                                              for b in ms.to_list(res)]}
    return out


SCENE_EXPR = {
    # scenes built by the reference's own definitions (re-evaluated after R2/R3)
    "test_scene": ("define", "test-scene"),
    "test_scene2": ("define", "test-scene2"),
    "cornell": ("define", "cornell-box"),
    "cover": ("call", "(random-scene)"),
    # the reference's default *scene* (main.scm:437): 100 line-upped spheres
    # (random albedos, main.scm:177-194) under its own SAH BVH (geometry.scm:294-371)
    "bvh_sah": ("defines", ["*spheres-list*", "*bvh-sah-node*", "test-scene-bvh-sah"]),
    # cubic Bezier curves (bezier.scm): three curves in a make-bvh-node, and the
    # Cornell frame with one wide curve
    "test_bezier": ("define", "test-bezier"),
    "cornell_bezier": ("define", "cornell-bezier"),
    # participating media: make-constant-medium draws inside its hit test
    "cornell_smoke": ("define", "cornell-smoke"),
    # Kleinian limit set, sphere traced (geometry.scm:590-673)
    "klein": ("define", "klein-scene"),
    "cornell_klein": ("define", "cornell-klein"),
}

SIZES = {"test_scene": (24, 16, 3), "test_scene2": (24, 16, 3), "cornell": (16, 16, 6), "cover": (24, 12, 2),
         "bvh_sah": (24, 12, 2), "test_bezier": (32, 18, 2), "cornell_bezier": (16, 16, 4),
         "cornell_smoke": (16, 16, 4), "klein": (24, 16, 2), "cornell_klein": (16, 16, 2)}


def render(ref, name):
    nx, ny, spp = SIZES[name]
    ref.set_size(nx, ny)
    kind, what = SCENE_EXPR[name]
    if kind == "defines":
        ref.it.random_real = rng.HostStream(SCENE_SEED)
        for nme in what:
            ref.it.eval(ref.define_form(ms.sym(nme)), ref.main)
        scene = ref.main.own[ms.sym(what[-1])]
    elif kind == "define":
        ref.it.random_real = rng.HostStream(SCENE_SEED)
        ref.it.eval(ref.define_form(ms.sym(what)), ref.main)
        scene = ref.main.own[ms.sym(what)]
    else:
        ref.it.random_real = rng.HostStream(SCENE_SEED)          # random-scene's draws (main.scm:45-70)
        scene = ref.ev(what)
    body = ref.pixel_body()
    samples = []
    raw = [[0.0, 0.0, 0.0] for _ in range(nx * ny)]
    t0 = time.time()
    for s in range(spp):
        for y in range(ny):
            for x in range(nx):
                j = y * nx + x
                state = {"d": 0}

                def rr(j=j, s=s, st=state):
                    d = st["d"]
                    st["d"] += 1
                    return rng.path_draw(PATH_SEED, j, s, d)
                ref.it.random_real = rr
                col = body(x, y, scene)
                samples.append([j, s, H(list(col)), state["d"]])
                raw[j] = [raw[j][k] + col[k] for k in range(3)]   # (v:sum raw col) main.scm:480
    img = []
    for j in range(nx * ny):
        for k in range(3):
            c = ms.ssqrt(ms.div(raw[j][k], spp))                 # correct-gamma of v:quot (main.scm:481-484)
            img.append(ms.floor_exact(ms.mul(255.99, ms.smin(1, c))))   # main.scm:485-487
    return {"scene": name, "nx": nx, "ny": ny, "spp": spp, "path_seed": PATH_SEED, "scene_seed": SCENE_SEED,
            "perlin_seed": PERLIN_SEED, "samples": samples, "accum": [H(v) for v in raw], "image": img,
            "seconds": round(time.time() - t0, 1)}


def main():
    ref = Ref()
    k = kat(ref)
    with open(os.path.join(HERE, "ref_kat.json"), "w") as f:
        json.dump(k, f)
    print("wrote ref_kat.json")
    for name in sys.argv[1:] or list(SIZES):
        r = render(ref, name)
        with open(os.path.join(HERE, "ref_%s.json" % name), "w") as f:
            json.dump(r, f)
        print("wrote ref_%s.json (%d samples, %.1fs)" % (name, len(r["samples"]), r["seconds"]))


if __name__ == "__main__":
    sys.setrecursionlimit(1000000)
    threading.stack_size(1 << 29)
    th = threading.Thread(target=main)
    th.start()
    th.join()
