"""Scene descriptors: the reference's constructors, kept name-for-name.

The reference builds closure vectors (geometry.scm:14-15, material.scm:15-22,
texture.scm:9-10).  Here each constructor returns a small immutable
descriptor; ``emit`` walks the descriptor graph once (shared objects are
emitted once, children before parents) and replays it into a *builder*:
``GpuBuilder`` (librtamd's C ABI) or, in tests, the oracle's builder.
"""
import math

from . import vec as v

# ----------------------------------------------------------------- textures


class Texture:
    __slots__ = ("kind", "args")

    def __init__(self, kind, *args):
        self.kind = kind
        self.args = args

    def __repr__(self):
        return "#<texture %s>" % self.kind


def constant_texture(color):
    """t:constant-texture (texture.scm:12-14)."""
    return Texture("constant", v.vec3(*color))


def checker_texture(even_tex, odd_tex):
    """t:checker-texture (texture.scm:16-23)."""
    _need(even_tex, Texture, "checker-texture even")
    _need(odd_tex, Texture, "checker-texture odd")
    return Texture("checker", even_tex, odd_tex)


def noise_texture(sc):
    """t:noise-texture (texture.scm:25-28)."""
    return Texture("noise", float(sc))


def marble_texture(sc):
    """t:marble-texture (texture.scm:30-34)."""
    return Texture("marble", float(sc))


# ---------------------------------------------------------------- materials


class Material:
    __slots__ = ("kind", "args")

    def __init__(self, kind, *args):
        self.kind = kind
        self.args = args

    def __repr__(self):
        return "#<material %s>" % self.kind


def make_lambertian(albedo):
    """m:make-lambertian (material.scm:24-39)."""
    _need(albedo, Texture, "make-lambertian albedo")
    return Material("lambertian", albedo)


def make_metal(albedo, fuzz):
    """m:make-metal (material.scm:45-57)."""
    _need(albedo, Texture, "make-metal albedo")
    return Material("metal", albedo, float(fuzz))


def make_dielectric(ref_idx):
    """m:make-dielectric (material.scm:76-101)."""
    return Material("dielectric", float(ref_idx))


def make_diffuse_light(emit):
    """m:make-diffuse-light (material.scm:103-111)."""
    _need(emit, Texture, "make-diffuse-light emit")
    return Material("diffuse_light", emit)


# ---------------------------------------------------------------- hitables


class Hitable:
    __slots__ = ("kind", "args")

    def __init__(self, kind, *args):
        self.kind = kind
        self.args = args

    def __repr__(self):
        return "#<hitable %s>" % self.kind


def make_sphere(center, radius, material):
    """g:make-sphere (geometry.scm:146-175)."""
    _need(material, Material, "make-sphere material")
    return Hitable("sphere", v.vec3(*center), float(radius), material)


def make_moving_sphere(center0, center1, time0, time1, radius, material):
    """g:make-moving-sphere (geometry.scm:177-215)."""
    _need(material, Material, "make-moving-sphere material")
    return Hitable("moving_sphere", v.vec3(*center0), v.vec3(*center1), float(time0), float(time1),
                   float(radius), material)


def make_xy_rect(x0, x1, y0, y1, k, material):
    """g:make-xy-rect (geometry.scm:376-393)."""
    _need(material, Material, "make-xy-rect material")
    return Hitable("rect", 0, float(x0), float(x1), float(y0), float(y1), float(k), material)


def make_xz_rect(x0, x1, z0, z1, k, material):
    """g:make-xz-rect (geometry.scm:395-412)."""
    _need(material, Material, "make-xz-rect material")
    return Hitable("rect", 1, float(x0), float(x1), float(z0), float(z1), float(k), material)


def make_yz_rect(y0, y1, z0, z1, k, material):
    """g:make-yz-rect (geometry.scm:414-431)."""
    _need(material, Material, "make-yz-rect material")
    return Hitable("rect", 2, float(y0), float(y1), float(z0), float(z1), float(k), material)


def make_bezier(a, b, c, d, width, material):
    """b:make-bezier (bezier.scm:61-223): cubic Bezier curve a..d of the given
    width.  Its hit t is a distance along unit(dir) used as a parameter of the
    raw ray (Q10) and its normal is -dir (Q12); see DESIGN.md."""
    _need(material, Material, "make-bezier material")
    w = float(width)
    if not (w > 0.0 and w != float("inf")):
        # the reference has no check, but for width <= 0 converge's depth estimate takes the log of a
        # number <= 0 (bezier.scm:179-192) and ceiling->exact raises on the first ray that tests the curve
        raise ValueError("make-bezier: width must be positive and finite")
    return Hitable("bezier", v.vec3(*a), v.vec3(*b), v.vec3(*c), v.vec3(*d), float(width), material)


def bezier_array(cps, width, material):
    """bezier->objs (points.scm:45-53) in bulk: ``cps`` is an (n, 12) float64
    array of control points (a, b, c, d per row), one curve per row, all of
    one width and material.  Behaves as the list of those curves."""
    import numpy as np
    _need(material, Material, "bezier->objs material")
    w = float(width)
    if not (w > 0.0 and w != float("inf")):
        raise ValueError("bezier->objs: width must be positive and finite")
    arr = np.ascontiguousarray(cps, dtype=np.float64)
    if arr.ndim != 2 or arr.shape[1] != 12:
        raise ValueError("bezier->objs: control points must have shape (n, 12)")
    return Hitable("curves", arr, float(width), material)


def make_klein(center, material):
    """g:make-klein (geometry.scm:645-673): a Kleinian limit set (six
    inversion spheres, geometry.scm:596-605) rendered by sphere tracing with
    the raw ray direction.  It has no bounding box, so it is never put in a
    BVH."""
    _need(material, Material, "make-klein material")
    return Hitable("klein", v.vec3(*center), material)


def make_constant_medium(obj, density, a):
    """g:make-constant-medium (geometry.scm:545-578): a participating medium
    of the given density inside ``obj`` whose phase function is
    (m:make-lambertian a).  Its hit test draws a random number."""
    _need(obj, Hitable, "make-constant-medium boundary")
    _need(a, Texture, "make-constant-medium albedo")
    if not float(density) > 0.0:
        raise ValueError("make-constant-medium: density must be positive")
    return Hitable("medium", obj, float(density), a)


def flip_normals(obj):
    """g:flip-normals (geometry.scm:433-442)."""
    _need(obj, Hitable, "flip-normals")
    return Hitable("flip", obj)


def make_box(p0, p1, material):
    """g:make-box (geometry.scm:444-463): six rects, back faces flipped."""
    _need(material, Material, "make-box material")
    return Hitable("box", v.vec3(*p0), v.vec3(*p1), material)


def translate(obj, offset):
    """g:translate (geometry.scm:465-481)."""
    _need(obj, Hitable, "translate")
    return Hitable("translate", obj, v.vec3(*offset))


def rotate_y(obj, angle):
    """g:rotate-y (geometry.scm:483-543); angle in degrees."""
    _need(obj, Hitable, "rotate-y")
    return Hitable("rotate_y", obj, float(angle))


def make_bvh_node(obj_list, time0, time1):
    """g:make-bvh-node (geometry.scm:226-260): closest hit over obj_list."""
    objs = list(obj_list)
    for o in objs:
        _need(o, Hitable, "make-bvh-node element")
    return Hitable("bvh", tuple(objs), float(time0), float(time1), 0)


def make_bvh_with_sah(obj_list, time0, time1):
    """g:make-bvh-with-sah (geometry.scm:294-371): closest hit over obj_list."""
    objs = list(obj_list)
    for o in objs:
        _need(o, Hitable, "make-bvh-with-sah element")
    return Hitable("bvh", tuple(objs), float(time0), float(time1), 1)


# ----------------------------------------------------------- sky functions
class SkyFunction:
    __slots__ = ("name", "code")

    def __init__(self, name, code):
        self.name = name
        self.code = code

    def __repr__(self):
        return "#<sky %s>" % self.name


#: sky-color (main.scm:91-95): white-to-blue gradient on unit(dir).y
sky_color = SkyFunction("sky-color", 0)
#: black (main.scm:97-98)
black = SkyFunction("black", 1)


# -------------------------------------------------------------------- scene
class Scene:
    """g:make-scene (geometry.scm:52-56): obj-list, camera, sky function.

    ``perlin`` holds the Perlin tables the scene's noise/marble textures read
    (the reference's module-level +ranvec+/+perm-*+, perlin.scm:32-36).
    """

    def __init__(self, obj_list, camera, sky_function, perlin=None, light=None):
        self.obj_list = tuple(obj_list)
        for o in self.obj_list:
            _need(o, Hitable, "make-scene obj-list element")
        self.camera = camera
        self.sky_function = sky_function
        self.perlin = perlin
        # extension (pdf.scm): lambertian bounces sample the
        # mixture of (hitable-pdf light p) and (cosine-pdf normal)
        if light is not None:
            _need(light, Hitable, "light-sampling target")
            if light.kind == "flip":
                inner = light.args[0]
            else:
                inner = light
            if inner.kind not in ("rect", "sphere"):
                raise ValueError("light sampling needs a rect or a sphere (optionally flipped)")
        self.light = light
        self._handles = {}

    def uses_perlin(self):
        seen = set()
        stack = list(self.obj_list)
        while stack:
            o = stack.pop()
            if id(o) in seen:
                continue
            seen.add(id(o))
            for a in o.args:
                if isinstance(a, (Hitable, Material, Texture)):
                    stack.append(a)
                elif isinstance(a, tuple) and a and isinstance(a[0], Hitable):
                    stack.extend(a)
            if isinstance(o, Texture) and o.kind in ("noise", "marble"):
                return True
        return False


def make_scene(obj_list, camera, sky_function, perlin=None, light=None):
    """g:make-scene (geometry.scm:52).  ``light`` (extension, pdf.scm): an
    object of obj_list (a rect or sphere, possibly flipped) that lambertian
    bounces sample through the light/cosine mixture pdf."""
    if not isinstance(sky_function, SkyFunction):
        raise TypeError("make-scene: sky function must be sky_color or black (got %r)" % (sky_function,))
    return Scene(obj_list, camera, sky_function, perlin, light)


def _need(x, cls, what):
    if not isinstance(x, cls):
        raise TypeError("%s: expected %s, got %r" % (what, cls.__name__.lower(), x))


# ------------------------------------------------------------------- emit
def emit(scene, b):
    """Replay the scene's descriptor graph into builder ``b`` and commit it.

    ``b`` provides texture_*/material_*/sphere/moving_sphere/rect/
    flip_normals/box/translate/rotate_y/list/bvh/set_camera/set_sky/
    set_perlin/commit (see GpuBuilder).  Returns b.commit(world)'s value.
    """
    memo = {}

    def tex(t):
        k = id(t)
        if k not in memo:
            if t.kind == "constant":
                memo[k] = b.texture_constant(t.args[0])
            elif t.kind == "checker":
                even, odd = tex(t.args[0]), tex(t.args[1])
                memo[k] = b.texture_checker(even, odd)
            elif t.kind == "noise":
                memo[k] = b.texture_noise(t.args[0])
            elif t.kind == "marble":
                memo[k] = b.texture_marble(t.args[0])
            else:
                raise ValueError(t.kind)
        return memo[k]

    def mat(m):
        k = id(m)
        if k not in memo:
            if m.kind == "lambertian":
                memo[k] = b.material_lambertian(tex(m.args[0]))
            elif m.kind == "metal":
                memo[k] = b.material_metal(tex(m.args[0]), m.args[1])
            elif m.kind == "dielectric":
                memo[k] = b.material_dielectric(m.args[0])
            elif m.kind == "diffuse_light":
                memo[k] = b.material_diffuse_light(tex(m.args[0]))
            else:
                raise ValueError(m.kind)
        return memo[k]

    def obj(o):
        k = id(o)
        if k in memo:
            return memo[k]
        a = o.args
        if o.kind == "sphere":
            r = b.sphere(a[0], a[1], mat(a[2]))
        elif o.kind == "moving_sphere":
            r = b.moving_sphere(a[0], a[1], a[2], a[3], a[4], mat(a[5]))
        elif o.kind == "rect":
            r = b.rect(a[0], a[1], a[2], a[3], a[4], a[5], mat(a[6]))
        elif o.kind == "bezier":
            r = b.bezier(a[0], a[1], a[2], a[3], a[4], mat(a[5]))
        elif o.kind == "curves":
            first = b.bezier_array(a[0], a[1], mat(a[2]))
            r = b.list(list(range(first, first + a[0].shape[0])))
        elif o.kind == "klein":
            r = b.klein(a[0], mat(a[1]))
        elif o.kind == "medium":
            r = b.constant_medium(obj(a[0]), a[1], tex(a[2]))
        elif o.kind == "flip":
            r = b.flip_normals(obj(a[0]))
        elif o.kind == "box":
            r = b.box(a[0], a[1], mat(a[2]))
        elif o.kind == "translate":
            r = b.translate(obj(a[0]), a[1])
        elif o.kind == "rotate_y":
            r = b.rotate_y(obj(a[0]), a[1])
        elif o.kind == "bvh":
            r = b.bvh([obj(c) for c in a[0]], a[1], a[2], a[3])
        else:
            raise ValueError(o.kind)
        memo[k] = r
        return r

    ids = [obj(o) for o in scene.obj_list]
    world = b.list(ids)
    if getattr(scene, "light", None) is not None:
        b.set_light(obj(scene.light))
    b.set_camera(scene.camera.slots())
    b.set_sky(scene.sky_function.code)
    if scene.uses_perlin():
        if scene.perlin is None:
            raise ValueError("scene uses noise/marble textures but has no Perlin tables (scene.perlin)")
        p = scene.perlin
        b.set_perlin(p.ranvec, p.perm_x, p.perm_y, p.perm_z)
    return b.commit(world)


def deg_to_rad(angle):
    """(* pi/180 angle) — geometry.scm:484."""
    return (math.pi / 180.0) * angle
