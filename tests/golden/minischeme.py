"""A small evaluator for the Gauche Scheme subset the reference is written in.

BUILDER TOOLING for fixture generation only (tests/golden/make_golden.py):
it executes the reference's own .scm files from /root/reference in THIS
container so the committed golden vectors come from the reference's source
text rather than from our restatement.  Nothing here is imported by the
product, by the GPU tests or by bench.py, and the reference never travels.

Scope: the forms and procedures the reference uses (define / define-inline /
lambda / let family / named let / let-values / receive / cond / dotimes /
push! pop! inc! dec! / define-syntax + syntax-rules (non-hygienic, enough for
onb.scm `local` and geometry.scm `surrounding-box`) / modules with `:prefix`
imports), numbers with Scheme's exact/inexact semantics (int, Fraction,
float, complex), f64vectors, pairs and vectors.  Module lookup: a module's
own bindings first, then its imports, the most recent `use` first.  GL,
threads and the profiler are stubbed; define-class and define-macro forms
are skipped (the reference's only uses are dead code: camera.scm:11-31,
main.scm:610-614).  Arguments and `let` inits are evaluated left to right.
"""
import cmath
import math
import os
from fractions import Fraction


# ------------------------------------------------------------------ data
class Sym(str):
    pass


_symtab = {}


def sym(name):
    s = _symtab.get(name)
    if s is None:
        s = _symtab[name] = Sym(name)
    return s


class Pair:
    __slots__ = ("car", "cdr")

    def __init__(self, a, d):
        self.car = a
        self.cdr = d


class Nil:
    __slots__ = ()

    def __repr__(self):
        return "()"


NIL = Nil()


class Undefined:
    def __repr__(self):
        return "#<undef>"


UNDEF = Undefined()


class Values(tuple):
    pass


class Keyword(str):
    pass


class F64Vec(list):
    """f64vector: a list of Python floats."""


class SchemeError(Exception):
    pass


def from_list(xs, tail=NIL):
    r = tail
    for x in reversed(xs):
        r = Pair(x, r)
    return r


def to_list(p):
    out = []
    while isinstance(p, Pair):
        out.append(p.car)
        p = p.cdr
    return out


def truthy(x):
    return x is not False


# ---------------------------------------------------------------- reader
def tokenize(src):
    toks = []
    i, n = 0, len(src)
    while i < n:
        c = src[i]
        if c in " \t\r\n\f":
            i += 1
        elif c == ";":
            while i < n and src[i] != "\n":
                i += 1
        elif c in "()[]":
            toks.append("(" if c in "([" else ")")
            i += 1
        elif c == "'":
            toks.append("'")
            i += 1
        elif c == "`":
            toks.append("`")
            i += 1
        elif c == ",":
            if i + 1 < n and src[i + 1] == "@":
                toks.append(",@")
                i += 2
            else:
                toks.append(",")
                i += 1
        elif c == '"':
            j = i + 1
            buf = []
            while src[j] != '"':
                if src[j] == "\\":
                    j += 1
                    buf.append({"n": "\n", "t": "\t"}.get(src[j], src[j]))
                else:
                    buf.append(src[j])
                j += 1
            toks.append(("str", "".join(buf)))
            i = j + 1
        elif c == "#" and i + 1 < n and src[i + 1] == "(":
            toks.append("#(")
            i += 2
        elif c == "#" and src.startswith("#f32(", i):
            toks.append("#f32(")
            i += 5
        elif c == "#" and i + 1 < n and src[i + 1] == "\\":
            j = i + 3
            while j < n and src[j] not in " \t\r\n()[]":
                j += 1
            toks.append(("char", src[i + 2:j]))
            i = j
        else:
            j = i
            while j < n and src[j] not in " \t\r\n()[]\";":
                j += 1
            toks.append(("atom", src[i:j]))
            i = j
    return toks


def parse_atom(t):
    if t == "#t":
        return True
    if t == "#f":
        return False
    if t in ("+inf.0",):
        return math.inf
    if t == "-inf.0":
        return -math.inf
    if t == "+nan.0":
        return math.nan
    try:
        return int(t)
    except ValueError:
        pass
    try:
        if "/" in t:
            return Fraction(t)
        return float(t)
    except ValueError:
        pass
    if t.startswith(":"):
        return Keyword(t)
    return sym(t)


def read_all(src):
    toks = tokenize(src)
    pos = [0]

    def read():
        t = toks[pos[0]]
        pos[0] += 1
        if t == "(":
            items = []
            dotted = None
            while toks[pos[0]] != ")":
                if toks[pos[0]] == ("atom", "."):
                    pos[0] += 1
                    dotted = read()
                    continue
                items.append(read())
            pos[0] += 1
            return from_list(items, dotted if dotted is not None else NIL)
        if t in ("#(", "#f32("):
            items = []
            while toks[pos[0]] != ")":
                items.append(read())
            pos[0] += 1
            return F64Vec(float(x) for x in items) if t == "#f32(" else list(items)
        if t == "'":
            return from_list([sym("quote"), read()])
        if t == "`":
            return from_list([sym("quasiquote"), read()])
        if t == ",":
            return from_list([sym("unquote"), read()])
        if t == ",@":
            return from_list([sym("unquote-splicing"), read()])
        if t == ")":
            raise SchemeError("unexpected )")
        kind, val = t
        if kind == "str":
            return val
        if kind == "char":
            return ("char", val)
        return parse_atom(val)

    out = []
    while pos[0] < len(toks):
        out.append(read())
    return out


# ------------------------------------------------------------ environments
class Env:
    __slots__ = ("vars", "parent")

    def __init__(self, vars, parent):
        self.vars = vars
        self.parent = parent


class Module:
    def __init__(self, name, interp):
        self.name = name
        self.own = {}
        self.imports = []          # (module, prefix, only) most recent first
        self.interp = interp

    def lookup(self, s):
        if s in self.own:
            return self.own[s]
        for mod, prefix, only in self.imports:
            if prefix:
                if not s.startswith(prefix):
                    continue
                base = sym(s[len(prefix):])
            else:
                base = s
            if only is not None and base not in only:
                continue
            v = mod.lookup_export(base)
            if v is not _MISSING:
                return v
        v = self.interp.core.get(s, _MISSING)
        if v is _MISSING:
            raise SchemeError("unbound variable %s in module %s" % (s, self.name))
        return v

    def lookup_export(self, s):
        if s in self.own:
            return self.own[s]
        return _MISSING

    def has(self, s):
        try:
            self.lookup(s)
            return True
        except SchemeError:
            return False


_MISSING = object()


class Procedure:
    __slots__ = ("params", "rest", "body", "env", "module", "name")

    def __init__(self, params, rest, body, env, module, name="lambda"):
        self.params = params
        self.rest = rest
        self.body = body
        self.env = env
        self.module = module
        self.name = name

    def __call__(self, *args):
        n = len(self.params)
        if len(args) < n or (self.rest is None and len(args) != n):
            raise SchemeError("arity mismatch calling %s: %d args" % (self.name, len(args)))
        d = dict(zip(self.params, args))
        if self.rest is not None:
            d[self.rest] = from_list(list(args[n:]))
        env = Env(d, self.env)
        r = UNDEF
        try:
            for f in self.body:
                r = f(env)
        except SchemeError as e:
            if len(e.args) < 2:
                e.args = (e.args[0], [])
            if len(e.args[1]) < 12:
                e.args[1].append("%s:%s" % (self.module.name, self.name))
            raise
        return r


class Macro:
    def __init__(self, rules, literals):
        self.rules = rules
        self.literals = literals


# ------------------------------------------------------------ syntax-rules
def _match(pat, form, lits, b):
    if isinstance(pat, Sym):
        if pat == "_":
            return True
        if pat in lits:
            return form == pat
        b[pat] = form
        return True
    if isinstance(pat, Pair):
        if isinstance(pat.cdr, Pair) and pat.cdr.car == "...":
            items = to_list(form)
            rest_pats = to_list(pat.cdr.cdr)
            need = len(rest_pats)
            if len(items) < need:
                return False
            reps = items[:len(items) - need]
            subs = []
            for it in reps:
                bb = {}
                if not _match(pat.car, it, lits, bb):
                    return False
                subs.append(bb)
            b[("...", id(pat))] = (pat.car, subs)
            for name in _pat_vars(pat.car, lits):
                b[name] = [s[name] for s in subs]
                b.setdefault("__ellipsis__", set()).add(name)
            tail = from_list(items[len(items) - need:])
            return _match(pat.cdr.cdr, tail, lits, b)
        if not isinstance(form, Pair):
            return False
        return _match(pat.car, form.car, lits, b) and _match(pat.cdr, form.cdr, lits, b)
    if pat is NIL:
        return form is NIL
    return pat == form


def _pat_vars(p, lits):
    if isinstance(p, Sym):
        return [] if (p in lits or p in ("_", "...")) else [p]
    if isinstance(p, Pair):
        return _pat_vars(p.car, lits) + _pat_vars(p.cdr, lits)
    return []


def _expand(t, b):
    if isinstance(t, Sym):
        return b.get(t, t) if t not in b.get("__ellipsis__", ()) else b[t]
    if isinstance(t, Pair):
        if isinstance(t.cdr, Pair) and t.cdr.car == "...":
            names = [n for n in _pat_vars(t.car, ()) if n in b.get("__ellipsis__", ())]
            count = len(b[names[0]]) if names else 0
            out = []
            for k in range(count):
                bb = dict(b)
                for nme in names:
                    bb[nme] = b[nme][k]
                bb["__ellipsis__"] = b["__ellipsis__"] - set(names)
                out.append(_expand(t.car, bb))
            return from_list(out, _expand(t.cdr.cdr, b))
        return Pair(_expand(t.car, b), _expand(t.cdr, b))
    return t


# ---------------------------------------------------------------- numbers
def _is_num(x):
    return isinstance(x, (int, float, Fraction, complex)) and not isinstance(x, bool)


def _norm(x):
    if isinstance(x, Fraction) and x.denominator == 1:
        return int(x.numerator)
    return x


def _inexact(x):
    return isinstance(x, (float, complex))


def add(*a):
    r = 0
    for x in a:
        r = r + x
    return _norm(r)


def sub(a, *b):
    if not b:
        return _norm(-a)
    for x in b:
        a = a - x
    return _norm(a)


def mul(*a):
    r = 1
    for x in a:
        r = r * x
    return _norm(r)


def _div2(a, b):
    if not _inexact(a) and not _inexact(b):
        if b == 0:
            raise SchemeError("division by exact zero")
        return _norm(Fraction(a) / Fraction(b))
    a, b = (complex(a), complex(b)) if isinstance(a, complex) or isinstance(b, complex) else (float(a), float(b))
    if b == 0:
        if isinstance(a, complex):
            raise SchemeError("complex division by zero")
        if a == 0 or math.isnan(a):
            return math.nan
        return math.copysign(math.inf, a) * math.copysign(1.0, b)
    return a / b


def div(a, *b):
    if not b:
        return _div2(1, a)
    for x in b:
        a = _div2(a, x)
    return a


def _cmp(op):
    def f(*a):
        for x, y in zip(a, a[1:]):
            if not op(x, y):
                return False
        return True
    return f


def smin(*a):
    r = min(a)
    return float(r) if any(_inexact(x) for x in a) else r


def smax(*a):
    r = max(a)
    return float(r) if any(_inexact(x) for x in a) else r


def ssqrt(x):
    if isinstance(x, complex):
        return cmath.sqrt(x)
    if not _inexact(x):
        if x >= 0:
            f = Fraction(x)
            n, d = math.isqrt(f.numerator), math.isqrt(f.denominator)
            if n * n == f.numerator and d * d == f.denominator:
                return _norm(Fraction(n, d))
            return math.sqrt(float(x))
        return cmath.sqrt(complex(x))
    if x < 0:
        return cmath.sqrt(complex(x))
    return math.sqrt(x)


def sasin(x):
    if isinstance(x, complex) or abs(x) > 1:
        return cmath.asin(complex(x))
    return math.asin(x)


def satan(y, x=None):
    if x is None:
        return math.atan(y)
    return math.atan2(float(y), float(x))


def slog(x, base=None):
    def ln(v):
        if isinstance(v, complex) or v < 0:
            return cmath.log(complex(v))
        if v == 0:
            if _inexact(v):
                return -math.inf
            raise SchemeError("log of exact 0")
        return math.log(v)
    return ln(x) if base is None else div(ln(x), ln(base))


def sexpt(a, b):
    if isinstance(b, int) and not _inexact(a):
        return _norm(Fraction(a) ** b) if b < 0 else a ** b
    return float(a) ** b if not isinstance(a, complex) else a ** b


def floor_exact(x):
    return math.floor(x)


def ceiling_exact(x):
    return math.ceil(x)


def clamp(x, lo=None, hi=None):
    r = x
    if lo is not None and r < lo:
        r = lo
    if hi is not None and r > hi:
        r = hi
    if any(_inexact(v) for v in (x, lo, hi) if v is not None):
        r = float(r)
    return r


def _logand(*a):
    r = -1
    for x in a:
        r &= x
    return r


def _logxor(*a):
    r = 0
    for x in a:
        r ^= x
    return r


def _logior(*a):
    r = 0
    for x in a:
        r |= x
    return r


# -------------------------------------------------------------- f64vector
def _vec_op(op):
    def f(a, b):
        if isinstance(b, list):
            return F64Vec(op(x, y) for x, y in zip(a, b))
        bf = float(b)
        return F64Vec(op(x, bf) for x in a)
    return f


def f64_div(x, y):
    return _div2(x, y)


def f64vector_dot(a, b):
    r = 0.0
    for x, y in zip(a, b):
        r += x * y
    return r


# ------------------------------------------------------------------ lists
def s_length(x):
    if isinstance(x, (list, str)):
        return len(x)
    n = 0
    while isinstance(x, Pair):
        n += 1
        x = x.cdr
    return n


def s_ref(obj, i):
    if isinstance(obj, list):
        return obj[i]
    for _ in range(i):
        obj = obj.cdr
    return obj.car


def s_subseq(obj, start, end=None):
    if isinstance(obj, list):
        return obj[start:end]
    items = to_list(obj)
    return from_list(items[start:end])


def s_sort(seq, less=None):
    items = list(seq) if isinstance(seq, list) else to_list(seq)
    if less is None:
        def less(a, b):
            return a < b

    def msort(xs):           # stable merge sort; `less` may be any truthy-returning procedure
        if len(xs) <= 1:
            return xs
        mid = len(xs) // 2
        a, b = msort(xs[:mid]), msort(xs[mid:])
        out = []
        i = j = 0
        while i < len(a) and j < len(b):
            if truthy(less(b[j], a[i])):
                out.append(b[j])
                j += 1
            else:
                out.append(a[i])
                i += 1
        return out + a[i:] + b[j:]
    r = msort(items)
    return r if isinstance(seq, list) else from_list(r)


def reduce_(f, ridentity, lst):
    items = to_list(lst)
    if not items:
        return ridentity
    acc = items[0]
    for x in items[1:]:
        acc = f(x, acc)
    return acc


def reduce_right(f, ridentity, lst):
    items = to_list(lst)
    if not items:
        return ridentity
    acc = items[-1]
    for x in reversed(items[:-1]):
        acc = f(x, acc)
    return acc


def s_append(*ls):
    if not ls:
        return NIL
    items = []
    for l in ls[:-1]:
        items.extend(to_list(l))
    return from_list(items, ls[-1])


def s_apply(f, *args):
    args = list(args[:-1]) + to_list(args[-1])
    return f(*args)


def s_map(f, *ls):
    cols = [to_list(l) if not isinstance(l, list) else l for l in ls]
    out = [f(*xs) for xs in zip(*cols)]
    return out if isinstance(ls[0], list) else from_list(out)


def s_for_each(f, *ls):
    cols = [to_list(l) if not isinstance(l, list) else l for l in ls]
    for xs in zip(*cols):
        f(*xs)
    return UNDEF


def s_last(l):
    return to_list(l)[-1]


def s_drop_right(l, k):
    items = to_list(l)
    return from_list(items[:len(items) - k])


def s_values(*a):
    return a[0] if len(a) == 1 else Values(a)


# ------------------------------------------------------------ gauche.array
class Array:
    def __init__(self, rows, cols, data):
        self.rows, self.cols, self.data = rows, cols, data


def s_shape(*bounds):
    return bounds


def s_array(shape, *vals):
    r0, r1, c0, c1 = shape
    return Array(r1 - r0, c1 - c0, list(vals))


def s_array_ref(a, i, j):
    return a.data[i * a.cols + j]


def s_array_mul(a, b):
    out = []
    for i in range(a.rows):
        for j in range(b.cols):
            s = 0
            for k in range(a.cols):
                s = add(s, mul(a.data[i * a.cols + k], b.data[k * b.cols + j]))
            out.append(s)
    return Array(a.rows, b.cols, out)


# ------------------------------------------------------------ interpreter
class Interp:
    def __init__(self, load_dir):
        self.load_dir = load_dir
        self.modules = {}
        self.random_real = None          # set by the driver
        self.core = self._core()
        self.user = Module("user", self)
        self.modules["user"] = self.user
        for name in ("gauche.uvector", "srfi-27", "math.const", "gauche.record", "srfi-11", "gauche.sequence",
                     "srfi-43", "gauche.array", "gauche.threads", "gauche.time", "gl", "gl.glut", "srfi-13",
                     "gauche.collection", "srfi-1"):
            self.modules[name] = Module(name, self)   # everything they provide lives in `core`

    def _core(self):
        c = {}

        def d(name, f):
            c[sym(name)] = f
        for name, f in {
            "+": add, "-": sub, "*": mul, "/": div,
            "<": _cmp(lambda a, b: a < b), ">": _cmp(lambda a, b: a > b), "<=": _cmp(lambda a, b: a <= b),
            ">=": _cmp(lambda a, b: a >= b), "=": _cmp(lambda a, b: a == b),
            "min": smin, "max": smax, "abs": abs, "sqrt": ssqrt, "expt": sexpt, "exp": math.exp, "log": slog,
            "sin": math.sin, "cos": math.cos, "tan": math.tan, "asin": sasin, "acos": math.acos, "atan": satan,
            "floor": math.floor, "ceiling": math.ceil, "floor->exact": floor_exact,
            "ceiling->exact": ceiling_exact, "exact->inexact": float, "inexact": float,
            "logand": _logand, "logxor": _logxor, "logior": _logior,
            "quotient": lambda a, b: int(a / b), "modulo": lambda a, b: a % b, "clamp": clamp,
            "zero?": lambda x: x == 0, "not": lambda x: x is False, "null?": lambda x: x is NIL,
            "pair?": lambda x: isinstance(x, Pair), "eq?": lambda a, b: a is b or (_is_num(a) and a == b),
            "eqv?": lambda a, b: a is b or a == b, "equal?": lambda a, b: a == b,
            "car": lambda p: p.car, "cdr": lambda p: p.cdr, "cons": Pair, "list": lambda *a: from_list(list(a)),
            "length": s_length, "append": s_append, "append!": s_append, "reverse": lambda l: from_list(to_list(l)[::-1]),
            "reverse!": lambda l: from_list(to_list(l)[::-1]), "list-copy": lambda l: from_list(to_list(l)),
            "last": s_last, "drop-right!": s_drop_right, "map": s_map, "for-each": s_for_each, "apply": s_apply,
            "reduce": reduce_, "reduce-right": reduce_right, "ref": s_ref, "subseq": s_subseq, "sort": s_sort,
            "vector": lambda *a: list(a), "make-vector": lambda n, fill=UNDEF: [fill] * n,
            "vector-ref": lambda v, i: v[i], "vector-length": len, "list->vector": lambda l: to_list(l),
            "vector->list": from_list, "vector-tabulate": lambda n, f: [f(i) for i in range(n)],
            "f64vector": lambda *a: F64Vec(float(x) for x in a), "f64vector-ref": lambda v, i: v[i],
            "f64vector-add": _vec_op(lambda x, y: x + y), "f64vector-sub": _vec_op(lambda x, y: x - y),
            "f64vector-mul": _vec_op(lambda x, y: x * y), "f64vector-div": _vec_op(f64_div),
            "f64vector-dot": f64vector_dot, "make-u8vector": lambda n, fill=0: [fill] * n,
            "u8vector-ref": lambda v, i: v[i], "values": s_values, "display": lambda *a: UNDEF,
            "format": lambda *a: "", "make-thread": lambda *a: UNDEF, "char->integer": lambda c: ord(c[1][0]),
            "dynamic-wind": lambda before, thunk, after: (before(), thunk(), after())[1],
            "array": s_array, "shape": s_shape, "array-ref": s_array_ref, "array-mul": s_array_mul,
            "number?": _is_num, "procedure?": callable, "vector?": lambda x: isinstance(x, list),
            "error": self._error,
        }.items():
            d(name, f)

        def f64vector_set(v, i, x):
            v[i] = float(x)
            return UNDEF

        def vector_set(v, i, x):
            v[i] = x
            return UNDEF

        def vector_swap(v, i, j):
            v[i], v[j] = v[j], v[i]
            return UNDEF
        d("f64vector-set!", f64vector_set)
        d("vector-set!", vector_set)
        d("u8vector-set!", vector_set)
        d("vector-swap!", vector_swap)
        d("random-real", lambda: self.random_real())
        pi = 4 * math.atan(1)
        for name, val in {"pi": pi, "pi/2": pi / 2, "pi/4": pi / 4, "pi/180": pi / 180, "1/pi": 1 / pi,
                          "180/pi": 180 / pi, "e": math.e}.items():
            d(name, val)
        return c

    @staticmethod
    def _error(*a):
        raise SchemeError(" ".join(str(x) for x in a))

    # ---- modules / loading
    def load_module(self, name):
        if name in self.modules:
            return self.modules[name]
        path = os.path.join(self.load_dir, name.replace(".", "/") + ".scm")
        if not os.path.exists(path):
            raise SchemeError("module %s not found" % name)
        mod = Module(name, self)
        self.modules[name] = mod
        self.eval_file(path, mod)
        return mod

    def eval_file(self, path, mod=None):
        mod = mod or self.user
        forms = read_all(open(path).read())
        cur = [mod]
        for f in forms:
            if isinstance(f, Pair) and f.car == "define-module":
                name = str(f.cdr.car)
                m = self.modules.get(name) or Module(name, self)
                self.modules[name] = m
                for clause in to_list(f.cdr.cdr):
                    self._module_clause(m, clause)
                continue
            if isinstance(f, Pair) and f.car == "select-module":
                cur[0] = self.modules[str(f.cdr.car)]
                continue
            self.eval(f, cur[0])
        return cur[0]

    def _module_clause(self, m, clause):
        head = clause.car
        if head == "use":
            parts = to_list(clause.cdr)
            name = str(parts[0])
            prefix = None
            only = None
            for k in range(1, len(parts), 2):
                if parts[k] == ":prefix":
                    prefix = str(parts[k + 1])
            imported = self.load_module(name)
            m.imports.insert(0, (imported, prefix, only))

    def eval(self, form, mod):
        return self.compile(form, mod, ())(None)

    # ---- compiler: form -> f(env)
    def compile(self, x, mod, scope):
        if isinstance(x, Sym):
            return self._compile_ref(x, mod, scope)
        if isinstance(x, Pair):
            head = x.car
            if isinstance(head, Sym) and head not in scope:
                sf = getattr(self, "sf_" + head.replace("-", "_").replace("*", "_star").replace("!", "_bang")
                             .replace("?", "_p").replace(">", "_gt"), None)
                if sf is not None and not (head in mod.own):
                    return sf(x, mod, scope)
                m = self._macro(head, mod)
                if m is not None:
                    return self.compile(self._expand_macro(m, x), mod, scope)
            fc = self.compile(head, mod, scope)
            acs = [self.compile(a, mod, scope) for a in to_list(x.cdr)]
            return _make_call(fc, acs)
        if isinstance(x, tuple) and len(x) == 2 and x[0] == "char":
            return lambda env, v=x: v
        return lambda env, v=x: v

    def _macro(self, head, mod):
        try:
            v = mod.lookup(head)
        except SchemeError:
            return None
        return v if isinstance(v, Macro) else None

    @staticmethod
    def _expand_macro(m, form):
        for pat, tmpl in m.rules:
            b = {}
            if _match(pat.cdr, form.cdr, m.literals, b):
                return _expand(tmpl, b)
        raise SchemeError("no syntax-rules clause matches %r" % form.car)

    def _compile_ref(self, s, mod, scope):
        if s in scope:
            def ref(env, s=s):
                e = env
                while e is not None:
                    v = e.vars
                    if s in v:
                        return v[s]
                    e = e.parent
                return mod.lookup(s)
            return ref
        cache = []

        def gref(env, s=s):
            if cache:
                return cache[0]
            v = mod.lookup(s)
            return v
        return gref

    def _body(self, forms, mod, scope):
        # internal defines become locals of the enclosing frame
        names = []
        for f in forms:
            if isinstance(f, Pair) and f.car in ("define", "define-inline"):
                t = f.cdr.car
                names.append(t.car if isinstance(t, Pair) else t)
        scope = tuple(scope) + tuple(names)
        return [self.compile(f, mod, scope) for f in forms], scope

    def _lambda(self, params, body_forms, mod, scope, name="lambda"):
        ps = []
        rest = None
        p = params
        while isinstance(p, Pair):
            ps.append(p.car)
            p = p.cdr
        if isinstance(p, Sym):
            rest = p
        inner = tuple(scope) + tuple(ps) + ((rest,) if rest else ())
        body, _ = self._body(to_list(body_forms), mod, inner)

        def mk(env):
            return Procedure(ps, rest, body, env, mod, name)
        return mk

    # ---- special forms
    def sf_quote(self, x, mod, scope):
        v = x.cdr.car
        return lambda env: v

    def sf_if(self, x, mod, scope):
        parts = to_list(x.cdr)
        c = self.compile(parts[0], mod, scope)
        t = self.compile(parts[1], mod, scope)
        e = self.compile(parts[2], mod, scope) if len(parts) > 2 else (lambda env: UNDEF)
        return lambda env: t(env) if c(env) is not False else e(env)

    def sf_define(self, x, mod, scope):
        target = x.cdr.car
        if isinstance(target, Pair):
            name = target.car
            f = self._lambda(target.cdr, x.cdr.cdr, mod, scope, str(name))
        else:
            name = target
            rest = to_list(x.cdr.cdr)
            f = self.compile(rest[0], mod, scope) if rest else (lambda env: UNDEF)
        if scope and name in scope:
            def local_def(env):
                env.vars[name] = f(env)
                return UNDEF
            return local_def

        def top_def(env):
            v = f(env)
            if isinstance(v, Procedure) and v.name == "lambda":
                v.name = str(name)
            mod.own[name] = v
            return UNDEF
        return top_def

    sf_define_inline = sf_define
    sf_define_constant = sf_define

    def sf_define_class(self, x, mod, scope):
        return lambda env: UNDEF

    def sf_define_macro(self, x, mod, scope):
        return lambda env: UNDEF

    def sf_add_load_path(self, x, mod, scope):
        return lambda env: UNDEF

    def sf_use(self, x, mod, scope):
        self._module_clause(mod, x)
        return lambda env: UNDEF

    def sf_export(self, x, mod, scope):
        return lambda env: UNDEF

    sf_export_all = sf_export

    def sf_define_syntax(self, x, mod, scope):
        name = x.cdr.car
        spec = x.cdr.cdr.car
        assert spec.car == "syntax-rules"
        lits = set(to_list(spec.cdr.car))
        rules = [(r.car, r.cdr.car) for r in to_list(spec.cdr.cdr)]
        mod.own[name] = Macro(rules, lits)
        return lambda env: UNDEF

    def sf_lambda(self, x, mod, scope):
        return self._lambda(x.cdr.car, x.cdr.cdr, mod, scope)

    def sf_begin(self, x, mod, scope):
        fs = [self.compile(f, mod, scope) for f in to_list(x.cdr)]

        def run(env):
            r = UNDEF
            for f in fs:
                r = f(env)
            return r
        return run

    def sf_set_bang(self, x, mod, scope):
        target = x.cdr.car
        val = self.compile(x.cdr.cdr.car, mod, scope)
        if isinstance(target, Pair):              # generalized set! (vector-ref v i)
            acc = target.car
            setter = {"vector-ref": "vector-set!", "f64vector-ref": "f64vector-set!"}[str(acc)]
            args = [self.compile(a, mod, scope) for a in to_list(target.cdr)]
            sf = self.compile(sym(setter), mod, scope)
            return lambda env: sf(env)(*[a(env) for a in args], val(env))
        return self._setter(target, mod, scope, val)

    def _setter(self, name, mod, scope, val):
        if name in scope:
            def st(env):
                v = val(env)
                e = env
                while e is not None:
                    if name in e.vars:
                        e.vars[name] = v
                        return UNDEF
                    e = e.parent
                raise SchemeError("set! of unbound %s" % name)
            return st

        def gst(env):
            mod.own[name] = val(env)
            return UNDEF
        return gst

    def _let_common(self, bindings, body, mod, scope, sequential):
        names = [b.car for b in bindings]
        inits = []
        sc = tuple(scope)
        for b in bindings:
            init = b.cdr.car if b.cdr is not NIL else False
            inits.append(self.compile(init, mod, sc))
            if sequential:
                sc = sc + (b.car,)
        inner = tuple(scope) + tuple(names)
        fs, _ = self._body(to_list(body), mod, inner)
        if sequential:
            def run(env):
                for nme, f in zip(names, inits):
                    env = Env({nme: f(env)}, env)
                env = Env({}, env)
                r = UNDEF
                for g in fs:
                    r = g(env)
                return r
        else:
            def run(env):
                vals = [f(env) for f in inits]
                e = Env(dict(zip(names, vals)), env)
                r = UNDEF
                for g in fs:
                    r = g(e)
                return r
        return run

    def sf_let(self, x, mod, scope):
        if isinstance(x.cdr.car, Sym):               # named let
            name = x.cdr.car
            bindings = to_list(x.cdr.cdr.car)
            body = x.cdr.cdr.cdr
            params = from_list([b.car for b in bindings])
            inits = [self.compile(b.cdr.car, mod, scope) for b in bindings]
            lam = self._lambda(params, body, mod, tuple(scope) + (name,), str(name))

            def run(env):
                e = Env({}, env)
                proc = lam(e)
                e.vars[name] = proc
                return proc(*[f(env) for f in inits])
            return run
        return self._let_common(to_list(x.cdr.car), x.cdr.cdr, mod, scope, False)

    def sf_let_star(self, x, mod, scope):
        return self._let_common(to_list(x.cdr.car), x.cdr.cdr, mod, scope, True)

    def sf_let1(self, x, mod, scope):
        b = from_list([from_list([x.cdr.car, x.cdr.cdr.car])])
        return self._let_common(to_list(b), x.cdr.cdr.cdr, mod, scope, False)

    def sf_letrec(self, x, mod, scope):
        bindings = to_list(x.cdr.car)
        names = [b.car for b in bindings]
        inner = tuple(scope) + tuple(names)
        inits = [self.compile(b.cdr.car, mod, inner) for b in bindings]
        fs, _ = self._body(to_list(x.cdr.cdr), mod, inner)

        def run(env):
            e = Env({}, env)
            for nme, f in zip(names, inits):
                e.vars[nme] = f(e)
            r = UNDEF
            for g in fs:
                r = g(e)
            return r
        return run

    sf_letrec_star = sf_letrec

    def _formals(self, f):
        ps, rest = [], None
        while isinstance(f, Pair):
            ps.append(f.car)
            f = f.cdr
        if isinstance(f, Sym):
            rest = f
        return ps, rest

    def _bind_values(self, v, ps, rest, d):
        vals = list(v) if isinstance(v, Values) else [v]
        if len(vals) < len(ps) or (rest is None and len(vals) != len(ps)):
            raise SchemeError("received %d values for %d formals" % (len(vals), len(ps)))
        for p, val in zip(ps, vals):
            d[p] = val
        if rest is not None:
            d[rest] = from_list(vals[len(ps):])

    def sf_receive(self, x, mod, scope):
        ps, rest = self._formals(x.cdr.car)
        expr = self.compile(x.cdr.cdr.car, mod, scope)
        inner = tuple(scope) + tuple(ps) + ((rest,) if rest else ())
        fs, _ = self._body(to_list(x.cdr.cdr.cdr), mod, inner)

        def run(env):
            d = {}
            self._bind_values(expr(env), ps, rest, d)
            e = Env(d, env)
            r = UNDEF
            for g in fs:
                r = g(e)
            return r
        return run

    def _let_values(self, x, mod, scope, sequential):
        clauses = to_list(x.cdr.car)
        specs = []
        sc = tuple(scope)
        allnames = []
        for c in clauses:
            ps, rest = self._formals(c.car)
            specs.append((ps, rest, self.compile(c.cdr.car, mod, sc)))
            names = ps + ([rest] if rest else [])
            allnames += names
            if sequential:
                sc = sc + tuple(names)
        inner = tuple(scope) + tuple(allnames)
        fs, _ = self._body(to_list(x.cdr.cdr), mod, inner)

        def run(env):
            if sequential:
                for ps, rest, f in specs:
                    d = {}
                    self._bind_values(f(env), ps, rest, d)
                    env = Env(d, env)
                e = Env({}, env)
            else:
                d = {}
                for ps, rest, f in specs:
                    self._bind_values(f(env), ps, rest, d)
                e = Env(d, env)
            r = UNDEF
            for g in fs:
                r = g(e)
            return r
        return run

    def sf_let_values(self, x, mod, scope):
        return self._let_values(x, mod, scope, False)

    def sf_let_star_values(self, x, mod, scope):
        return self._let_values(x, mod, scope, True)

    def sf_let_optionals_star(self, x, mod, scope):
        src = self.compile(x.cdr.car, mod, scope)
        specs = to_list(x.cdr.cdr.car)
        names = [s.car for s in specs]
        defaults = [self.compile(s.cdr.car, mod, scope) for s in specs]
        inner = tuple(scope) + tuple(names)
        fs, _ = self._body(to_list(x.cdr.cdr.cdr), mod, inner)

        def run(env):
            given = to_list(src(env))
            d = {}
            for k, nme in enumerate(names):
                d[nme] = given[k] if k < len(given) else defaults[k](env)
            e = Env(d, env)
            r = UNDEF
            for g in fs:
                r = g(e)
            return r
        return run

    def sf_cond(self, x, mod, scope):
        clauses = []
        for c in to_list(x.cdr):
            test = c.car
            body = [self.compile(f, mod, scope) for f in to_list(c.cdr)]
            clauses.append((None if test == "else" else self.compile(test, mod, scope), body))

        def run(env):
            for t, body in clauses:
                v = True if t is None else t(env)
                if v is not False:
                    r = v
                    for g in body:
                        r = g(env)
                    return r
            return UNDEF
        return run

    def sf_and(self, x, mod, scope):
        fs = [self.compile(f, mod, scope) for f in to_list(x.cdr)]

        def run(env):
            r = True
            for f in fs:
                r = f(env)
                if r is False:
                    return False
            return r
        return run

    def sf_or(self, x, mod, scope):
        fs = [self.compile(f, mod, scope) for f in to_list(x.cdr)]

        def run(env):
            for f in fs:
                r = f(env)
                if r is not False:
                    return r
            return False
        return run

    def sf_when(self, x, mod, scope):
        c = self.compile(x.cdr.car, mod, scope)
        body = self.sf_begin(x.cdr, mod, scope)
        return lambda env: body(env) if c(env) is not False else UNDEF

    def sf_unless(self, x, mod, scope):
        c = self.compile(x.cdr.car, mod, scope)
        body = self.sf_begin(x.cdr, mod, scope)
        return lambda env: body(env) if c(env) is False else UNDEF

    def sf_dotimes(self, x, mod, scope):
        spec = x.cdr.car
        var = spec.car
        n = self.compile(spec.cdr.car, mod, scope)
        fs, _ = self._body(to_list(x.cdr.cdr), mod, tuple(scope) + (var,))

        def run(env):
            for i in range(n(env)):
                e = Env({var: i}, env)
                for g in fs:
                    g(e)
            return UNDEF
        return run

    def _update(self, x, mod, scope, fn):
        name = x.cdr.car
        delta = self.compile(x.cdr.cdr.car, mod, scope) if x.cdr.cdr is not NIL else (lambda env: 1)
        get = self.compile(name, mod, scope)
        box = {}

        def val(env):
            box["v"] = fn(get(env), delta(env))
            return box["v"]
        st = self._setter(name, mod, scope, val)

        def run(env):
            st(env)
            return box["v"]
        return run

    def sf_inc_bang(self, x, mod, scope):
        return self._update(x, mod, scope, add)

    def sf_dec_bang(self, x, mod, scope):
        return self._update(x, mod, scope, sub)

    def sf_push_bang(self, x, mod, scope):
        name = x.cdr.car
        item = self.compile(x.cdr.cdr.car, mod, scope)
        get = self.compile(name, mod, scope)
        return self._setter(name, mod, scope, lambda env: Pair(item(env), get(env)))

    def sf_pop_bang(self, x, mod, scope):
        name = x.cdr.car
        get = self.compile(name, mod, scope)
        box = {}

        def val(env):
            p = get(env)
            box["v"] = p.car
            return p.cdr
        st = self._setter(name, mod, scope, val)

        def run(env):
            st(env)
            return box["v"]
        return run

    def sf_cut(self, x, mod, scope):
        parts = to_list(x.cdr)
        fs = [None if p == "<>" else self.compile(p, mod, scope) for p in parts]

        def run(env):
            fixed = [None if f is None else f(env) for f in fs]

            def proc(*args):
                it = iter(args)
                vals = [next(it) if v is None and f is None else v for v, f in zip(fixed, fs)]
                return vals[0](*vals[1:])
            return proc
        return run


def _one(v):
    """A multiple-values result in a single-value context: Gauche takes the
    first value (e.g. get-normal subtracting dist-func results,
    geometry.scm:637-643)."""
    if v.__class__ is Values:
        return v[0] if len(v) else UNDEF
    return v


def _make_call(fc, acs):
    n = len(acs)
    if n == 0:
        return lambda env: fc(env)()
    if n == 1:
        a0 = acs[0]
        return lambda env: fc(env)(_one(a0(env)))
    if n == 2:
        a0, a1 = acs
        return lambda env: fc(env)(_one(a0(env)), _one(a1(env)))
    if n == 3:
        a0, a1, a2 = acs
        return lambda env: fc(env)(_one(a0(env)), _one(a1(env)), _one(a2(env)))
    return lambda env: fc(env)(*[_one(a(env)) for a in acs])
