"""GML evaluator (host front end): restates internal/gml/evaluator.go.

The evaluator runs a GML program on the host; the `render` builtin hands a
RenderArgs (scene.RenderArgs) to a callback, exactly like EvalState.Render
(evaluator.go:48, :1168-1199). Values mirror the Go types: VInt (int64
wraparound), VReal (float64), VBool, VString, Vec3 (*prim.Vec3), VClosure
(code + environment snapshot), VArray, Material (value), PointLight and the
scene objects of ../scene.py (with `surface` a SurfaceFn).
"""
import math

from .. import gomath
from .. import scene as S
from . import syntax as X
from .gofmt import format_float, go_g

INT64_MIN = -(1 << 63)


def wrap64(v):
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def go_f2i(x):
    """int(x) for float64 x on amd64 (CVTTSD2SQ): truncation, MinInt64 on NaN/overflow."""
    if x != x or not (-9223372036854775808.0 <= x < 9223372036854775808.0):
        return INT64_MIN
    return int(x)


class GMLError(Exception):
    pass


class VInt(int):
    def __str__(self):
        return "%d" % int(self)


class VReal(float):
    def __str__(self):
        return format_float(float(self))


class VBool:
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = bool(v)

    def __str__(self):
        return "true" if self.v else "false"


class VString(str):
    def __str__(self):
        return X._go_quote(str.__str__(self))


class Vec3(tuple):
    """*prim.Vec3; String() = "[%v, %v, %v]" (vec.go:13-15)."""

    def __new__(cls, x, y, z):
        return tuple.__new__(cls, (float(x), float(y), float(z)))

    def __str__(self):
        return "[%s, %s, %s]" % (go_g(self[0]), go_g(self[1]), go_g(self[2]))


class VClosure:
    __slots__ = ("code", "env")

    def __init__(self, code, env):
        self.code = code
        self.env = env

    def __str__(self):
        return "Closure(%s, env=%s)" % (X.token_list_string(self.code), env_string(self.env))


class VArray:
    __slots__ = ("elements",)

    def __init__(self, elements):
        self.elements = elements

    def __str__(self):
        return "[" + ", ".join(value_str(e) for e in self.elements) + "]"


class SurfaceFn:
    """VSurfaceFn (evaluator.go:95-101): exactly one of closure / material."""
    __slots__ = ("closure", "material", "state")

    def __init__(self, closure=None, material=None, state=None):
        self.closure = closure
        self.material = material
        self.state = state


def value_str(v):
    if isinstance(v, S.Material):
        return "Material(Color: %s Refl: %s Kd: %s Ks: %s N: %s)" % (
            Vec3(*v.color), go_g(v.reflectivity), go_g(v.kd), go_g(v.ks), go_g(v.specular_exponent))
    if isinstance(v, S.PointLight):
        return "PointLight(pos=%s, color=%s)" % (Vec3(*v.position), Vec3(*v.color))
    if isinstance(v, S.Sphere):
        return "Sphere(C: [0, 0, 0], R: 1)"
    if isinstance(v, S.Cube):
        return "Cube(...)"
    if isinstance(v, S.Cylinder):
        return "Cylinder(...)"
    if isinstance(v, S.Plane):
        return "Pt: %s, Normal: %s" % (Vec3(*v.point), Vec3(*v.normal))
    if isinstance(v, S.Union):
        return "Union([%s])" % " ".join(value_str(o) for o in v.objects)
    if isinstance(v, S.Difference):
        return "Difference(%s, %s)" % (value_str(v.a), value_str(v.b))
    return str(v)


def env_string(env, idmap=None):
    """Environment.String / DebugStringCtx: bindings sorted by id."""
    parts = []
    for i in sorted(env):
        if idmap is not None:
            name = idmap.id_name.get(i, "%d (?)" % i)
            parts.append("%s: %s" % (name, debug_str(env[i], idmap)))
        else:
            parts.append("%d: %s" % (i, value_str(env[i])))
    return "{" + ", ".join(parts) + "}"


def debug_str(v, idmap):
    if isinstance(v, VClosure):
        return "Closure(%s, env=%s)" % (X.token_list_string(v.code), env_string(v.env, idmap))
    return value_str(v)


class EvalState:
    """EvalState (evaluator.go:43-50)."""

    def __init__(self, render=None, extensions=False):
        self.stack = []
        self.ids = X.IDMapping()
        self.env = {}
        self.render = render
        self.cur = None
        # ICFP 2000 operators the reference lacks (cone, light, spotlight,
        # real): off by default, so programs behave exactly as in the reference
        # ("unbound identifier" for these names).
        self.extensions = extensions

    # -- program entry points (evaluator.go:305-356) --
    def parse_and_eval(self, text):
        self.eval(X.parse_text(text, self.ids))

    def parse_and_eval_file(self, path):
        self.eval(X.parse_file(path, self.ids))

    def clone(self):
        c = EvalState(self.render, self.extensions)
        c.stack = list(self.stack)
        c.ids = self.ids.clone()
        c.env = dict(self.env)
        c.cur = self.cur
        return c

    def eval(self, program):
        for tok in program:
            self.step(tok)

    def step(self, tok):
        """EvalOneStep (evaluator.go:365-414)."""
        self.cur = tok
        t = type(tok)
        if t is X.IntLit:
            self.stack.append(VInt(tok.value))
        elif t is X.FloatLit:
            self.stack.append(VReal(tok.value))
        elif t is X.BoolLit:
            self.stack.append(VBool(tok.value))
        elif t is X.StringLit:
            self.stack.append(VString(tok.value))
        elif t is X.Function:
            self.stack.append(VClosure(tok.body, dict(self.env)))
        elif t is X.Binder:
            self.env[tok.id] = self.pop()
        elif t is X.Identifier:
            b = BUILTINS.get(tok.name)
            if b is None and self.extensions:
                b = EXT_BUILTINS.get(tok.name)
            if b is not None:
                b(self)
                return
            v = self.env.get(tok.id)
            if v is None:
                raise GMLError("%d:%d: unbound identifier: %s" % (tok.pos[0], tok.pos[1], tok.name))
            self.stack.append(v)
        elif t is X.Array:
            old = self.stack
            self.stack = []
            try:
                self.eval(tok.elements)
                arr = VArray(self.stack)
            finally:
                self.stack = old
            self.stack.append(arr)
        else:
            raise GMLError("unknown token: %r" % tok)

    def pop(self):
        if not self.stack:
            p = self.cur.pos if self.cur is not None else (0, 0)
            raise GMLError("%d:%d: empty stack" % p)
        return self.stack.pop()

    def pop_t(self, typ, what):
        v = self.pop()
        if not isinstance(v, typ):
            raise GMLError("type mismatch: expected %s, got %s (%s)" % (what, value_str(v), type(v).__name__))
        return v

    def eval_closure(self, c):
        """EvalClosure (evaluator.go:433-438): run with a copy of the closure's
        environment, then restore the caller's."""
        old = self.env
        self.env = dict(c.env)
        try:
            self.eval(c.code)
        finally:
            self.env = old


def _real(e):
    return e.pop_t(VReal, "gml.VReal")


def _int(e):
    return e.pop_t(VInt, "gml.VInt")


def _pop2(e, fn):
    y = fn(e)
    x = fn(e)
    return x, y


def _vec(e):
    return e.pop_t(Vec3, "*prim.Vec3")


def _closure(e):
    return e.pop_t(VClosure, "gml.VClosure")


_SCENE_TYPES = (S.Sphere, S.Cube, S.Cylinder, S.Plane, S.Union, S.Difference, S.Cone, S.Intersect)


def _sceneobj(e):
    return e.pop_t(_SCENE_TYPES, "gml.SceneObject")


def eval_surface_fn(face, u, v, state, sf):
    """EvalSurfaceFn (evaluator.go:672-727): a Material, or the contest's
    `color kd ks n` with Reflectivity = ks."""
    if sf.material is not None:
        return sf.material
    if state is None:
        raise GMLError("nil GML eval state")
    state.stack.append(VInt(face))
    state.stack.append(VReal(u))
    state.stack.append(VReal(v))
    state.eval_closure(sf.closure)
    first = state.pop()
    if isinstance(first, S.Material):
        return first
    if not isinstance(first, VReal):
        raise GMLError("type mismatch: expected gml.VReal")
    kd, ks = _pop2(state, _real)
    color = _vec(state)
    return S.Material(color=tuple(color), kd=float(kd), ks=float(ks), specular_exponent=float(first),
                      reflectivity=float(ks))


def referenced_vars(code):
    """referencedVars (evaluator.go:616-650): non-builtin identifiers, nested included."""
    out = []
    todo = list(code)
    while todo:
        nxt = []
        for t in todo:
            if isinstance(t, X.Identifier):
                if t.name not in BUILTINS:
                    out.append(t.name)
            elif isinstance(t, X.Array):
                nxt.extend(t.elements)
            elif isinstance(t, X.Function):
                nxt.extend(t.body)
        todo = nxt
    return out


def _surface(e):
    """maybeSimplifySurfaceFn (evaluator.go:729-750)."""
    c = _closure(e)
    if not referenced_vars(c.code):
        try:
            m = eval_surface_fn(0, 0.0, 0.0, e, SurfaceFn(closure=c))
        except GMLError as err:
            raise GMLError("error while precomputing closure: %s" % err)
        return SurfaceFn(material=m)
    return SurfaceFn(closure=c)


# ---- builtins (evaluator.go:550-602, 752-1199) ----

def b_apply(e):
    e.eval_closure(_closure(e))


def b_point(e):
    z = _real(e)
    y = _real(e)
    x = _real(e)
    e.stack.append(Vec3(x, y, z))


def b_pointlight(e):
    color = _vec(e)
    pos = _vec(e)
    e.stack.append(S.PointLight(tuple(pos), tuple(color)))


def b_sphere(e):
    e.stack.append(S.Sphere(_surface(e)))


def b_cube(e):
    e.stack.append(S.Cube(_surface(e)))


def b_cylinder(e):
    e.stack.append(S.Cylinder(_surface(e)))


def b_plane(e):
    e.stack.append(S.Plane(_surface(e)))


def _binop(fn, typ):
    def run(e):
        b = typ(e)
        a = typ(e)
        e.stack.append(fn(a, b))
    return run


def _idiv(a, b):
    if b == 0:
        raise GMLError("runtime error: integer divide by zero")
    q = abs(int(a)) // abs(int(b))
    return VInt(wrap64(q if (a < 0) == (b < 0) else -q))


def _imod(a, b):
    if b == 0:
        raise GMLError("runtime error: integer divide by zero")
    r = abs(int(a)) % abs(int(b))
    return VInt(r if a >= 0 else -r)


def b_material(e):
    floats = [None] * 7
    for i in range(6, -1, -1):
        floats[i] = float(_real(e))
    color = _vec(e)
    e.stack.append(S.Material(color=tuple(color), reflectivity=floats[0], fuzziness=floats[1],
                              transparency=floats[2], refractive_index=floats[3], kd=floats[4],
                              ks=floats[5], specular_exponent=floats[6]))


def _clamp(typ, zero, one):
    def run(e):
        x = typ(e)
        if x < 0:
            x = zero
        elif x > 1:
            x = one
        e.stack.append(x)
    return run


DEG_TO_RAD = 0.017453292519943295  # Go const math.Pi / 180.0, rounded once


def b_sin(e):
    e.stack.append(VReal(gomath.go_sin(DEG_TO_RAD * float(_real(e)))))


def b_cos(e):
    e.stack.append(VReal(gomath.go_cos(DEG_TO_RAD * float(_real(e)))))


def b_getx(e):
    e.stack.append(VReal(_vec(e)[0]))


def b_gety(e):
    e.stack.append(VReal(_vec(e)[1]))


def b_getz(e):
    e.stack.append(VReal(_vec(e)[2]))


def b_length(e):
    e.stack.append(VInt(len(e.pop_t(VArray, "gml.VArray").elements)))


def b_sqrt(e):
    x = float(_real(e))
    e.stack.append(VReal(math.sqrt(x) if x >= 0 else (x if x != x else math.nan)))


def b_frac(e):
    x = float(_real(e))
    e.stack.append(VReal(x - float(go_f2i(x))))


def b_get(e):
    i = _int(e)
    arr = e.pop_t(VArray, "gml.VArray")
    n = len(arr.elements)
    if i < 0 or i >= n:
        raise GMLError("array index out of bounds: %d vs %d" % (i, n))
    e.stack.append(arr.elements[i])


def b_if(e):
    tc, fc = _pop2(e, _closure)
    cond = e.pop_t(VBool, "gml.VBool")
    e.eval_closure(tc if cond.v else fc)


def _xform(mk):
    def run(e):
        args = mk(e)
        s = _sceneobj(e)
        e.stack.append(s.transform(args))
    return run


def _translate(e):
    z = _real(e)
    y = _real(e)
    x = _real(e)
    return gomath.translate(float(x), float(y), float(z))


def _scale(e):
    z = _real(e)
    y = _real(e)
    x = _real(e)
    return gomath.scale(float(x), float(y), float(z))


def _uscale(e):
    s = float(_real(e))
    return gomath.scale(s, s, s)


def _rot(fn):
    def mk(e):
        a = float(_real(e))
        return fn(a * math.pi / 180)
    return mk


def b_union(e):
    a = _sceneobj(e)
    b = _sceneobj(e)
    e.stack.append(S.Union((a, b)))


def b_difference(e):
    a, b = _pop2(e, _sceneobj)
    e.stack.append(S.Difference(a, b))


def pop_render_args(e):
    """popRenderArgs (evaluator.go:1113-1166)."""
    file = e.pop_t(VString, "gml.VString")
    height = _int(e)
    width = _int(e)
    fov = _real(e)
    depth = _int(e)
    obj = _sceneobj(e)
    lights = e.pop_t(VArray, "gml.VArray")
    amb = _vec(e)
    ls = []
    ok = (S.PointLight, S.DirectionalLight, S.SpotLight) if e.extensions else (S.PointLight,)
    for l in lights.elements:
        if not isinstance(l, ok):
            raise GMLError("expected lights array to contain *PointLight, got %s" % type(l).__name__)
        ls.append(l)
    return S.RenderArgs(ambient=tuple(amb), lights=ls, scene=obj, depth=int(depth), fov=float(fov),
                        width=int(width), height=int(height), file=str.__str__(file))


def b_render(e):
    args = pop_render_args(e)
    if e.render is None:
        raise GMLError("render function not set")
    e.render(e, args)


def b_render_bg(e):
    bg0, bg1 = _pop2(e, _vec)
    args = pop_render_args(e)
    args.bg_start = tuple(bg0)
    args.bg_end = tuple(bg1)
    if e.render is None:
        raise GMLError("render function not set")
    e.render(e, args)


def _mkbool(fn):
    return lambda a, b: VBool(fn(a, b))


BUILTINS = {
    "addf": _binop(lambda a, b: VReal(float(a) + float(b)), _real),
    "addi": _binop(lambda a, b: VInt(wrap64(a + b)), _int),
    "apply": b_apply,
    "clampf": _clamp(_real, VReal(0.0), VReal(1.0)),
    "cos": b_cos,
    "cube": b_cube,
    "cylinder": b_cylinder,
    "if": b_if,
    "difference": b_difference,
    "divi": _binop(_idiv, _int),
    "divf": _binop(lambda a, b: VReal(_fdiv(float(a), float(b))), _real),
    "eqi": _binop(_mkbool(lambda a, b: int(a) == int(b)), _int),
    "eqf": _binop(_mkbool(lambda a, b: float(a) == float(b)), _real),
    "floor": None,
    "frac": b_frac,
    "get": b_get,
    "getx": b_getx,
    "gety": b_gety,
    "getz": b_getz,
    "length": b_length,
    "lessi": _binop(_mkbool(lambda a, b: int(a) < int(b)), _int),
    "lessf": _binop(_mkbool(lambda a, b: float(a) < float(b)), _real),
    "material": b_material,
    "modi": _binop(_imod, _int),
    "muli": _binop(lambda a, b: VInt(wrap64(a * b)), _int),
    "mulf": _binop(lambda a, b: VReal(float(a) * float(b)), _real),
    "negi": lambda e: e.stack.append(VInt(wrap64(-_int(e)))),
    "negf": lambda e: e.stack.append(VReal(-float(_real(e)))),
    "plane": b_plane,
    "point": b_point,
    "pointlight": b_pointlight,
    "render": b_render,
    "renderWithBgGradient": b_render_bg,
    "rotatex": _xform(_rot(gomath.rotate_x)),
    "rotatey": _xform(_rot(gomath.rotate_y)),
    "rotatez": _xform(_rot(gomath.rotate_z)),
    "scale": _xform(_scale),
    "sin": b_sin,
    "sphere": b_sphere,
    "sqrt": b_sqrt,
    "subi": _binop(lambda a, b: VInt(wrap64(a - b)), _int),
    "subf": _binop(lambda a, b: VReal(float(a) - float(b)), _real),
    "translate": _xform(_translate),
    "union": b_union,
    "uscale": _xform(_uscale),
}


def _fdiv(a, b):
    """float64 a / b with IEEE semantics (Python raises on /0)."""
    if b == 0.0:
        if a != a or a == 0.0:
            return math.nan
        neg = (a < 0) != (math.copysign(1.0, b) < 0)
        return -math.inf if neg else math.inf
    return a / b


def b_floor2(e):
    x = float(_real(e))
    f = math.floor(x) if math.isfinite(x) else x
    e.stack.append(VInt(go_f2i(f)))


BUILTINS["floor"] = b_floor2


# ---- contest extensions (ICFP 2000 task; not in the reference, parity-unpinned) ----

def b_cone(e):
    e.stack.append(S.Cone(_surface(e)))


def b_light(e):
    """`dir color light`: directional light travelling along dir."""
    color = _vec(e)
    d = _vec(e)
    e.stack.append(S.DirectionalLight(tuple(d), tuple(color)))


def b_spotlight(e):
    """`pos at color cutoff exp spotlight`."""
    exp = float(_real(e))
    cutoff = float(_real(e))
    color = _vec(e)
    at = _vec(e)
    pos = _vec(e)
    e.stack.append(S.SpotLight(tuple(pos), tuple(at), tuple(color), cutoff, exp))


def b_real(e):
    """`i real`: Go float64(int64) (round to nearest)."""
    e.stack.append(VReal(float(int(_int(e)))))


def b_intersect(e):
    """`s1 s2 intersect`: the solid in both (argument order as `difference`)."""
    a, b = _pop2(e, _sceneobj)
    e.stack.append(S.Intersect(a, b))


EXT_BUILTINS = {"cone": b_cone, "light": b_light, "spotlight": b_spotlight, "real": b_real,
                "intersect": b_intersect}
