"""Compile GML surface closures to the device VM bytecode.

The reference evaluates a closure surface per hit with the GML interpreter
(EvalSurfaceFn, internal/gml/evaluator.go:672-727: push face, u, v; run the
closure in a copy of its environment; pop a Material or `color kd ks n`). Here
the closure is evaluated once on the host *symbolically*: face, u and v are
runtime registers, everything else (the captured environment, literals,
constant arrays and closures) is folded; operations on runtime values are
emitted as register instructions. Control flow on runtime conditions (`if`)
evaluates both branch closures and merges their results with selects; error
conditions the reference would raise at run time (array bounds, integer
division by zero, |y| > 1 on spheres) become error checks predicated on the
path that reaches them. The result is a straight-line program -- no loops, no
calls -- executed per hit by the kernel's VM (csrc/rt_kernel.hip `run_vm`).

Bytecode (include/rt_abi.h, rt_program_set): instruction = 2 x uint32,
  w0 = op | dst << 8 | a << 16 | b << 24,   w1 = c (third operand / constant index)
registers are 64-bit (f64, i64 or bool 0/1); r0..r9 = the result Material
(colour xyz, reflectivity, fuzziness, transparency, refractive index, kd, ks,
n); r10 = face (i64), r11 = u, r12 = v; temporaries from r13.
"""
import math

from .. import scene as S
from . import syntax as X
from .evaluator import (BUILTINS, VArray, VBool, VClosure, VInt, VReal, Vec3, _fdiv, go_f2i, wrap64,
                        DEG_TO_RAD)
from .. import gomath

# opcodes (keep in sync with csrc/rt_kernel.hip enum VmOp)
OPS = ["NOP", "CONST", "MOV", "ADDF", "SUBF", "MULF", "DIVF", "NEGF", "ADDI", "SUBI", "MULI", "DIVI", "MODI",
       "NEGI", "LTF", "EQF", "LTI", "EQI", "SEL", "FLOOR", "FRAC", "SQRT", "SIN", "COS", "CLAMPF", "CLAMPI",
       "TBL", "AND", "OR", "NOT", "ERR", "RET"]
OP = {n: i for i, n in enumerate(OPS)}
R_OUT = 0
R_FACE, R_U, R_V = 10, 11, 12
R_FIRST_TEMP = 13
MAX_REGS = 64
MAX_INSTRS = 4096
MAX_APPLY_DEPTH = 64


class CompileError(Exception):
    pass


class Reg:
    __slots__ = ("r", "t")

    def __init__(self, r, t):
        self.r = r
        self.t = t  # 'f', 'i', 'b'


class SVec3:
    __slots__ = ("c",)

    def __init__(self, c):
        self.c = tuple(c)


class SMat:
    __slots__ = ("color", "f")  # f: refl, fuzz, transp, ior, kd, ks, n

    def __init__(self, color, f):
        self.color = color
        self.f = tuple(f)


class SClosure:
    __slots__ = ("code", "env")

    def __init__(self, code, env):
        self.code = code
        self.env = env


class SArray:
    __slots__ = ("el",)

    def __init__(self, el):
        self.el = list(el)


def _is_real(v):
    return isinstance(v, VReal) or (isinstance(v, Reg) and v.t == "f")


def _is_int(v):
    return isinstance(v, VInt) or (isinstance(v, Reg) and v.t == "i")


def _is_bool(v):
    return isinstance(v, VBool) or (isinstance(v, Reg) and v.t == "b")


def _is_vec(v):
    return isinstance(v, (Vec3, SVec3))


def _bits_f(x):
    import struct
    return struct.unpack("<Q", struct.pack("<d", float(x)))[0]


def _bits_i(x):
    return int(x) & ((1 << 64) - 1)


class Program:
    def __init__(self):
        self.code = []      # (op, dst, a, b, c)
        self.consts = []    # u64 bit patterns
        self.nreg = R_FIRST_TEMP
        self._cmemo = {}

    def words(self):
        out = []
        for op, d, a, b, c in self.code:
            out.append(op | (d << 8) | (a << 16) | (b << 24))
            out.append(c & 0xFFFFFFFF)
        return out


class Compiler:
    def __init__(self, base_stack):
        self.p = Program()
        self.stack = list(base_stack)
        self.base = list(base_stack)
        self.env = {}
        self.pred = True  # path predicate: True or Reg('b')
        self.depth = 0

    # ---- emission ----
    def _reg(self, t):
        if self.p.nreg >= MAX_REGS:
            raise CompileError("surface function needs more than %d registers" % MAX_REGS)
        r = Reg(self.p.nreg, t)
        self.p.nreg += 1
        return r

    def emit(self, op, t, a=0, b=0, c=0, dst=None):
        if len(self.p.code) >= MAX_INSTRS:
            raise CompileError("surface function too large for the device VM")
        if dst is None:
            dst = self._reg(t)
        self.p.code.append((OP[op], dst.r, a, b, c))
        return dst

    def const(self, bits, t):
        key = (bits, t)
        r = self.p._cmemo.get(key)
        if r is not None:
            return r
        try:
            k = self.p.consts.index(bits)
        except ValueError:
            k = len(self.p.consts)
            self.p.consts.append(bits)
        r = self.emit("CONST", t, c=k)
        self.p._cmemo[key] = r
        return r

    def freg(self, v):
        if isinstance(v, Reg):
            return v
        return self.const(_bits_f(float(v)), "f")

    def ireg(self, v):
        if isinstance(v, Reg):
            return v
        return self.const(_bits_i(int(v)), "i")

    def breg(self, v):
        if isinstance(v, Reg):
            return v
        return self.const(1 if v.v else 0, "b")

    def check(self, bad):
        """Flag a run-time error when `bad` (Reg b) holds on the current path."""
        if self.pred is not True:
            bad = self.emit("AND", "b", bad.r, self.pred.r)
        self.emit("ERR", "b", bad.r, dst=Reg(0, "b"))

    # ---- stack ----
    def pop(self):
        if len(self.stack) == 0:
            raise CompileError("empty stack")
        return self.stack.pop()

    def push(self, v):
        self.stack.append(v)

    def pop_real(self):
        v = self.pop()
        if not _is_real(v):
            raise CompileError("type mismatch: expected gml.VReal")
        return v

    def pop_int(self):
        v = self.pop()
        if not _is_int(v):
            raise CompileError("type mismatch: expected gml.VInt")
        return v

    def pop_bool(self):
        v = self.pop()
        if not _is_bool(v):
            raise CompileError("type mismatch: expected gml.VBool")
        return v

    def pop_vec(self):
        v = self.pop()
        if not _is_vec(v):
            raise CompileError("type mismatch: expected *prim.Vec3")
        return v

    def pop_closure(self):
        v = self.pop()
        if isinstance(v, VClosure):
            return SClosure(v.code, dict(v.env))
        if isinstance(v, SClosure):
            return v
        raise CompileError("type mismatch: expected gml.VClosure (or a closure chosen at run time)")

    def pop_array(self):
        v = self.pop()
        if isinstance(v, (VArray, SArray)):
            return v
        raise CompileError("type mismatch: expected gml.VArray")

    # ---- evaluation ----
    def run_closure(self, c):
        self.depth += 1
        if self.depth > MAX_APPLY_DEPTH:
            raise CompileError("surface function recursion too deep for the device VM")
        old = self.env
        self.env = dict(c.env)
        try:
            self.run(c.code)
        finally:
            self.env = old
            self.depth -= 1

    def run(self, code):
        for tok in code:
            self.step(tok)

    def step(self, tok):
        t = type(tok)
        if t is X.IntLit:
            self.push(VInt(tok.value))
        elif t is X.FloatLit:
            self.push(VReal(tok.value))
        elif t is X.BoolLit:
            self.push(VBool(tok.value))
        elif t is X.StringLit:
            from .evaluator import VString
            self.push(VString(tok.value))
        elif t is X.Function:
            self.push(SClosure(tok.body, dict(self.env)))
        elif t is X.Binder:
            self.env[tok.id] = self.pop()
        elif t is X.Identifier:
            if tok.name in BUILTINS:
                fn = getattr(self, "b_" + tok.name, None)
                if fn is None:
                    raise CompileError("builtin %s is not supported in device surface functions" % tok.name)
                fn()
                return
            v = self.env.get(tok.id)
            if v is None:
                raise CompileError("unbound identifier: %s" % tok.name)
            if isinstance(v, VClosure):
                v = SClosure(v.code, dict(v.env))
            self.push(v)
        elif t is X.Array:
            old = self.stack
            self.stack = []
            try:
                self.run(tok.elements)
                els = self.stack
            finally:
                self.stack = old
            if all(not isinstance(e, (Reg, SVec3, SMat, SClosure, SArray)) for e in els):
                self.push(VArray(els))
            else:
                self.push(SArray(els))
        else:
            raise CompileError("unknown token")

    # ---- arithmetic builtins ----
    def _fbin(self, op, fold):
        b = self.pop_real()
        a = self.pop_real()
        if not isinstance(a, Reg) and not isinstance(b, Reg):
            self.push(VReal(fold(float(a), float(b))))
        else:
            self.push(self.emit(op, "f", self.freg(a).r, self.freg(b).r))

    def b_addf(self):
        self._fbin("ADDF", lambda a, b: a + b)

    def b_subf(self):
        self._fbin("SUBF", lambda a, b: a - b)

    def b_mulf(self):
        self._fbin("MULF", lambda a, b: a * b)

    def b_divf(self):
        self._fbin("DIVF", _fdiv)

    def b_negf(self):
        a = self.pop_real()
        self.push(VReal(-float(a)) if not isinstance(a, Reg) else self.emit("NEGF", "f", a.r))

    def _ibin(self, op, fold, zero_check=False):
        b = self.pop_int()
        a = self.pop_int()
        if not isinstance(a, Reg) and not isinstance(b, Reg):
            if zero_check and int(b) == 0:
                raise CompileError("runtime error: integer divide by zero (on every hit)")
            self.push(VInt(fold(int(a), int(b))))
            return
        if zero_check:
            if not isinstance(b, Reg):
                if int(b) == 0:
                    raise CompileError("runtime error: integer divide by zero (on every hit)")
            else:
                z = self.ireg(VInt(0))
                self.check(self.emit("EQI", "b", b.r, z.r))
        self.push(self.emit(op, "i", self.ireg(a).r, self.ireg(b).r))

    def b_addi(self):
        self._ibin("ADDI", lambda a, b: wrap64(a + b))

    def b_subi(self):
        self._ibin("SUBI", lambda a, b: wrap64(a - b))

    def b_muli(self):
        self._ibin("MULI", lambda a, b: wrap64(a * b))

    def b_divi(self):
        def f(a, b):
            q = abs(a) // abs(b)
            return wrap64(q if (a < 0) == (b < 0) else -q)
        self._ibin("DIVI", f, True)

    def b_modi(self):
        def f(a, b):
            r = abs(a) % abs(b)
            return r if a >= 0 else -r
        self._ibin("MODI", f, True)

    def b_negi(self):
        a = self.pop_int()
        self.push(VInt(wrap64(-int(a))) if not isinstance(a, Reg) else self.emit("NEGI", "i", a.r))

    def _cmp(self, pop, op, fold, conv, reg):
        b = pop()
        a = pop()
        if not isinstance(a, Reg) and not isinstance(b, Reg):
            self.push(VBool(fold(conv(a), conv(b))))
        else:
            self.push(self.emit(op, "b", reg(a).r, reg(b).r))

    def b_lessf(self):
        self._cmp(self.pop_real, "LTF", lambda a, b: a < b, float, self.freg)

    def b_eqf(self):
        self._cmp(self.pop_real, "EQF", lambda a, b: a == b, float, self.freg)

    def b_lessi(self):
        self._cmp(self.pop_int, "LTI", lambda a, b: a < b, int, self.ireg)

    def b_eqi(self):
        self._cmp(self.pop_int, "EQI", lambda a, b: a == b, int, self.ireg)

    def _funary(self, op, fold):
        a = self.pop_real()
        if not isinstance(a, Reg):
            self.push(fold(float(a)))
        else:
            t = "i" if op == "FLOOR" else "f"
            self.push(self.emit(op, t, a.r))

    def b_floor(self):
        self._funary("FLOOR", lambda x: VInt(go_f2i(math.floor(x) if math.isfinite(x) else x)))

    def b_frac(self):
        self._funary("FRAC", lambda x: VReal(x - float(go_f2i(x))))

    def b_sqrt(self):
        self._funary("SQRT", lambda x: VReal(math.sqrt(x) if x >= 0 else math.nan))

    def b_sin(self):
        self._funary("SIN", lambda x: VReal(gomath.go_sin(DEG_TO_RAD * x)))

    def b_cos(self):
        self._funary("COS", lambda x: VReal(gomath.go_cos(DEG_TO_RAD * x)))

    def b_clampf(self):
        def f(x):
            return VReal(0.0 if x < 0 else (1.0 if x > 1 else x))
        self._funary("CLAMPF", f)

    def b_clampi(self):
        a = self.pop_int()
        if not isinstance(a, Reg):
            x = int(a)
            self.push(VInt(0 if x < 0 else (1 if x > 1 else x)))
        else:
            self.push(self.emit("CLAMPI", "i", a.r))

    # ---- points, arrays, materials ----
    def b_point(self):
        z = self.pop_real()
        y = self.pop_real()
        x = self.pop_real()
        if any(isinstance(c, Reg) for c in (x, y, z)):
            self.push(SVec3((x, y, z)))
        else:
            self.push(Vec3(x, y, z))

    def _get_comp(self, k):
        v = self.pop_vec()
        c = v[k] if isinstance(v, Vec3) else v.c[k]
        self.push(VReal(c) if not isinstance(c, Reg) else c)

    def b_getx(self):
        self._get_comp(0)

    def b_gety(self):
        self._get_comp(1)

    def b_getz(self):
        self._get_comp(2)

    def b_length(self):
        a = self.pop_array()
        self.push(VInt(len(a.elements if isinstance(a, VArray) else a.el)))

    def b_get(self):
        i = self.pop_int()
        arr = self.pop_array()
        els = arr.elements if isinstance(arr, VArray) else arr.el
        n = len(els)
        if not isinstance(i, Reg):
            if int(i) < 0 or int(i) >= n:
                raise CompileError("array index out of bounds (on every hit)")
            v = els[int(i)]
            self.push(SClosure(v.code, dict(v.env)) if isinstance(v, VClosure) else v)
            return
        # run-time index: bounds check, then a table lookup / select
        if n == 0:
            raise CompileError("array index out of bounds (on every hit)")
        zero = self.ireg(VInt(0))
        nn = self.ireg(VInt(n))
        neg = self.emit("LTI", "b", i.r, zero.r)
        inr = self.emit("LTI", "b", i.r, nn.r)
        out = self.emit("NOT", "b", inr.r)
        self.check(self.emit("OR", "b", neg.r, out.r))
        self.push(self._select(i, els))

    def _table(self, idx, values, t):
        k = len(self.p.consts)
        self.p.consts.append(len(values))
        for v in values:
            self.p.consts.append(_bits_f(v) if t == "f" else _bits_i(v))
        return self.emit("TBL", t, idx.r, c=k)

    def _select(self, idx, els):
        """Value of els[idx] for a run-time idx (already bounds-checked)."""
        if all(isinstance(e, VReal) for e in els):
            return self._table(idx, [float(e) for e in els], "f")
        if all(isinstance(e, VInt) for e in els):
            return self._table(idx, [int(e) for e in els], "i")
        if all(isinstance(e, VBool) for e in els):
            return self._table(idx, [1 if e.v else 0 for e in els], "b")
        if all(isinstance(e, Vec3) for e in els):
            return SVec3([self._table(idx, [float(e[k]) for e in els], "f") for k in range(3)])
        if all(isinstance(e, (VArray, SArray)) for e in els):
            # nested arrays: defer -- select element-wise when indexed again
            return _DynRow(idx, els)
        # general: select chain over the elements
        acc = els[0]
        for k in range(1, len(els)):
            kk = self.ireg(VInt(k))
            c = self.emit("EQI", "b", idx.r, kk.r)
            acc = self.merge(c, els[k], acc)
        return acc

    def b_material(self):
        fl = [self.pop_real() for _ in range(7)][::-1]
        color = self.pop_vec()
        if isinstance(color, Vec3) and not any(isinstance(f, Reg) for f in fl):
            self.push(S.Material(color=tuple(color), reflectivity=float(fl[0]), fuzziness=float(fl[1]),
                                 transparency=float(fl[2]), refractive_index=float(fl[3]), kd=float(fl[4]),
                                 ks=float(fl[5]), specular_exponent=float(fl[6])))
        else:
            c = color.c if isinstance(color, SVec3) else tuple(VReal(x) for x in color)
            self.push(SMat(c, fl))

    # ---- control ----
    def b_apply(self):
        self.run_closure(self.pop_closure())

    def b_if(self):
        fc = self.pop_closure()
        tc = self.pop_closure()
        cond = self.pop_bool()
        if not isinstance(cond, Reg):
            self.run_closure(tc if cond.v else fc)
            return
        base = list(self.stack)
        pred0 = self.pred
        ncond = self.emit("NOT", "b", cond.r)
        res = []
        for c, br in ((cond, tc), (ncond, fc)):
            self.stack = list(base)
            self.pred = c if pred0 is True else self.emit("AND", "b", pred0.r, c.r)
            self.run_closure(br)
            res.append(self.stack)
        self.pred = pred0
        st, sf = res
        if len(st) != len(sf):
            raise CompileError("if branches leave different stack depths (run-time dependent)")
        merged = []
        for a, b in zip(st, sf):
            merged.append(a if a is b else self.merge(cond, a, b))
        self.stack = merged

    def merge(self, c, a, b):
        """Value that is `a` when c holds, else `b`."""
        if _is_real(a) and _is_real(b):
            if not isinstance(a, Reg) and not isinstance(b, Reg) and _bits_f(a) == _bits_f(b):
                return a
            return self.emit("SEL", "f", c.r, self.freg(a).r, self.freg(b).r)
        if _is_int(a) and _is_int(b):
            if not isinstance(a, Reg) and not isinstance(b, Reg) and int(a) == int(b):
                return a
            return self.emit("SEL", "i", c.r, self.ireg(a).r, self.ireg(b).r)
        if _is_bool(a) and _is_bool(b):
            if not isinstance(a, Reg) and not isinstance(b, Reg) and a.v == b.v:
                return a
            return self.emit("SEL", "b", c.r, self.breg(a).r, self.breg(b).r)
        if _is_vec(a) and _is_vec(b):
            ca = a.c if isinstance(a, SVec3) else tuple(VReal(x) for x in a)
            cb = b.c if isinstance(b, SVec3) else tuple(VReal(x) for x in b)
            comps = [self.merge(c, x, y) for x, y in zip(ca, cb)]
            if all(not isinstance(x, Reg) for x in comps):
                return Vec3(*comps)
            return SVec3(comps)
        if isinstance(a, (S.Material, SMat)) and isinstance(b, (S.Material, SMat)):
            fa, fb = _mat_fields(a), _mat_fields(b)
            col = [self.merge(c, x, y) for x, y in zip(fa[0], fb[0])]
            fs = [self.merge(c, x, y) for x, y in zip(fa[1], fb[1])]
            return SMat(col, fs)
        if isinstance(a, (VArray, SArray)) and isinstance(b, (VArray, SArray)):
            ea = a.elements if isinstance(a, VArray) else a.el
            eb = b.elements if isinstance(b, VArray) else b.el
            if len(ea) != len(eb):
                raise CompileError("if branches yield arrays of different lengths")
            return SArray([x if x is y else self.merge(c, x, y) for x, y in zip(ea, eb)])
        if isinstance(a, _DynRow) and isinstance(b, _DynRow) and a.rows is b.rows:
            return _DynRow(self.merge(c, a.idx, b.idx), a.rows)
        raise CompileError("if branches yield values of different types (run-time dependent)")

    # ---- result ----
    def result(self):
        first = self.pop()
        if isinstance(first, (S.Material, SMat)):
            col, fs = _mat_fields(first)
        elif _is_real(first):
            ks = self.pop_real()
            kd = self.pop_real()
            color = self.pop_vec()
            col = color.c if isinstance(color, SVec3) else tuple(VReal(x) for x in color)
            z = VReal(0.0)
            fs = (ks, z, z, z, kd, ks, first)  # Reflectivity = ks (evaluator.go:724)
        else:
            raise CompileError("surface function must return a Material or `color kd ks n`")
        if len(self.stack) != len(self.base) or any(a is not b for a, b in zip(self.stack, self.base)):
            raise CompileError("surface function leaves values on the stack (hit-order dependent)")
        outs = list(col) + list(fs)
        for k, v in enumerate(outs):
            self.emit("MOV", "f", self.freg(v).r, dst=Reg(R_OUT + k, "f"))
        self.emit("RET", "f", dst=Reg(0, "f"))
        return self.p


class _DynRow:
    """els[idx] where els are arrays: indexed again -> 2-D table."""
    __slots__ = ("idx", "rows")

    def __init__(self, idx, rows):
        self.idx = idx
        self.rows = rows


def _mat_fields(m):
    if isinstance(m, S.Material):
        return (tuple(VReal(x) for x in m.color),
                tuple(VReal(x) for x in (m.reflectivity, m.fuzziness, m.transparency, m.refractive_index,
                                          m.kd, m.ks, m.specular_exponent)))
    return m.color, m.f


# `get` on a _DynRow (a row chosen at run time): patch b_get to handle it
_orig_get = Compiler.b_get


def _b_get(self):
    i = self.stack[-1] if self.stack else None
    arr = self.stack[-2] if len(self.stack) >= 2 else None
    if isinstance(arr, _DynRow):
        self.pop()
        self.pop()
        rows = [r.elements if isinstance(r, VArray) else r.el for r in arr.rows]
        lens = {len(r) for r in rows}
        if len(lens) != 1:
            raise CompileError("ragged nested array indexed at run time")
        L = lens.pop()
        if L == 0:
            raise CompileError("array index out of bounds (on every hit)")
        if not _is_int(i):
            raise CompileError("type mismatch: expected gml.VInt")
        ii = self.ireg(i)
        zero = self.ireg(VInt(0))
        nn = self.ireg(VInt(L))
        neg = self.emit("LTI", "b", ii.r, zero.r)
        inr = self.emit("LTI", "b", ii.r, nn.r)
        out = self.emit("NOT", "b", inr.r)
        self.check(self.emit("OR", "b", neg.r, out.r))
        lin = self.emit("ADDI", "i", self.emit("MULI", "i", arr.idx.r, nn.r).r, ii.r)
        flat = [e for r in rows for e in r]
        self.push(self._select(lin, flat))
        return
    _orig_get(self)


Compiler.b_get = _b_get


def compile_surface(sf, state_stack=()):
    """SurfaceFn (closure) -> Program. `state_stack`: the EvalState stack at
    render time (the per-thread clone EvalSurfaceFn pushes onto)."""
    c = Compiler(state_stack)
    c.push(Reg(R_FACE, "i"))
    c.push(Reg(R_U, "f"))
    c.push(Reg(R_V, "f"))
    clo = sf.closure
    c.run_closure(SClosure(clo.code, dict(clo.env)))
    return c.result()
