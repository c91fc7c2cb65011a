"""Python emulator of the device surface VM (csrc/rt_kernel.hip run_vm) --
test infrastructure: checks gml/surface_compiler.py against the GML
interpreter (gml/evaluator.py, the restatement of evaluator.go)."""
import math
import struct

from go_raytracer_amd import gomath
from go_raytracer_amd.gml.evaluator import DEG_TO_RAD, go_f2i, wrap64
from go_raytracer_amd.gml.surface_compiler import OPS, R_FACE, R_U, R_V


def f2b(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def b2f(b):
    return struct.unpack("<d", struct.pack("<Q", b & ((1 << 64) - 1)))[0]


def b2i(b):
    b &= (1 << 64) - 1
    return b - (1 << 64) if b >= (1 << 63) else b


def fdiv(a, b):
    if b == 0.0:
        if a != a or a == 0.0:
            return math.nan
        return -math.inf if (a < 0) != (math.copysign(1.0, b) < 0) else math.inf
    return a / b


def run(words, consts, face, u, v):
    R = [0] * 64
    R[R_FACE] = face & ((1 << 64) - 1)
    R[R_U] = f2b(u)
    R[R_V] = f2b(v)
    err = False
    pc = 0
    while True:
        w0, w1 = words[pc], words[pc + 1]
        pc += 2
        op = OPS[w0 & 0xFF]
        d, a, b = (w0 >> 8) & 0xFF, (w0 >> 16) & 0xFF, (w0 >> 24) & 0xFF
        c = w1
        F = lambda r: b2f(R[r])
        I = lambda r: b2i(R[r])
        if op == "RET":
            break
        elif op == "CONST":
            R[d] = consts[c]
        elif op == "MOV":
            R[d] = R[a]
        elif op == "ADDF":
            R[d] = f2b(F(a) + F(b))
        elif op == "SUBF":
            R[d] = f2b(F(a) - F(b))
        elif op == "MULF":
            R[d] = f2b(F(a) * F(b))
        elif op == "DIVF":
            R[d] = f2b(fdiv(F(a), F(b)))
        elif op == "NEGF":
            R[d] = f2b(-F(a))
        elif op == "ADDI":
            R[d] = wrap64(I(a) + I(b)) & ((1 << 64) - 1)
        elif op == "SUBI":
            R[d] = wrap64(I(a) - I(b)) & ((1 << 64) - 1)
        elif op == "MULI":
            R[d] = wrap64(I(a) * I(b)) & ((1 << 64) - 1)
        elif op == "DIVI":
            x, y = I(a), I(b)
            q = 0 if y == 0 else (abs(x) // abs(y)) * (1 if (x < 0) == (y < 0) else -1)
            R[d] = wrap64(q) & ((1 << 64) - 1)
        elif op == "MODI":
            x, y = I(a), I(b)
            r = 0 if y == 0 else (abs(x) % abs(y)) * (1 if x >= 0 else -1)
            R[d] = r & ((1 << 64) - 1)
        elif op == "NEGI":
            R[d] = wrap64(-I(a)) & ((1 << 64) - 1)
        elif op == "LTF":
            R[d] = int(F(a) < F(b))
        elif op == "EQF":
            R[d] = int(F(a) == F(b))
        elif op == "LTI":
            R[d] = int(I(a) < I(b))
        elif op == "EQI":
            R[d] = int(I(a) == I(b))
        elif op == "SEL":
            R[d] = R[b] if R[a] else R[c]
        elif op == "FLOOR":
            x = F(a)
            R[d] = go_f2i(math.floor(x) if math.isfinite(x) else x) & ((1 << 64) - 1)
        elif op == "FRAC":
            x = F(a)
            R[d] = f2b(x - float(go_f2i(x)))
        elif op == "SQRT":
            x = F(a)
            R[d] = f2b(math.sqrt(x) if x >= 0 else math.nan)
        elif op == "SIN":
            R[d] = f2b(gomath.go_sin(DEG_TO_RAD * F(a)))
        elif op == "COS":
            R[d] = f2b(gomath.go_cos(DEG_TO_RAD * F(a)))
        elif op == "CLAMPF":
            x = F(a)
            R[d] = f2b(0.0 if x < 0 else (1.0 if x > 1 else x))
        elif op == "CLAMPI":
            x = I(a)
            R[d] = (0 if x < 0 else (1 if x > 1 else x)) & ((1 << 64) - 1)
        elif op == "TBL":
            n = consts[c]
            i = min(max(I(a), 0), n - 1)
            R[d] = consts[c + 1 + i]
        elif op == "AND":
            R[d] = int(bool(R[a]) and bool(R[b]))
        elif op == "OR":
            R[d] = int(bool(R[a]) or bool(R[b]))
        elif op == "NOT":
            R[d] = int(not R[a])
        elif op == "ERR":
            if R[a]:
                err = True
        else:
            raise ValueError(op)
    return [b2f(R[k]) for k in range(10)], err
