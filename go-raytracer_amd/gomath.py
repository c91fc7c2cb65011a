"""Go float64 arithmetic the host side of the path needs, restated in Python.

Python floats are IEEE-754 binary64 with one rounding per operation and no
fused multiply-adds, which is what Go does on amd64 (GOAMD64=v1). Used by the
host-side scene builder for transforms (internal/prim/vec.go:258-268,
376-425) -- the same values the reference's GML evaluator produces.

Third-party algorithms (Go standard library, go 1.24.5 per go.mod:3):
math.Sin / math.Cos (sin.go, Cephes with Cody-Waite reduction).
"""
import math

_SIN = (
    1.58962301576546568060e-10, -2.50507477628578072866e-8,
    2.75573136213857245213e-6, -1.98412698295895385996e-4,
    8.33333333332211858878e-3, -1.66666666666666307295e-1,
)
_COS = (
    -1.13585365213876817300e-11, 2.08757008419747316778e-9,
    -2.75573141792967388112e-7, 2.48015872888517045348e-5,
    -1.38888888888730564116e-3, 4.16666666666665929218e-2,
)
PI4A = 7.85398125648498535156e-1
PI4B = 3.77489470793079817668e-8
PI4C = 2.69515142907905952645e-15
FOUR_OVER_PI = 1.2732395447351628  # Go const 4/Pi, rounded once
REDUCE_THRESHOLD = float(1 << 29)


def _poly_sin(z, zz):
    return z + z * zz * ((((((_SIN[0] * zz) + _SIN[1]) * zz + _SIN[2]) * zz + _SIN[3]) * zz + _SIN[4]) * zz + _SIN[5])


def _poly_cos(zz):
    return 1.0 - 0.5 * zz + zz * zz * ((((((_COS[0] * zz) + _COS[1]) * zz + _COS[2]) * zz + _COS[3]) * zz + _COS[4]) * zz + _COS[5])


def go_sin(x):
    """math.Sin (sin.go)."""
    if x == 0 or math.isnan(x):
        return x
    if math.isinf(x):
        return math.nan
    if abs(x) >= REDUCE_THRESHOLD:
        raise ValueError("go_sin: Payne-Hanek range not restated")
    sign = False
    if x < 0:
        x = -x
        sign = True
    j = int(x * FOUR_OVER_PI)
    y = float(j)
    if j & 1 == 1:
        j += 1
        y += 1
    j &= 7
    z = ((x - y * PI4A) - y * PI4B) - y * PI4C
    if j > 3:
        sign = not sign
        j -= 4
    zz = z * z
    if j == 1 or j == 2:
        y = _poly_cos(zz)
    else:
        y = _poly_sin(z, zz)
    return -y if sign else y


def go_cos(x):
    """math.Cos (sin.go)."""
    if math.isnan(x) or math.isinf(x):
        return math.nan
    if abs(x) >= REDUCE_THRESHOLD:
        raise ValueError("go_cos: Payne-Hanek range not restated")
    sign = False
    x = abs(x)
    j = int(x * FOUR_OVER_PI)
    y = float(j)
    if j & 1 == 1:
        j += 1
        y += 1
    j &= 7
    z = ((x - y * PI4A) - y * PI4B) - y * PI4C
    if j > 3:
        j -= 4
        sign = not sign
    if j > 1:
        sign = not sign
    zz = z * z
    if j == 1 or j == 2:
        y = _poly_sin(z, zz)
    else:
        y = _poly_cos(zz)
    return -y if sign else y


# ---- prim.Mat4 (internal/prim/vec.go:256-425) -----------------------------

def identity():
    return [[1.0, 0.0, 0.0, 0.0], [0.0, 1.0, 0.0, 0.0], [0.0, 0.0, 1.0, 0.0], [0.0, 0.0, 0.0, 1.0]]


def mul_mat(m, n):
    """Mat4.MulMat (vec.go:258-268): product[i][j] += m[i][k]*n[k][j], k=0..3 from 0."""
    p = [[0.0] * 4 for _ in range(4)]
    for i in range(4):
        for j in range(4):
            acc = 0.0
            for k in range(4):
                acc += m[i][k] * n[k][j]
            p[i][j] = acc
    return p


def translate(x, y, z):
    """Mat4Translate (vec.go:376-383)."""
    return [[1.0, 0.0, 0.0, x], [0.0, 1.0, 0.0, y], [0.0, 0.0, 1.0, z], [0.0, 0.0, 0.0, 1.0]]


def scale(x, y, z):
    """Mat4Scale (vec.go:385-392)."""
    return [[x, 0.0, 0.0, 0.0], [0.0, y, 0.0, 0.0], [0.0, 0.0, z, 0.0], [0.0, 0.0, 0.0, 1.0]]


def rotate_x(angle):
    """Mat4RotateX (vec.go:394-403), angle in radians."""
    c, s = go_cos(angle), go_sin(angle)
    return [[1.0, 0.0, 0.0, 0.0], [0.0, c, -s, 0.0], [0.0, s, c, 0.0], [0.0, 0.0, 0.0, 1.0]]


def rotate_y(angle):
    """Mat4RotateY (vec.go:405-414)."""
    c, s = go_cos(angle), go_sin(angle)
    return [[c, 0.0, s, 0.0], [0.0, 1.0, 0.0, 0.0], [-s, 0.0, c, 0.0], [0.0, 0.0, 0.0, 1.0]]


def rotate_z(angle):
    """Mat4RotateZ (vec.go:416-425)."""
    c, s = go_cos(angle), go_sin(angle)
    return [[c, -s, 0.0, 0.0], [s, c, 0.0, 0.0], [0.0, 0.0, 1.0, 0.0], [0.0, 0.0, 0.0, 1.0]]


def deg_to_rad(angle):
    """The GML rotate builtins' conversion: angle * math.Pi / 180 (evaluator.go:1052)."""
    return angle * math.pi / 180
