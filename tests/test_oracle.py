"""The CPU oracle against the reference's own golden vectors and KATs.

Pins (reference files):
  testdata/goldens/example_canned.png   raytracer_test.go:71-77 (canned.gml)
  cylinder_test.go:21-165               Cylinder Intersect / normal KATs
The reference's bar is SSIM >= 0.99 (raytracer_test.go:42); ours is exact bytes.
"""
import ctypes as C
import math
import os

import numpy as np
import pytest
from PIL import Image

import go_raytracer_amd as rt
import oracle_bind

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load_golden(name):
    return np.asarray(Image.open(os.path.join(GOLDEN, name)).convert("RGB"))


def test_oracle_matches_canned_golden_exactly():
    packed = rt.scene.convert(rt.configs.canned())
    img, st = oracle_bind.render_rows(packed, threads=8)
    gold = load_golden("example_canned.png")
    assert img.shape[:2] == gold.shape[:2]
    assert (img[..., 3] == 255).all()
    diff = img[..., :3] != gold
    assert int(diff.sum()) == 0, "oracle differs from example_canned.png in %d channels" % int(diff.sum())
    assert st.primary_rays == 4 * 1900 * 1200


def test_oracle_row_band_equals_full_frame():
    packed = rt.scene.convert(rt.configs.canned(width=190, height=120))
    full, _ = oracle_bind.render_rows(packed)
    for y0, y1 in [(0, 13), (13, 47), (47, 120), (33, 34)]:
        band, _ = oracle_bind.render_rows(packed, y0, y1)
        assert np.array_equal(band, full[y0:y1])


def test_oracle_thread_count_invariant():
    packed = rt.scene.convert(rt.configs.c2(width=96, height=54))
    a, sa = oracle_bind.render_rows(packed, threads=1)
    b, sb = oracle_bind.render_rows(packed, threads=8)
    assert np.array_equal(a, b)
    assert sa.as_dict() == sb.as_dict()


def _identity_cylinder_scene():
    args = rt.scene.RenderArgs(ambient=(0, 0, 0), lights=[], scene=rt.scene.Cylinder(rt.scene.Material()),
                               depth=1, fov=90.0, width=4, height=4)
    return rt.scene.convert(args)


def _intersect(packed, origin, direction):
    t = C.c_double()
    p = (C.c_double * 3)()
    f = C.c_int()
    ok = oracle_bind.lib().oracle_intersect(C.addressof(packed.scene), 0, (C.c_double * 3)(*origin),
                                           (C.c_double * 3)(*direction), C.byref(t), p, C.byref(f))
    return (ok == 1), t.value, tuple(p), f.value


# cylinder_test.go:21-114
@pytest.mark.parametrize("origin,direction,face,t,point", [
    ((-2, 0.5, 0), (1, 0, 0), 0, 1.0, (-1, 0.5, 0)),     # TestCylinderIntersectSide
    ((0, 2, 0), (0, -1, 0), 1, 1.0, None),               # TestCylinderIntersectTopCap
    ((0, -2, 0), (0, 1, 0), 2, 2.0, None),               # TestCylinderIntersectBottomCap
    ((0, 0.5, 0), (0, 1, 0), 1, 0.5, None),              # ...FromInsideHitsNearestCap
])
def test_cylinder_intersect_kats(origin, direction, face, t, point):
    ok, tt, p, f = _intersect(_identity_cylinder_scene(), origin, direction)
    assert ok and f == face and abs(tt - t) <= 1e-9
    if point is not None:
        assert math.dist(p, point) <= 1e-9


@pytest.mark.parametrize("origin,direction", [
    ((5, -1, 0), (0, 1, 0)), ((-2, 5, 0), (1, 0, 0)),   # TestCylinderIntersectMiss
    ((2, 0.5, 0), (1, 0, 0)),                           # TestCylinderIntersectBehindRay
])
def test_cylinder_intersect_misses(origin, direction):
    ok, _, _, _ = _intersect(_identity_cylinder_scene(), origin, direction)
    assert not ok


# cylinder_test.go:116-165
@pytest.mark.parametrize("face,point,normal", [
    (0, (1, 0.5, 0), (1, 0, 0)), (1, (0.2, 1, 0.3), (0, 1, 0)), (2, (0.2, 0, 0.3), (0, -1, 0)),
])
def test_cylinder_normals(face, point, normal):
    packed = _identity_cylinder_scene()
    nw = (C.c_double * 3)()
    pw = (C.c_double * 3)()
    rc = oracle_bind.lib().oracle_surface_normal(C.addressof(packed.scene), 0, face, (C.c_double * 3)(*point), nw, pw)
    assert rc == 0 and math.dist(tuple(nw), normal) <= 1e-9


def test_cylinder_invalid_face_is_an_error():
    packed = _identity_cylinder_scene()
    nw = (C.c_double * 3)()
    pw = (C.c_double * 3)()
    rc = oracle_bind.lib().oracle_surface_normal(C.addressof(packed.scene), 0, 99, (C.c_double * 3)(0, 0, 0), nw, pw)
    assert rc != 0


def test_go_pow_integer_exponents_match_repeated_squaring():
    l = oracle_bind.lib()
    assert l.oracle_go_pow(0.0, 50.0) == 0.0
    assert l.oracle_go_pow(0.3, 0.0) == 1.0
    assert l.oracle_go_pow(0.3, 1.0) == 0.3
    assert l.oracle_go_pow(0.5, 5.0) == 0.03125
    x = 0.987654321
    assert abs(l.oracle_go_pow(x, 50.0) - x ** 50) <= 4e-16


def _ulps(a, b):
    ia = int(np.array(a).view(np.int64))
    ib = int(np.array(b).view(np.int64))
    return abs(ia - ib)


def test_go_exp_log_restatement():
    """math.Exp / math.Log (Go exp.go, log.go; the fractional branch of
    math.Pow): special cases, exact points, and within 1 ulp of libm (both
    algorithms are < 1 ulp; bit-exactness with the device is tests/hip/pow_check)."""
    l = oracle_bind.lib()
    assert l.oracle_go_exp(0.0) == 1.0 and l.oracle_go_log(1.0) == 0.0
    assert l.oracle_go_exp(float("-inf")) == 0.0 and l.oracle_go_exp(float("inf")) == float("inf")
    assert l.oracle_go_exp(710.0) == float("inf") and l.oracle_go_exp(-746.0) == 0.0
    assert math.isnan(l.oracle_go_exp(float("nan"))) and math.isnan(l.oracle_go_log(-1.0))
    assert l.oracle_go_log(0.0) == float("-inf") and l.oracle_go_log(float("inf")) == float("inf")
    assert l.oracle_go_exp(1e-9) == 1.0 + 1e-9  # |x| < 2^-28: 1 + x
    assert l.oracle_go_log(2.0) == 0.6931471805599453 and l.oracle_go_log(0.5) == -0.6931471805599453
    rng = np.random.default_rng(5)
    for x in rng.uniform(-700, 700, 20000):
        assert _ulps(l.oracle_go_exp(x), math.exp(x)) <= 1, x
    for x in np.exp(rng.uniform(-700, 700, 20000)):
        assert _ulps(l.oracle_go_log(x), math.log(x)) <= 1, x
    for x in np.concatenate([rng.uniform(0, 1, 5000), [5e-324, 1e-310, 0.7071067811865476, 1 - 2 ** -53]]):
        assert _ulps(l.oracle_go_log(x), math.log(x)) <= 1, x


def test_go_exp_amd64_restatement():
    """math.Exp as Go runs it on amd64 (exp_amd64.s, with and without FMA;
    recalled): special cases, overflow / underflow thresholds,
    within 4 ulp of libm, and genuinely different from the portable exp.go in
    the last bit of a sizeable share of inputs -- which is why the platform
    is a scene option (rt_scene.exp_mode)."""
    l = oracle_bind.lib()
    for f in (0, 1):
        e = lambda x: l.oracle_go_exp_amd64(x, f)  # noqa: E731
        assert e(0.0) == 1.0 and e(float("-inf")) == 0.0 and e(float("inf")) == float("inf")
        assert math.isnan(e(float("nan"))) and e(709.79) == float("inf") and e(-1e10) == 0.0
        assert e(-745.0) == 5e-324 and e(-740.0) == 4.2e-322  # the two-factor denormal path
        # biased exponent exactly 0 (e = -1023) takes the denormal path too
        # (exp_amd64.s branches with JLE): a subnormal within 4 ulp, not 0
        for x in (-709.5, -709.2, -709.7):
            assert 0.0 < e(x) < 2.2250738585072014e-308 and _ulps(e(x), math.exp(x)) <= 4, x
        rng = np.random.default_rng(7 + f)
        for x in rng.uniform(-700, 700, 20000):
            assert _ulps(e(x), math.exp(x)) <= 4, x
    rng = np.random.default_rng(11)
    xs = rng.uniform(-30, 30, 20000)
    fma_vs_plain = sum(l.oracle_go_exp_amd64(x, 1) != l.oracle_go_exp_amd64(x, 0) for x in xs)
    amd64_vs_portable = sum(l.oracle_go_exp_amd64(x, 1) != l.oracle_go_exp(x) for x in xs)
    assert 0 < fma_vs_plain < 0.05 * len(xs) and amd64_vs_portable > 0.1 * len(xs)
    # log_amd64.s: log.go's algorithm (bit-level Frexp: equal for normal inputs)
    for x in np.exp(rng.uniform(-700, 700, 5000)):
        assert l.oracle_go_log_amd64(x) == l.oracle_go_log(x), x


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_go_pow_modes(mode):
    """Pow with each platform's Exp / Log: integer exponents never reach
    Exp (identical in every mode); fractional ones stay within Pow's error."""
    l = oracle_bind.lib()
    rng = np.random.default_rng(mode)
    for x in rng.uniform(1e-3, 1.0, 2000):
        for y in (2.0, 5.0, 40.0):
            assert l.oracle_go_pow_mode(x, y, mode) == l.oracle_go_pow(x, y)
        got, want = l.oracle_go_pow_mode(x, 7.3, mode), x ** 7.3
        assert abs(got - want) <= 64 * abs(want) * 2.0 ** -52, (x, got, want)


@pytest.mark.parametrize("y", [0.5, 2.5, 7.3, 33.3, -1.5, 0.75])
def test_go_pow_fractional_exponents(y):
    """Pow's fractional part: yf > 0.5 folds to yf - 1 (yi + 1), then
    Exp(yf * Log(x)) times the repeated-squaring integer part."""
    l = oracle_bind.lib()
    rng = np.random.default_rng(int(y * 100) & 0xffff)
    for x in rng.uniform(1e-3, 1.0, 3000):
        got, want = l.oracle_go_pow(x, y), x ** y
        assert abs(got - want) <= 64 * abs(want) * 2.0 ** -52, (x, y, got, want)  # not correctly rounded
    assert math.isnan(l.oracle_go_pow(-0.5, y))
    assert l.oracle_go_pow(1.0, y) == 1.0


def test_go_tan_matches_libm_closely():
    l = oracle_bind.lib()
    for deg in (30.0, 45.0, 60.0, 89.0):
        x = deg * math.pi / 180.0
        assert abs(l.oracle_go_tan(x) - math.tan(x)) <= 2e-16 * max(1.0, abs(math.tan(x)))


def test_host_gomath_sin_cos_equal_oracle():
    from go_raytracer_amd import gomath
    l = oracle_bind.lib()
    rng = np.random.default_rng(3)
    for x in rng.uniform(-20, 20, 2000):
        x = float(x)
        assert gomath.go_sin(x) == l.oracle_go_sin(x)
        assert gomath.go_cos(x) == l.oracle_go_cos(x)
