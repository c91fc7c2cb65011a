"""The diagonal rayToObjectSpace of scale + translation spheres (rt_render.h
axis_o / axis_d, used by the brute-force sphere runs) against the full
MulPoint / MulDir (reference internal/prim/vec.go:298-313, raytracer.go:51-56),
bit for bit, on the inputs the kernel admits (axis_sphere on the host,
axis_o_ok / axis_d_ok per ray): random values, signed zeros in every
off-diagonal slot and ray component, and magnitudes at the admitted range's
edges. IEEE float64 in numpy rounds every operation once (no contraction), as
Go does on amd64 and the kernel does with -ffp-contract=off."""
import numpy as np


def _full_point(m, o):
    # ((m0*x + m1*y) + m2*z) + m3, per row (vec.go:298-304)
    return np.stack([((m[:, 4 * r] * o[:, 0] + m[:, 4 * r + 1] * o[:, 1]) + m[:, 4 * r + 2] * o[:, 2]) + m[:, 4 * r + 3]
                     for r in range(3)], axis=1)


def _full_dir(m, d):
    # (m0*x + m1*y) + m2*z, per row (vec.go:307-313)
    return np.stack([(m[:, 4 * r] * d[:, 0] + m[:, 4 * r + 1] * d[:, 1]) + m[:, 4 * r + 2] * d[:, 2]
                     for r in range(3)], axis=1)


def _diag(m, v, point):
    out = np.stack([m[:, 0] * v[:, 0], m[:, 5] * v[:, 1], m[:, 10] * v[:, 2]], axis=1)
    if point:
        out = np.stack([out[:, 0] + m[:, 3], out[:, 1] + m[:, 7], out[:, 2] + m[:, 11]], axis=1)
    return out


def _ax_mag(x, zero_ok):
    """rt_render.h ax_mag: |x| in [2^-900, 2^900), or +-0 when zero_ok."""
    e = (x.view(np.uint64) >> np.uint64(52)) & np.uint64(0x7FF)
    ok = (e.astype(np.int64) - 123 >= 0) & (e.astype(np.int64) - 123 < 1800)
    return ok | (zero_ok & (x == 0.0))


def _axis_sphere(m):
    """rt_kernel.hip axis_sphere."""
    ok = np.ones(len(m), bool)
    for q in (1, 2, 4, 6, 8, 9):
        ok &= m[:, q] == 0.0
    for q in (0, 5, 10):
        a = np.abs(m[:, q])
        ok &= (a >= 2.0 ** -100) & (a <= 2.0 ** 100)
    for q in (3, 7, 11):
        ok &= np.isfinite(m[:, q]) & (m[:, q] != 0.0)
    return ok


def _values(rng, n, zeros):
    """Random magnitudes over the admitted range and its edges, random signs."""
    kind = rng.integers(0, 6, n)
    mag = np.where(kind == 0, 10.0 ** rng.uniform(-3, 3, n),
          np.where(kind == 1, 2.0 ** rng.uniform(-900, 899.99, n),
          np.where(kind == 2, 2.0 ** -900 * (1 + rng.uniform(0, 1e-3, n)),
          np.where(kind == 3, 2.0 ** 900 * (1 - rng.uniform(1e-12, 1e-3, n)),
          np.where(kind == 4, rng.uniform(0, 1, n), 1.0)))))
    v = mag * np.where(rng.integers(0, 2, n) == 1, -1.0, 1.0)
    if zeros:
        z = rng.integers(0, 5, n) == 0
        v = np.where(z, np.where(rng.integers(0, 2, n) == 1, -0.0, 0.0), v)
    return v


def _matrices(rng, n):
    m = np.zeros((n, 12))
    for q in (1, 2, 4, 6, 8, 9):  # signed zeros in every off-diagonal slot
        m[:, q] = np.where(rng.integers(0, 2, n) == 1, -0.0, 0.0)
    for q in (0, 5, 10):
        kind = rng.integers(0, 4, n)
        a = np.where(kind == 0, 2.0 ** rng.uniform(-100, 100, n),
            np.where(kind == 1, 2.0 ** -100, np.where(kind == 2, 2.0 ** 100, 1.0 / rng.uniform(0.01, 2, n))))
        m[:, q] = a * np.where(rng.integers(0, 2, n) == 1, -1.0, 1.0)
    for q in (3, 7, 11):
        m[:, q] = rng.uniform(-20, 20, n) * 10.0 ** rng.integers(-5, 5, n)
    return m


def test_diagonal_transform_equals_full_form():
    rng = np.random.default_rng(2026)
    n = 400_000
    m = _matrices(rng, n)
    assert _axis_sphere(m).all()
    o = np.stack([_values(rng, n, True) for _ in range(3)], axis=1)
    d = np.stack([_values(rng, n, False) for _ in range(3)], axis=1)
    ok = _ax_mag(o, True).all(axis=1) & _ax_mag(d, False).all(axis=1)
    assert ok.mean() > 0.9
    m, o, d = m[ok], o[ok], d[ok]
    with np.errstate(all="ignore"):
        fo, go = _full_point(m, o), _diag(m, o, True)
        fd, gd = _full_dir(m, d), _diag(m, d, False)
    assert np.array_equal(fo.view(np.uint64), go.view(np.uint64))
    assert np.array_equal(fd.view(np.uint64), gd.view(np.uint64))
    # the cases the argument singles out were drawn
    assert (o == 0.0).any() and (np.signbit(o) & (o == 0.0)).any()
    assert (np.abs(d) < 2.0 ** -899).any() and (np.abs(d) > 2.0 ** 899).any()


def test_admission_rules_reject_the_counterexamples():
    """What the predicates keep out does break the diagonal form: a zero
    direction component (signed-zero sums), a zero translation (signed-zero
    sums), a product that underflows, and non-finite components (0 * inf)."""
    m = np.zeros((1, 12))
    m[0, 0] = m[0, 5] = m[0, 10] = 1.0
    m[0, 3] = m[0, 7] = m[0, 11] = 1.0
    m[0, 1] = 0.0
    # zero direction component: -0 from the diagonal, +0 from the full sum
    d = np.array([[-0.0, 1.0, 1.0]])
    assert not _ax_mag(d, False).all()
    assert np.signbit(_diag(m, d, False)[0, 0]) != np.signbit(_full_dir(m, d)[0, 0])
    # zero translation: the full row's sign of zero can differ
    m2 = m.copy()
    m2[0, 3] = -0.0
    assert not _axis_sphere(m2).all()
    o = np.array([[-0.0, 1.0, 1.0]])
    assert np.signbit(_diag(m2, o, True)[0, 0]) != np.signbit(_full_point(m2, o)[0, 0])
    # tiny components are outside [2^-900, 2^900)
    assert not _ax_mag(np.array([2.0 ** -1000]), True).all()
    assert not _ax_mag(np.array([np.inf]), True).all() and not _ax_mag(np.array([np.nan]), True).all()
    with np.errstate(all="ignore"):
        inf = np.array([[1.0, np.inf, 1.0]])
        assert np.isnan(_full_dir(m, inf)[0, 0]) and not np.isnan(_diag(m, inf, False)[0, 0])
