"""FET exact mode: the reference's tail algorithm (cFisher.c:405-455)
over table probabilities from ln k! instead of the u64 binomials of fet_p (cFisher.c:473-483),
which overflow from C(68, 31) on (the reference then divides by 0 or by a wrapped product).

Parity is not against the reference (it has no exact mode) but against two independent
computations: the oracle's long-double lgammal restatement and scipy's hypergeometric pmf.
Both follow the walk in exact rational arithmetic to 1e-12 relative (tests below); where the
u64 path overflows, exact mode stays finite, in (0, 1], and matches the oracle."""
import ctypes

import numpy as np
import pytest

from conftest import close, oracle_fet_scan

SHIM_EXACT = ("shim_fet_exact", "shim_fet_p_exact", "shim_score_exact")


@pytest.fixture(scope="module")
def ex(shim, oracle):
    C = ctypes
    for fn in SHIM_EXACT:
        getattr(shim, fn).argtypes = [C.c_int] * 4
        getattr(shim, fn).restype = C.c_double
    oracle.orc_set_fet_mode.argtypes = [C.c_int]
    oracle.orc_set_fet_mode.restype = C.c_int
    return shim, oracle


def _oracle_exact(orc, fn, *args):
    old = orc.orc_set_fet_mode(1)
    try:
        return fn(*args)
    finally:
        orc.orc_set_fet_mode(old)


def _tables(rng, n, nmax):
    out = []
    while len(out) < n:
        N = int(rng.integers(1, nmax + 1))
        cuts = np.sort(rng.integers(0, N + 1, 3))
        out.append((int(cuts[0]), int(cuts[1] - cuts[0]), int(cuts[2] - cuts[1]), int(N - cuts[2])))
    return out


# ---------------------------------------------------------------- CPU
def test_table_p_matches_scipy_hypergeom(ex):
    from scipy.stats import hypergeom
    shim, _ = ex
    rng = np.random.default_rng(1)
    for a, b, c, d in _tables(rng, 400, 255):
        want = hypergeom.pmf(a, a + b + c + d, a + c, a + b)
        got = shim.shim_fet_p_exact(a, b, c, d)
        assert got == pytest.approx(want, rel=1e-10, abs=1e-300), (a, b, c, d)


def test_table_p_matches_oracle_long_double(ex):
    shim, orc = ex
    rng = np.random.default_rng(2)
    for t in _tables(rng, 2000, 255):
        want = _oracle_exact(orc, orc.orc_fet_p, *t)
        assert shim.shim_fet_p_exact(*t) == pytest.approx(want, rel=1e-13, abs=1e-300), t


def _fet_rational(a, b, c, d):
    """The reference's two-tailed walk (fet, cFisher.c:405-455) in exact rational arithmetic:
    the p-value the u64 and the ln k! evaluations both approximate (ties compare equal)."""
    from fractions import Fraction
    from math import comb

    def table_p(f):
        return Fraction(comb(f[0] + f[1], f[0]) * comb(f[2] + f[3], f[2]), comb(sum(f), f[0] + f[2]))

    def min_to_a(f):
        ring = [f[0], f[1], f[3], f[2]]
        s = ring.index(min(ring))
        r = [ring[(s + i) % 4] for i in range(4)]
        return [r[0], r[1], r[3], r[2]]

    def opposite(f):
        R1, R2, C1, C2 = f[0] + f[1], f[2] + f[3], f[0] + f[2], f[1] + f[3]
        m = min(R1, R2, C1, C2)
        f = list(f)
        if R1 <= R2 and C1 <= C2:
            f[0] = m - f[0]; f[1] = R1 - f[0]; f[2] = C1 - f[0]; f[3] = C2 - f[1]
        elif R1 <= R2 and C2 <= C1:
            f[1] = m - f[1]; f[0] = R1 - f[1]; f[3] = C2 - f[1]; f[2] = C1 - f[0]
        elif R1 >= R2 and C1 <= C2:
            f[2] = m - f[2]; f[0] = C1 - f[2]; f[3] = R2 - f[2]; f[1] = R1 - f[0]
        else:
            f[3] = m - f[3]; f[1] = C2 - f[3]; f[2] = R2 - f[3]; f[0] = R1 - f[1]
        return f

    tie = (a + b == c + d) or (a + c == b + d)
    f = min_to_a([a, b, c, d])
    p0 = table_p(f)
    tot = p0
    while f[0] > 0:
        f = [f[0] - 1, f[1] + 1, f[2] + 1, f[3] - 1]
        tot += table_p(f)
    if tie:
        tot *= 2
    else:
        f = min_to_a(opposite(f))
        far = table_p(f)
        while far < p0:
            tot += far
            if f[1] == 0 or f[2] == 0:
                break
            f = [f[0] + 1, f[1] - 1, f[2] - 1, f[3] + 1]
            far = table_p(f)
    return float(min(tot, 1))


def test_exact_matches_rational_walk(ex):
    """Tables of two groups of <= 20 (where the u64 path does not overflow either) and random
    tables up to 255 individuals: exact mode equals the walk in rational arithmetic.  (Reference
    mode can differ where a far-tail table ties the observed one: its recurrence rounds the tie
    either way.)"""
    shim, _ = ex
    tables = [(a, b, c, (B - c) // 2) for A in (1, 7, 20) for B in (1, 13, 20)
              for a in range(A + 1) for b in range(A - a + 1) for c in range(B + 1)]
    tables += _tables(np.random.default_rng(5), 300, 255)
    agree_ref = 0
    for t in tables:
        want = _fet_rational(*t)
        assert shim.shim_fet_exact(*t) == pytest.approx(want, rel=1e-12), t
        if sum(t) <= 40:
            agree_ref += shim.shim_fet(*t) == pytest.approx(want, rel=1e-12)
    small = sum(sum(t) <= 40 for t in tables)
    assert agree_ref >= 0.95 * small  # reference mode: all but the rounded ties


def test_exact_finite_where_reference_overflows(ex):
    shim, orc = ex
    cases = [(31, 37, 0, 0), (40, 0, 0, 40), (50, 10, 10, 50), (35, 35, 30, 40), (20, 20, 20, 20),
             (60, 60, 60, 60), (100, 27, 50, 78)]
    wrong = 0
    for t in cases:
        want = _oracle_exact(orc, orc.orc_fet, *t)
        got = shim.shim_fet_exact(*t)
        assert np.isfinite(got) and 0 < got <= 1, (t, got)
        assert got == pytest.approx(want, rel=1e-12), t
        ref = orc.orc_fet(*t)
        wrong += not (np.isfinite(ref) and abs(ref - want) <= 1e-6 * want)
    assert wrong >= 3  # reference mode really does break on these tables


def test_exact_p_value_known_answers(ex):
    """Symmetric margins: the reference's doubled near tail is the textbook two-sided p, so
    scipy's fisher_exact is a known answer."""
    from scipy.stats import fisher_exact
    shim, _ = ex
    for a, b, c, d in [(3, 1, 1, 3), (10, 2, 2, 10), (40, 5, 5, 40), (70, 30, 30, 70)]:
        want = fisher_exact([[a, b], [c, d]])[1]
        assert shim.shim_fet_exact(a, b, c, d) == pytest.approx(want, rel=1e-9), (a, b, c, d)


def test_exact_score_matches_oracle(ex):
    shim, orc = ex
    rng = np.random.default_rng(4)
    for t in _tables(rng, 500, 160):
        want = _oracle_exact(orc, orc.orc_fet_score, *t)
        assert shim.shim_score_exact(*t) == pytest.approx(want, rel=1e-12, abs=1e-12), t


# ---------------------------------------------------------------- GPU
def _synth(c, nsnp, a, b):
    from gdscan import synth
    return synth.chromosome(c, nsnp, a, b)


def _oracle_scan_exact(orc, av, bv, ap, bp, regend, seed):
    old = orc.orc_set_fet_mode(1)
    try:
        return oracle_fet_scan(orc, av, bv, ap, bp, regend, seed=seed)
    finally:
        orc.orc_set_fet_mode(old)


@pytest.mark.gpu
@pytest.mark.parametrize("a,b,nsnp", [(40, 40, 30_000), (34, 50, 25_000), (10, 10, 30_000)])
def test_exact_scan_matches_oracle(ex, a, b, nsnp):
    from gdscan import fet
    _, orc = ex
    av, bv, ap, bp, regend = _synth(120 + a, nsnp, a, b)
    s, d = fet.scan(av, bv, ap, bp, regend, seed=9, exact=True)
    s_ref, d_ref = _oracle_scan_exact(orc, av, bv, ap, bp, regend, 9)
    assert (s_ref != 0).sum() > 50
    assert np.all(np.isfinite(s[s_ref != 0]))
    assert close(s, s_ref) and close(d, d_ref)


@pytest.mark.gpu
def test_exact_mode_agrees_with_reference_mode_below_overflow():
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(130, 30_000, 12, 12)
    s0, d0 = fet.scan(av, bv, ap, bp, regend, seed=3)
    s1, d1 = fet.scan(av, bv, ap, bp, regend, seed=3, exact=True)
    ok = np.isclose(s1, s0, rtol=1e-12, atol=0) & np.isclose(d1, d0, rtol=1e-12, atol=1e-13)
    assert ok.mean() >= 0.9  # the rest hold a SNP whose far tail ties (see test_exact_matches_rational_walk)
    # the device score table is cached per (asize, bsize, mode): switching back is exact
    s2, d2 = fet.scan(av, bv, ap, bp, regend, seed=3)
    assert np.array_equal(s2, s0) and np.array_equal(d2, d0)


@pytest.mark.gpu
def test_reference_entry_point_follows_global_mode(ex):
    """gd_set_fet_mode switches the reference-signature entry points (fisher_exact_tester)."""
    import fisher_cython_parallel as fcp
    from gdscan import fet, lib
    from gdscan._lib import GD_ERR_ARG
    _, orc = ex
    av, bv, ap, bp, regend = _synth(131, 25_000, 40, 40)
    lib.gd_set_seed(20261015)
    n = regend // 500
    out_ref = (np.zeros(n), np.zeros(n))
    fcp.fisher_exact_tester(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 0.95, *out_ref)
    assert fet.set_mode(exact=True) is False
    try:
        out_ex = (np.zeros(n), np.zeros(n))
        fcp.fisher_exact_tester(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 0.95, *out_ex)
    finally:
        assert fet.set_mode(exact=False) is True
    s_ref, d_ref = _oracle_scan_exact(orc, av, bv, ap, bp, regend, 20261015)
    assert close(out_ex[0], s_ref) and close(out_ex[1], d_ref)
    assert not np.array_equal(out_ex[0], out_ref[0])  # 40+40 tables overflow in reference mode
    assert lib.gd_set_fet_mode(7) == GD_ERR_ARG
    assert lib.gd_get_fet_mode() == 0
