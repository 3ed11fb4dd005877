"""GPU: the CSS permutation kernel (k_css_perm, gd_css_perm.hip) isolated from the
eigen-solver.

The end-to-end p tests (test_css_gpu.py) compare two pipelines whose MDS coordinates X
come from different eigen-solvers (~1e-14 apart), so a permuted score that ties the
observed one to within rounding can flip a hit.  Here the oracle's restatement of
significance_treshold (css.c:727-752; orc_css_perm_from_x) runs on the DEVICE's own X
(gd_css_coords_host), with the same per-window nrand48 stream and identity start
tracks.  Bar: in 100 % of the computed windows, p lies in the oracle's bracket
[p_lo, p_hi], where near ties (within 1e-11 of the score's magnitude: the two sides sum
the same S entries in different orders) are resolved all-miss / all-hit; a window with
no near tie has p_lo == p_hi, so its p must be identical.  Covers every permutation tier
(24, 40, 64, 80, 96, 128), the 64-bit `hi` member branch of the 128 tier, early exits,
full runs, exact-tie-heavy data (duplicated individuals) and the serial window set."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TIE_REL = 1e-11


def _bind(orc):
    C = ctypes
    DP = np.ctypeslib.ndpointer(np.float64, flags="C")
    f = orc.orc_css_perm_from_x
    f.argtypes = [DP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_double, C.POINTER(C.c_double),
                  C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int)]
    f.restype = None
    orc.orc_window_state.argtypes = [C.c_uint64, C.c_uint64, C.c_long]
    orc.orc_window_state.restype = C.c_uint64
    return f


def _oracle_p(orc, X, a, b, treshold, runs, seed, w):
    C = ctypes
    f = _bind(orc)
    sc, p, lo, hi = C.c_double(), C.c_double(), C.c_double(), C.c_double()
    nt = C.c_int()
    f(np.ascontiguousarray(X), a, b, treshold, runs, orc.orc_window_state(seed, 1, w), TIE_REL, C.byref(sc),
      C.byref(p), C.byref(lo), C.byref(hi), C.byref(nt))
    return sc.value, p.value, lo.value, hi.value, nt.value


def _check(orc, a, b, nsnp, treshold, runs, seed, chrom=5, dup=False, serial=False):
    from gdscan import css, synth
    av, bv, ap, bp, regend = synth.chromosome(chrom, nsnp, a, b)
    if dup:  # odd individuals copy their even neighbour: exact ties in every window
        for arr, size in ((av, a), (bv, b)):
            v = arr.reshape(-1, size)
            v[:, 1::2] = v[:, 0:size - 1:2][:, :v[:, 1::2].shape[1]]
    s, p, X = css.scan_coords(av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=seed, serial=serial)
    comp = np.flatnonzero(s != 0)
    assert len(comp) > 20
    inside = exact = ties = 0
    bad = []
    for w in comp:
        sc, p_lit, lo, hi, nt = _oracle_p(orc, X[w], a, b, treshold, runs, seed, int(w))
        # the device's score of the same window came from the same X
        assert abs(sc - s[w]) <= 1e-12 * abs(s[w]) + 1e-12, (w, sc, s[w])
        ok = lo <= p[w] <= hi
        inside += ok
        exact += p[w] == p_lit
        ties += nt > 0
        if not ok:
            bad.append((int(w), p[w], lo, hi, nt))
        if nt == 0:
            assert lo == hi == p_lit
    assert not bad, bad[:10]
    return len(comp), exact, ties


@pytest.mark.parametrize("a,b,nsnp,treshold,runs", [
    (10, 10, 12_000, 10, 300),   # tier 24
    (12, 12, 10_000, 10, 300),   # tier 24 filled (m == MP: the straight-line Fisher-Yates)
    (12, 13, 6_000, 10, 300),    # p40 tier, m = 25
    (16, 17, 6_000, 10, 300),    # m = 33
    (20, 20, 6_000, 50, 400),    # m = 40, full runs and early exits
    (33, 31, 3_000, 10, 200),    # tier 64
    (40, 40, 2_500, 10, 1000),   # tier 80 (the C5 shape)
    (45, 45, 1_800, 10, 150),    # tier 96
    (48, 48, 1_600, 10, 150),    # tier 96 filled (straight-line Fisher-Yates)
    (50, 47, 1_500, 20, 120),    # tier 128, m = 97: the 64-bit hi member word
    (64, 64, 1_400, 10, 100),    # tier 128, m = 128
    (1, 30, 6_000, 10, 300),     # a single individual in A (no within-A pairs)
])
def test_perm_on_device_coordinates(oracle, a, b, nsnp, treshold, runs):
    n, exact, ties = _check(oracle, a, b, nsnp, treshold, runs, seed=77)
    # ordinary data: essentially no near ties, every p identical to the literal decision
    assert exact >= n - ties and ties <= max(1, n // 100), (n, exact, ties)


@pytest.mark.parametrize("a,b,nsnp,runs", [(6, 9, 10_000, 1000), (12, 12, 8_000, 500), (40, 40, 2_500, 500),
                                            (45, 45, 1_800, 200)])
def test_perm_exact_ties(oracle, a, b, nsnp, runs):
    """Duplicated individuals make many permuted scores equal the observed one in exact
    arithmetic: p must still lie inside the tie bracket in every window."""
    _check(oracle, a, b, nsnp, 100_000, runs, seed=5, dup=True)


def test_perm_serial_window_set(oracle):
    _check(oracle, 9, 11, 12_000, 10, 200, seed=9, serial=True)
