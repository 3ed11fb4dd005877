"""The CSS options beside classical MDS on the count metric:
SMACOF (mds = 1: smacof_runs, css.c:807-835; mds = 2: classical MDS refined by one
SMACOF run, css.c:211-213) and the drosophila allele-frequency metric (compare_freq,
css.c:245-264).

CPU: the oracle restatement (oracle/css_options_oracle.c) against testcss.c's known
answers.  GPU: the HIP path through the C ABI against the oracle.  SMACOF runs in the
reference's evaluation order on both sides, so mds = 1 scores are compared at 1e-9
relative (in practice bit-identical); mds = 2 starts from the classical coordinates,
whose eigen-solvers differ by ~1e-14, and a start that close can still end one
SMACOF iteration apart when the stress decrease sits at the 1e-6 exit threshold, so
mds = 2 is held to 1e-9 on >= 98% of windows and 1e-4 on all."""
import ctypes

import numpy as np
import pytest

from conftest import DP, IP

F64 = np.ctypeslib.ndpointer(np.float64, flags="C")


@pytest.fixture(scope="module")
def opt(oracle):
    C = ctypes
    oracle.orc_css_compare_freq.argtypes = [F64, F64, C.c_int, F64]
    oracle.orc_css_stress.argtypes = [F64, F64, C.c_int]
    oracle.orc_css_stress.restype = C.c_double
    oracle.orc_css_smacof.argtypes = [F64, C.c_int, F64, C.c_int, C.c_double, C.POINTER(C.c_int)]
    oracle.orc_css_smacof.restype = C.c_double
    oracle.orc_css_scan_ex.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, DP, DP]
    return oracle


def oracle_scan_ex(orc, av, bv, ap, bp, regend, drosophila, mds, treshold=10, runs=0, seed=20261015, serial=False):
    n = regend // 500
    s, p = np.zeros(n), np.zeros(n)
    rc = orc.orc_css_scan_ex(av, bv, ap, bp, regend, 2500, 500, len(av), len(bv), treshold, runs, drosophila, mds,
                             seed, int(serial), s, p)
    assert rc == 0
    return s, p


def assert_smacof2_mismatches_are_start_effects(orc, av, bv, ap, bp, regend, a, b, s_dev, s_ref, serial=False):
    """mds 2 runs SMACOF from the classical coordinates (css.c:208-218).  The device's and
    the oracle's classical coordinates come from different eigen-solvers (~1e-14 apart),
    and a start that close can end one iteration apart at the 1e-6 exit test.  Every window
    whose score misses the oracle's by more than 1e-9 must therefore equal, to 1e-9, the
    oracle's SMACOF (css.c:767-938) re-run from the DEVICE's classical coordinates
    (scan_coords, mds 0).  Returns the number of such windows."""
    from gdscan import css
    from conftest import window_slices
    ok = (np.abs(s_dev - s_ref) <= 1e-9 * np.abs(s_ref) + 1e-12) | (np.isnan(s_dev) & np.isnan(s_ref))
    bad = np.flatnonzero(~ok)
    if bad.size == 0:
        return 0
    _, _, X0 = css.scan_coords(av, bv, ap, bp, regend, runs=0, serial=serial)
    sl = window_slices(ap, bp, regend, a, b, serial=serial)
    C = ctypes
    orc.orc_css_compare_all.argtypes = [F64, F64, C.c_int, C.c_int, C.c_int, F64]
    orc.orc_css_fill_averages.argtypes = [F64, C.c_int]
    orc.orc_css_dist.argtypes = [F64, C.c_int, F64]
    orc.orc_css_score.argtypes = [F64, C.c_int, np.ctypeslib.ndpointer(np.int32, flags="C"),
                                  np.ctypeslib.ndpointer(np.int32, flags="C"), C.c_int, C.c_int]
    orc.orc_css_score.restype = C.c_double
    m = a + b
    out = []
    for w in bad:
        la0, lb0, npos = sl[int(w)]
        D = np.zeros(m * m)
        orc.orc_css_compare_all(np.ascontiguousarray(av[la0:la0 + npos * a]),
                                np.ascontiguousarray(bv[lb0:lb0 + npos * b]), a, b, npos, D)
        assert orc.orc_css_fill_averages(D, m)
        X = np.ascontiguousarray(X0[w].reshape(-1))
        it = C.c_int()
        orc.orc_css_smacof(D, m, X, 300, 0.000001, C.byref(it))
        S = np.zeros(m * m)
        orc.orc_css_dist(X, m, S)
        sc = orc.orc_css_score(S, m, np.arange(a, dtype=np.int32), np.arange(a, m, dtype=np.int32), a, b)
        if not abs(sc - s_dev[w]) <= 1e-9 * abs(sc) + 1e-12:
            out.append((int(w), s_dev[w], s_ref[w], sc))
    assert not out, f"mds 2 mismatches not explained by the start: {out[:10]}"
    return int(bad.size)


def freq_tracks(c, nsnp):
    """One allele-frequency value per population and SNP (the drosophila input, asize =
    bsize = 1), positions as the synthetic generator lays them out."""
    from gdscan import synth
    _, _, ap, _, regend = synth.chromosome(c, nsnp, 1, 1)
    rng = np.random.default_rng(c)
    qa = rng.beta(0.5, 0.5, nsnp)
    qb = np.clip(qa + rng.normal(0, 0.2, nsnp), 0, 1)
    qb[nsnp // 3:nsnp // 3 + 300] = 1 - qa[nsnp // 3:nsnp // 3 + 300]
    return qa, qb, ap, ap.copy(), regend


# ---------------------------------------------------------------- CPU: the oracle
def test_compare_freq_kat(opt):
    # testcss.c:337-367
    D = np.full(4, -1.0)
    opt.orc_css_compare_freq(np.array([0.75, 0.3, 0.2]), np.array([0.2, 0.5, 0.75]), 3, D)
    assert D[0] == 0 and D[3] == 0 and D[1] == D[2] and abs(D[1] - 0.433333) < 1e-6


def test_stress_kat(opt):
    # testcss.c:796-838; the expected 34.29899413 comes from unrounded distances, the
    # test's D holds them to 3 decimals
    delta = np.array([0, 5, 3, 4, 5, 0, 2, 2, 3, 2, 0, 1, 4, 2, 1, 0], np.float64)
    D = np.array([0, 1.068, 0.412, 1.065, 1.068, 0, 0.655, 0.706, 0.412, 0.655, 0, 0.792, 1.065, 0.706, 0.792, 0])
    s = opt.orc_css_stress(delta, D, 4)
    iu = np.tril_indices(4, -1)
    assert s == pytest.approx(((D.reshape(4, 4) - delta.reshape(4, 4))[iu] ** 2).sum(), rel=1e-15)
    assert abs(s - 34.29899413) < 1e-3


def test_smacof_kat(opt):
    # testcss.c:632-699: Borg & Groenen's example, X to 3 decimals
    delta = np.array([0, 5, 3, 4, 5, 0, 2, 2, 3, 2, 0, 1, 4, 2, 1, 0], np.float64)
    X = np.array([-0.266, -0.539, 0.451, 0.252, 0.016, -0.238, -0.200, 0.524])
    it = ctypes.c_int()
    opt.orc_css_smacof(delta, 4, X, 300, 0.000001, ctypes.byref(it))
    want = np.array([[-1.457, -2.575], [1.730, 1.23], [-0.028, 0.16], [-0.245, 1.185]])
    assert np.allclose(X.reshape(4, 2), want, atol=6e-3), X
    assert 1 <= it.value <= 301


def test_smacof_decreases_stress(opt):
    """Majorization never increases the stress; more iterations never end higher."""
    rng = np.random.default_rng(3)
    m = 12
    P = rng.normal(size=(m, 2)) * 5
    delta = np.sqrt(((P[:, None] - P[None]) ** 2).sum(-1)) + rng.uniform(0, 0.5, (m, m))
    delta = np.triu(delta, 1) + np.triu(delta, 1).T
    X0 = rng.uniform(size=2 * m)
    d0 = np.sqrt(((X0.reshape(m, 2)[:, None] - X0.reshape(m, 2)[None]) ** 2).sum(-1))
    s0 = opt.orc_css_stress(np.ascontiguousarray(delta.ravel()), np.ascontiguousarray(d0.ravel()), m)
    last = s0
    for iters in (1, 5, 50, 300):
        X = X0.copy()
        s = opt.orc_css_smacof(np.ascontiguousarray(delta.ravel()), m, X, iters, 0.0, None)
        assert s <= last + 1e-12
        last = s


# ---------------------------------------------------------------- GPU: HIP vs oracle
def _synth(c, nsnp, a, b):
    from gdscan import synth
    return synth.chromosome(c, nsnp, a, b)


def _close_frac(s, s_ref, rel):
    ok = (np.abs(s - s_ref) <= rel * np.abs(s_ref) + 1e-12) | (np.isnan(s) & np.isnan(s_ref))
    return ok.mean()


@pytest.mark.gpu
@pytest.mark.parametrize("a,b,nsnp", [(6, 6, 4000), (9, 7, 3000), (12, 12, 2500)])
def test_smacof_runs_match_oracle(opt, a, b, nsnp):
    from gdscan import css
    av, bv, ap, bp, regend = _synth(70 + a, nsnp, a, b)
    s, p = css.scan(av, bv, ap, bp, regend, runs=0, mds=1, seed=11)
    s_ref, p_ref = oracle_scan_ex(opt, av, bv, ap, bp, regend, 0, 1, seed=11)
    assert np.array_equal(s == 0, s_ref == 0)
    assert (s_ref != 0).sum() > 50
    assert _close_frac(s, s_ref, 1e-9) == 1.0
    assert np.array_equal(p, p_ref)


@pytest.mark.gpu
def test_smacof_after_cmds_matches_oracle(opt):
    from gdscan import css
    av, bv, ap, bp, regend = _synth(80, 4000, 8, 8)
    s, _ = css.scan(av, bv, ap, bp, regend, runs=0, mds=2)
    s_ref, _ = oracle_scan_ex(opt, av, bv, ap, bp, regend, 0, 2)
    assert np.array_equal(s == 0, s_ref == 0)
    assert_smacof2_mismatches_are_start_effects(opt, av, bv, ap, bp, regend, 8, 8, s, s_ref)


@pytest.mark.gpu
def test_smacof_with_permutations(opt):
    from gdscan import css
    av, bv, ap, bp, regend = _synth(81, 3000, 6, 6)
    s, p = css.scan(av, bv, ap, bp, regend, treshold=10, runs=200, mds=1, seed=5)
    s_ref, p_ref = oracle_scan_ex(opt, av, bv, ap, bp, regend, 0, 1, treshold=10, runs=200, seed=5)
    assert _close_frac(s, s_ref, 1e-9) == 1.0
    comp = s_ref != 0
    from conftest import assert_p_mismatches_are_ties
    assert_p_mismatches_are_ties(opt, av, bv, ap, bp, regend, 6, 6, np.where(comp, p, 0.0),
                                 np.where(comp, p_ref, 0.0), 10, 200, 5, mds=1)


@pytest.mark.gpu
@pytest.mark.parametrize("mds", [0, 1, 2])
def test_drosophila_metric_matches_oracle(opt, mds):
    from gdscan import css
    av, bv, ap, bp, regend = freq_tracks(90 + mds, 60_000)
    s, p = css.scan(av, bv, ap, bp, regend, treshold=10, runs=50, drosophila=1, mds=mds, seed=3)
    s_ref, p_ref = oracle_scan_ex(opt, av, bv, ap, bp, regend, 1, mds, treshold=10, runs=50, seed=3)
    assert np.array_equal(s == 0, s_ref == 0)
    assert (s_ref != 0).sum() > 5000
    assert _close_frac(s, s_ref, 1e-9) == 1.0
    # two points: a permutation keeps or swaps them, so every permuted score equals the
    # observed one in exact arithmetic and only rounding decides hit or miss -- the tie
    # bracket is the whole feasible range [1 / (runs + 1), 1]; a differing p must be a
    # value the p = (hits + 1) / (permutations + 1) rule can produce
    comp = s_ref != 0
    diff = comp & (p != p_ref)
    assert np.all((p[diff] >= 1.0 / 51) & (p[diff] <= 1.0))
    for v in np.unique(p[diff]):
        assert any(abs(v - (h + 1) / (n + 1)) < 1e-15 for n in range(1, 51) for h in range(0, min(n, 10) + 1))


@pytest.mark.gpu
def test_option_errors():
    import css_cython_parallel as ccp
    from gdscan import GdError
    av, bv, ap, bp, regend = _synth(9, 6_000, 4, 4)
    out = np.zeros(regend // 500)
    for dro, mds in ((1, 0), (0, 3), (2, 0), (0, -1)):  # drosophila needs 1 + 1; mds in 0..2
        with pytest.raises(GdError):
            ccp.cluster_separation_scorer(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 10, 0, dro, mds,
                                          out, out.copy())


@pytest.mark.gpu
def test_reference_entry_point_with_options(opt):
    """cluster_separation_scorer(..., drosophila, mds, ...) drives the options."""
    import css_cython_parallel as ccp
    from gdscan import lib
    av, bv, ap, bp, regend = _synth(82, 3000, 5, 5)
    lib.gd_set_seed(20261015)
    scores, p = np.zeros(regend // 500), np.full(regend // 500, -7.0)
    ccp.cluster_separation_scorer(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 10, 0, 0, 1, scores, p)
    s_ref, _ = oracle_scan_ex(opt, av, bv, ap, bp, regend, 0, 1)
    assert _close_frac(scores, s_ref, 1e-9) == 1.0
    assert np.all(p[s_ref == 0] == -7.0)
