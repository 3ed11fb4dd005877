"""GPU: the general CSS path for cohorts above the register tiers (128 < m <= 2048;
k_css_mds_big, k_css_perm_big, k_css_smacof<.., BIG>), which the reference supports for
any m (threadcss.c:191,207-215; css.c:181-223).  Scores against the oracle at 1e-9
relative; permutation p on the device's own coordinates inside the oracle's near-tie
bracket (as tests/test_css_perm_isolated.py); SMACOF (mds 1) against the oracle's
reference-order restatement (SMACOF up to 1024); cohorts above 2048 refused.  The serial window set keeps
the oracle's O(m^3) per-window cost to seconds."""
import numpy as np
import pytest

from conftest import oracle_css_scan
from test_css_options import _close_frac, assert_smacof2_mismatches_are_start_effects, opt, oracle_scan_ex  # noqa: F401
from test_css_perm_isolated import _oracle_p

pytestmark = pytest.mark.gpu


def _cmp(s, s_ref, min_windows=20):
    assert np.array_equal(s == 0, s_ref == 0), "computed-window sets differ"
    assert (s_ref != 0).sum() >= min_windows
    ok = np.isnan(s_ref) | (np.abs(s - s_ref) <= 1e-9 * np.abs(s_ref) + 1e-12)
    assert ok.all(), (np.flatnonzero(~ok)[:10], s[~ok][:5], s_ref[~ok][:5])


@pytest.mark.parametrize("a,b,nsnp", [(70, 70, 500), (100, 100, 400), (129, 3, 500), (150, 120, 300),
                                      (140, 120, 120)])
def test_general_path_scores(oracle, a, b, nsnp):
    from gdscan import css, synth
    av, bv, ap, bp, regend = synth.chromosome(200 + a, nsnp, a, b)
    s, p = css.scan(av, bv, ap, bp, regend, runs=0, serial=True)
    s_ref, _ = oracle_css_scan(oracle, av, bv, ap, bp, regend, runs=0, serial=True)
    _cmp(s, s_ref, 20 if nsnp > 200 else 6)  # 257..512 (the MP = 512 kernel): the oracle's
    assert np.all(p[s != 0] == 1.0)            # Jacobi solver takes ~1.5 s per window


def test_general_path_literal_windows(oracle):
    from gdscan import css, synth
    av, bv, ap, bp, regend = synth.chromosome(210, 400, 80, 70)
    rng = np.random.default_rng(1)
    idx = rng.choice(len(av), 30, replace=False)
    av[idx] = rng.choice([1.0, 9.0, -9.0, np.nan, 4.5, -3.0000001], 30)
    s, _ = css.scan(av, bv, ap, bp, regend, serial=True)
    s_ref, _ = oracle_css_scan(oracle, av, bv, ap, bp, regend, serial=True)
    _cmp(s, s_ref)


@pytest.mark.parametrize("a,b,nsnp,treshold,runs", [(100, 100, 400, 10, 100), (70, 80, 500, 30, 150),
                                                  (150, 110, 120, 10, 40)])
def test_general_path_permutations(oracle, a, b, nsnp, treshold, runs):
    from gdscan import css, synth
    av, bv, ap, bp, regend = synth.chromosome(220 + a, nsnp, a, b)
    s, p, X = css.scan_coords(av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=13, serial=True)
    s_ref, _ = oracle_css_scan(oracle, av, bv, ap, bp, regend, serial=True)
    _cmp(s, s_ref, 20 if nsnp > 200 else 6)
    bad = []
    for w in np.flatnonzero(s != 0):
        sc, p_lit, lo, hi, nt = _oracle_p(oracle, X[w], a, b, treshold, runs, 13, int(w))
        assert abs(sc - s[w]) <= 1e-12 * abs(s[w]) + 1e-12
        if not lo <= p[w] <= hi:
            bad.append((int(w), p[w], lo, hi, nt))
    assert not bad, bad[:10]


def test_general_path_smacof(opt):
    from gdscan import css, synth
    oracle = opt
    av, bv, ap, bp, regend = synth.chromosome(230, 300, 70, 66)
    s, p = css.scan(av, bv, ap, bp, regend, runs=0, mds=1, seed=11, serial=True)
    s_ref, p_ref = oracle_scan_ex(oracle, av, bv, ap, bp, regend, 0, 1, seed=11, serial=True)
    assert np.array_equal(s == 0, s_ref == 0) and (s_ref != 0).sum() >= 20
    assert _close_frac(s, s_ref, 1e-9) == 1.0
    s2, _ = css.scan(av, bv, ap, bp, regend, runs=0, mds=2, serial=True)
    s2_ref, _ = oracle_scan_ex(oracle, av, bv, ap, bp, regend, 0, 2, serial=True)
    assert_smacof2_mismatches_are_start_effects(oracle, av, bv, ap, bp, regend, 70, 66, s2, s2_ref, serial=True)


def test_above_the_general_path_raises():
    """above 2048 individuals a scan returns GD_ERR_SIZE, classical or SMACOF"""
    from gdscan import GdError, css, synth
    av, bv, ap, bp, regend = synth.chromosome(240, 60, 1030, 1030)
    for mds in (0, 1):
        with pytest.raises(GdError):
            css.scan(av, bv, ap, bp, regend, runs=0, mds=mds, serial=True)


def _lapack_scores(orc, av, bv, ap, bp, regend, a, b, wsize=2500, wstep=500):
    """Serial-window CSS scores with the eigen-step on LAPACK (numpy eigh) instead of the
    oracle's cyclic Jacobi, whose O(m^3) sweeps take minutes per window above 512
    individuals: window slicing as orc_css_scan (slide_right, comparative.c:49-71),
    compare_all and fill_averages from the oracle, X = top-2 eigenpairs of
    B = -1/2 Z D^2 Z (test_oracle_css.numpy_cmds, pinned there to the oracle at 1e-11),
    calc_dist and css from the oracle."""
    import ctypes
    from test_oracle_css import numpy_cmds
    F64 = np.ctypeslib.ndpointer(np.float64, flags="C")
    I32 = np.ctypeslib.ndpointer(np.int32, flags="C")
    C = ctypes
    orc.orc_css_compare_all.argtypes = [F64, F64, C.c_int, C.c_int, C.c_int, F64]
    orc.orc_css_fill_averages.argtypes = [F64, C.c_int]
    orc.orc_css_score.argtypes = [F64, C.c_int, I32, I32, C.c_int, C.c_int]
    orc.orc_css_score.restype = C.c_double
    orc.orc_serial_window_end.argtypes = [C.c_int] * 3
    m = a + b
    out = np.zeros(regend // wstep)
    for w in range(orc.orc_serial_window_end(regend, wsize, wstep)):
        start, stop = w * wstep, w * wstep + wsize
        la0, la1 = np.searchsorted(ap, start, "left"), np.searchsorted(ap, stop, "right")
        lb0 = np.searchsorted(bp, start, "left")
        npos = (la1 - la0) // a
        if npos <= 0:
            continue
        D = np.zeros(m * m)
        orc.orc_css_compare_all(np.ascontiguousarray(av[la0:la0 + npos * a]),
                                np.ascontiguousarray(bv[lb0:lb0 + npos * b]), a, b, int(npos), D)
        if not orc.orc_css_fill_averages(D, m):
            continue
        X = numpy_cmds(D.reshape(m, m))
        S = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)).ravel()
        out[w] = orc.orc_css_score(np.ascontiguousarray(S), m, np.arange(a, dtype=np.int32),
                                   np.arange(a, m, dtype=np.int32), a, b)
    return out


@pytest.mark.parametrize("a,b,nsnp,runs", [(300, 300, 150, 30), (700, 290, 110, 0), (512, 512, 100, 0),
                                            # the 2048 tier (1025..2048: four rows per thread, the masks,
                                            # iterates and coordinates in the slab, 16 permutations per pass)
                                            (520, 520, 100, 20), (1000, 700, 90, 0)])
def test_cohorts_above_512(oracle, a, b, nsnp, runs):
    """The 1024 tier (513..1024 individuals: two rows per thread in k_css_mds_big, the
    inverse-iteration factors in the slab, 32 permutations per pass in k_css_perm_big) and
    the 2048 tier:
    scores against the LAPACK-eigen-step restatement at 1e-9, permutation p on the
    device's own coordinates inside the oracle's tie bracket.  The reference scores any
    m (threadcss.c:191,207-215; css.c:181-223)."""
    from gdscan import css, synth
    treshold = 10
    av, bv, ap, bp, regend = synth.chromosome(270 + a, nsnp, a, b)
    if runs:
        s, p, X = css.scan_coords(av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=19, serial=True)
    else:
        s, p = css.scan(av, bv, ap, bp, regend, treshold=treshold, runs=0, seed=19, serial=True)
    s_ref = _lapack_scores(oracle, av, bv, ap, bp, regend, a, b)
    _cmp(s, s_ref, 4)
    bad = []
    for w in np.flatnonzero(s != 0) if runs else []:
        sc, p_lit, lo, hi, nt = _oracle_p(oracle, X[w], a, b, treshold, runs, 19, int(w))
        assert abs(sc - s[w]) <= 1e-12 * abs(s[w]) + 1e-12
        if not lo <= p[w] <= hi:
            bad.append((int(w), p[w], lo, hi))
    assert not bad, bad[:10]
    if not runs:
        assert np.all(p[s != 0] == 1.0)


def test_general_path_several_windows_per_workgroup(oracle, opt, monkeypatch):
    """The general-path kernels loop over windows with a slab per workgroup (grid = the
    device's resident capacity); GD_CSS_BIG_GRID=3 forces each workgroup through many
    windows, reusing its slab: MDS scores, permutation p (inside the oracle's tie bracket
    on the device's coordinates) and SMACOF must still match the oracle."""
    from gdscan import css, synth
    monkeypatch.setenv("GD_CSS_BIG_GRID", "3")
    a, b, nsnp, treshold, runs = 90, 80, 400, 10, 60
    av, bv, ap, bp, regend = synth.chromosome(250, nsnp, a, b)
    s, p, X = css.scan_coords(av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=17, serial=True)
    s_ref, _ = oracle_css_scan(oracle, av, bv, ap, bp, regend, serial=True)
    _cmp(s, s_ref, 20)
    assert (s != 0).sum() > 3 * 6  # at least six windows per workgroup
    bad = []
    for w in np.flatnonzero(s != 0):
        sc, p_lit, lo, hi, nt = _oracle_p(oracle, X[w], a, b, treshold, runs, 17, int(w))
        if not lo <= p[w] <= hi:
            bad.append((int(w), p[w], lo, hi))
    assert not bad, bad[:10]
    s1, _ = css.scan(av, bv, ap, bp, regend, runs=0, mds=1, seed=11, serial=True)
    s1_ref, _ = oracle_scan_ex(opt, av, bv, ap, bp, regend, 0, 1, seed=11, serial=True)
    assert _close_frac(s1, s1_ref, 1e-9) == 1.0


@pytest.mark.parametrize("a,b,nsnp,nwin", [(300, 300, 100, 5), (520, 520, 60, 2)])
def test_cohorts_above_512_smacof(opt, a, b, nsnp, nwin):
    """SMACOF (mds 1) at the 1024 tier (1024-thread workgroups, counts and stress triangle
    in the slab) and the 2048 tier (two individuals per thread) against the oracle's
    reference-order restatement."""
    from gdscan import css, synth
    av, bv, ap, bp, regend = synth.chromosome(275 + a - 300, nsnp, a, b)
    s, _ = css.scan(av, bv, ap, bp, regend, runs=0, mds=1, seed=11, serial=True)
    s_ref, _ = oracle_scan_ex(opt, av, bv, ap, bp, regend, 0, 1, seed=11, serial=True)
    assert np.array_equal(s == 0, s_ref == 0) and (s_ref != 0).sum() >= nwin
    assert _close_frac(s, s_ref, 1e-9) == 1.0
