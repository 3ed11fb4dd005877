"""GPU: the general CSS path for cohorts above the register tiers (128 < m <= 512;
k_css_mds_big, k_css_perm_big, k_css_smacof<.., BIG>), which the reference supports for
any m (threadcss.c:191,207-215; css.c:181-223).  Scores against the oracle at 1e-9
relative; permutation p on the device's own coordinates inside the oracle's near-tie
bracket (as tests/test_css_perm_isolated.py); SMACOF (mds 1) against the oracle's
reference-order restatement; cohorts above 512 refused.  The serial window set keeps
the oracle's O(m^3) per-window cost to seconds."""
import numpy as np
import pytest

from conftest import oracle_css_scan
from test_css_options import _close_frac, opt, oracle_scan_ex  # noqa: F401  (opt: the options' argtypes)
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
    assert _close_frac(s2, s2_ref, 1e-9) >= 0.95 and _close_frac(s2, s2_ref, 1e-4) == 1.0


def test_above_the_general_path_raises():
    from gdscan import GdError, css, synth
    av, bv, ap, bp, regend = synth.chromosome(240, 200, 300, 300)
    with pytest.raises(GdError):
        css.scan(av, bv, ap, bp, regend, serial=True)


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
