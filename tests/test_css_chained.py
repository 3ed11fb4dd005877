"""Statistical check of deviation 1: the reference's chained permutation
convention (Q9: one time-seeded nrand48 state per scan and one `signtracks` array that
every window keeps shuffling, css.c:49-156, 727-752; threadcss.c:197-204, 269) against
the per-window convention used here (each window its own (seed, w) stream, identity start
tracks).

A uniformly random shuffle composed with any fixed start arrangement is uniform again, so
the two conventions draw every window's permutations from the same distribution and the
p-values must agree in distribution (not bit for bit).  Tests, over ~1-2 thousand windows:
  * sign test: log p_here - log p_chained is symmetric about 0 (|z| < 4)
  * hit counts of the windows that ran all mcR permutations in both: equal totals within 4
    standard deviations (binomial variance from the pooled rate)
  * the per-window difference is consistent with Monte-Carlo noise: the fraction of
    windows whose two p differ by more than 5 binomial standard deviations is < 1 %.
CPU: oracle (per-window) vs oracle (chained).  GPU: the HIP scan vs oracle (chained)."""
import ctypes

import numpy as np
import pytest

from conftest import DP, IP, oracle_css_scan


def _chained(orc, av, bv, ap, bp, regend, treshold, runs, state48, serial=False):
    C = ctypes
    f = orc.orc_css_scan_chained
    f.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                  C.c_int, DP, DP]
    n = regend // 500
    s, p = np.zeros(n), np.zeros(n)
    assert f(av, bv, ap, bp, regend, 2500, 500, len(av), len(bv), treshold, runs, state48, int(serial), s, p) == 0
    return s, p


def _runs_hits(p, treshold, runs):
    """(permutations run, hits) from p = (hits + 1) / (run + 1)."""
    early = p * (runs + 1) > treshold + 0.5
    n = np.where(early, np.rint((treshold + 1) / p) - 1, runs)
    h = np.where(early, treshold, np.rint(p * (runs + 1)) - 1)
    return n, h


def _compare(p1, p2, treshold, runs):
    assert len(p1) > 500
    d = np.log(p1) - np.log(p2)
    pos, neg = int((d > 0).sum()), int((d < 0).sum())
    z_sign = (pos - neg) / np.sqrt(max(pos + neg, 1))
    assert abs(z_sign) < 4, (pos, neg, z_sign)
    n1, h1 = _runs_hits(p1, treshold, runs)
    n2, h2 = _runs_hits(p2, treshold, runs)
    full = (n1 == runs) & (n2 == runs)
    assert full.sum() > 100
    pi = (h1[full] + h2[full]) / (2.0 * runs)
    var = 2.0 * runs * pi * (1 - pi)
    z_hits = (h1[full].sum() - h2[full].sum()) / np.sqrt(max(var.sum(), 1.0))
    assert abs(z_hits) < 4, z_hits
    sd = np.sqrt(np.maximum(var, 1.0))
    far = np.abs(h1[full] - h2[full]) > 5 * sd
    assert far.mean() < 0.01, far.mean()
    return z_sign, z_hits


@pytest.mark.parametrize("a,b,treshold,runs", [(10, 10, 50, 400), (6, 9, 20, 300)])
def test_chained_convention_matches_per_window_oracle(oracle, a, b, treshold, runs):
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(70, 15_000, a, b)
    s1, p1 = oracle_css_scan(oracle, av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=123)
    s2, p2 = _chained(oracle, av, bv, ap, bp, regend, treshold, runs, 0x1234ABCD5678)
    assert np.array_equal(s1, s2)  # scores do not depend on the permutation convention
    comp = s1 != 0
    _compare(p1[comp], p2[comp], treshold, runs)


@pytest.mark.gpu
@pytest.mark.parametrize("a,b,treshold,runs,nsnp", [(20, 20, 50, 400, 15_000), (12, 13, 30, 300, 15_000)])
def test_chained_convention_matches_gpu(oracle, a, b, treshold, runs, nsnp):
    from gdscan import css, synth
    av, bv, ap, bp, regend = synth.chromosome(71, nsnp, a, b)
    s1, p1 = css.scan(av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=321)
    s2, p2 = _chained(oracle, av, bv, ap, bp, regend, treshold, runs, 0x0F0E0D0C0B0A)
    comp = s2 != 0
    assert np.array_equal(s1 != 0, comp)
    _compare(p1[comp], p2[comp], treshold, runs)
