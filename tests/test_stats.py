"""The HyperBrowser statistics' contract (FisherExactScoreStat.py:28-61,
CategoryClusterSeparationStat.py:32-80)."""
import numpy as np
import pytest

from conftest import close, oracle_css_scan, oracle_fet_scan


def _tracks(c, nsnp, a, b):
    from gdscan import synth
    from gdscan.stats import TrackData
    av, bv, ap, bp, regend = synth.chromosome(c, nsnp, a, b)
    return TrackData(ap, av), TrackData(bp, bv), (av, bv, ap, bp, regend)


def test_empty_track_returns_marker():
    from gdscan.stats import (CategoryClusterSeparationStatUnsplittable, FisherExactScoreStatUnsplittable,
                              Region, TrackData)
    empty = TrackData([], [])
    other = TrackData([5], [3.0])
    assert FisherExactScoreStatUnsplittable(Region(0, 10_000), empty, other, wSize=2500, wStep=500,
                                            percentile=0.95).compute() == {"0": 0}
    assert CategoryClusterSeparationStatUnsplittable(Region(0, 10_000), empty, other, wSize=2500, wStep=500,
                                                     mcT=10, mcR=0, func="False", mds=0).compute() == {"0": 0}


@pytest.mark.gpu
def test_fisher_stat_matches_oracle(oracle):
    from gdscan import lib
    from gdscan.stats import FisherExactScoreStatUnsplittable, Region
    ta, tb, (av, bv, ap, bp, regend) = _tracks(50, 30_000, 10, 10)
    lib.gd_set_seed(20261015)
    scores, stddev = FisherExactScoreStatUnsplittable(Region(0, regend), ta, tb, wSize="2500", wStep="500",
                                                      percentile="0.95").compute()
    assert scores.shape == (regend // 500,)
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend)
    assert close(scores, s_ref) and close(stddev, d_ref)


@pytest.mark.gpu
def test_css_stat_matches_oracle(oracle):
    from gdscan import lib
    from gdscan.stats import CategoryClusterSeparationStatUnsplittable, Region
    ta, tb, (av, bv, ap, bp, regend) = _tracks(51, 20_000, 8, 8)
    lib.gd_set_seed(20261015)
    scores, p = CategoryClusterSeparationStatUnsplittable(Region(0, regend), ta, tb, wSize="2500", wStep="500",
                                                          mcT="10", mcR="0", func="False", mds="0").compute()
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend)
    assert close(scores, s_ref)
    assert np.array_equal(p, p_ref)
