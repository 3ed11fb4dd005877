"""The HyperBrowser statistics that call the hot path, restated for Python 3.

FisherExactScoreStatUnsplittable._compute   statistics/FisherExactScoreStat.py:28-61
CategoryClusterSeparationStatUnsplittable._compute
                                            statistics/CategoryClusterSeparationStat.py:32-80

HyperBrowser (`gold.*`, `quick.*`) is not part of this repository; these classes keep
the statistics' contract -- the kwargs they read, the `{"0": 0}` result for an empty
track A, `zeros(regend // wStep)` outputs, the positional call into the Cython-named
function and the `(scores, stddev|p)` result -- over any child results that expose
`startsAsNumpyArray()` / `valsAsNumpyArray()` (HyperBrowser's TrackView API).  The
reference's diagnostic prints are dropped.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .css import cluster_separation_scorer
from .fet import fisher_exact_tester


@dataclass
class Region:
    """The fields of gold.track.GenomeRegion the statistics read."""
    start: int
    end: int
    chr: str = ""


class TrackData:
    """Minimal stand-in for a HyperBrowser TrackView (one population's track)."""

    def __init__(self, starts, vals):
        self._starts = np.asarray(starts, dtype=np.int32)
        self._vals = np.asarray(vals, dtype=np.float64)

    def startsAsNumpyArray(self):  # noqa: N802 (HyperBrowser API name)
        return self._starts

    def valsAsNumpyArray(self):  # noqa: N802
        return self._vals


class _Child:
    def __init__(self, result):
        self._result = result

    def getResult(self):  # noqa: N802
        return self._result


class _TwoTrackStat:
    def __init__(self, region, track_a, track_b, **kwArgs):
        self._region = region
        self._children = [_Child(track_a), _Child(track_b)]
        self._kwArgs = kwArgs

    def _inputs(self):
        group_a = self._children[0].getResult()
        group_b = self._children[1].getResult()
        apos = group_a.startsAsNumpyArray()
        if len(apos) == 0:
            return None
        return (group_a.valsAsNumpyArray(), group_b.valsAsNumpyArray(), apos, group_b.startsAsNumpyArray())

    def compute(self):
        return self._compute()


class FisherExactScoreStatUnsplittable(_TwoTrackStat):
    """kwargs: wSize, wStep, percentile (FisherExactScoreStat.py:45-50)."""

    def _compute(self):
        ins = self._inputs()
        if ins is None:
            return {"0": 0}
        avals, bvals, apos, bpos = ins
        reg = self._region
        w_size = int(self._kwArgs["wSize"])
        w_step = int(self._kwArgs["wStep"])
        perc = float(self._kwArgs["percentile"])
        num_win = reg.end // w_step
        scores = np.zeros(num_win)
        stddev = np.zeros(num_win)
        fisher_exact_tester(avals, bvals, apos, bpos, reg.start, reg.end, w_size, w_step, avals.shape[0],
                            bvals.shape[0], perc, scores, stddev)
        return scores, stddev


class CategoryClusterSeparationStatUnsplittable(_TwoTrackStat):
    """kwargs: wSize, wStep, mcT, mcR, func ("True" -> drosophila metric), mds
    (CategoryClusterSeparationStat.py:46-66)."""

    def _compute(self):
        ins = self._inputs()
        if ins is None:
            return {"0": 0}
        avals, bvals, apos, bpos = ins
        reg = self._region
        w_size = int(self._kwArgs["wSize"])
        w_step = int(self._kwArgs["wStep"])
        treshold = int(self._kwArgs["mcT"])
        runs = int(self._kwArgs["mcR"])
        drosophila = 1 if self._kwArgs["func"] == "True" else 0
        mds = int(self._kwArgs["mds"])
        num_win = reg.end // w_step
        scores = np.zeros(num_win)
        p = np.zeros(num_win)
        cluster_separation_scorer(avals, bvals, apos, bpos, reg.start, reg.end, w_size, w_step, avals.shape[0],
                                  bvals.shape[0], treshold, runs, drosophila, mds, scores, p)
        return scores, p
