"""CPU restatement of the region filters that follow the scans -- TEST INFRASTRUCTURE ONLY.

Only tests/ and bench.py's CPU-baseline leg (the numpy restatement timed beside the
device region filters, after the timed steps) may import this module, as the checker
of gd_fet_region_limit, gd_css_fdr_threshold, gd_css_top_limit and gd_merge_regions;
the product path never calls it.

Restated from the reference tools (Python 2 + HyperBrowser, not importable here):
  filter_limit      tools/FilterFisherScores.py:83-87
  bh_threshold      tools/SignificantCSSRegions.py:102-123
  top_limit         tools/SignificantCSSRegions.py:124-127
  merge_regions     tools/FilterFisherScores.py:97-114 (== SignificantCSSRegions.py:129-150)
  parse_tabular     FilterFisherScores.py:117-131 / SignificantCSSRegions.py:157-173

Third-party arithmetic the tools call:
  scipy.stats.cmedian(a, numbins=1000) -- removed from scipy in 0.12, so it is restated
    here from the scipy 0.9-0.11 source, floating-point steps included (scipy.stats.histogram
    over its default limits, binsize = bin_edges[1] - bin_edges[0], LRL = smallest +
    binsize * cfbin, then linear interpolation inside the median bin).  PARITY UNPINNED against a
    live scipy: no reference fixture holds a cmedian value; the tests pin it against the
    exact median within one bin width and against a hand-computed case.
  scipy.stats.scoreatpercentile(a, per) -- restated in its scipy 0.x form
    (a + (b - a) * (idx % 1)); checked against the installed scipy within 1e-12.
  scipy.stats.norm.ppf -- the installed scipy (cephes ndtri, unchanged since).
"""
from __future__ import annotations

import numpy as np

CMEDIAN_BINS = 1000


def histogram_limits(a, numbins):
    """scipy.stats.histogram(a, numbins) of scipy 0.9-0.11, default limits: (hist,
    smallest = min - s, binsize = bin_edges[1] - bin_edges[0]); numpy.histogram widens an
    empty range internally, smallest stays min - s."""
    data_min, data_max = a.min(), a.max()
    s = (data_max - data_min) / (2.0 * (numbins - 1.0))
    lo, hi = data_min - s, data_max + s
    hist, bins = np.histogram(a, numbins, range=(lo, hi))
    return np.asarray(hist, dtype=np.float64), lo, bins[1] - bins[0]


def cmedian(a, numbins=CMEDIAN_BINS):
    """scipy.stats.cmedian (scipy <= 0.11): LRL = smallest + binsize * cfbin."""
    a = np.ravel(np.asarray(a, dtype=np.float64))
    n = float(len(a))
    hist, smallest, binsize = histogram_limits(a, numbins)
    cumhist = np.cumsum(hist)
    cfbin = int(np.searchsorted(cumhist, n / 2.0))
    lrl = smallest + binsize * cfbin
    cfbelow = cumhist[cfbin - 1]  # Python index: cumhist[-1] when cfbin == 0
    freq = float(hist[cfbin])
    return lrl + ((n / 2.0 - cfbelow) / freq) * binsize


def scoreatpercentile(a, per):
    values = np.sort(np.asarray(a, dtype=np.float64), axis=0)
    idx = per / 100.0 * (values.shape[0] - 1)
    if idx % 1 == 0:
        return values[int(idx)]
    return values[int(idx)] + (values[int(idx) + 1] - values[int(idx)]) * (idx % 1)


def filter_limit(scores, stddev, normquantile, percentile):
    """FilterFisherScores.py:84-87 -> (limit, median, upperquant, qnorm)."""
    from scipy import stats
    m = cmedian(scores)
    upperquant = scoreatpercentile(stddev, percentile)
    qnorm = stats.norm.ppf(normquantile)
    return m + qnorm * upperquant, m, upperquant, qnorm


def bh_threshold(p, fdr):
    """SignificantCSSRegions.py:104-114 -> (testp, k); k == 0 means "NONE found"."""
    p = np.asarray(p, dtype=np.float64)
    psorted = np.argsort(p)[::-1]
    k = float(len(p))
    n = k
    testp = 0
    for pi in psorted:
        if p[pi] <= k / n * fdr:
            testp = p[pi]
            break
        k -= 1
    return testp, int(k)


def top_limit(scores, num_top):
    scores = np.asarray(scores, dtype=np.float64)
    scoresorted = np.argsort(scores)[::-1]
    return scores[scoresorted[num_top - 1]]


def merge_regions(seqids, starts, keep, window_size, chrom_end):
    """FilterFisherScores.py:97-114: [(first kept index, end)], pure-Python loop.

    seqids/starts: per window (strings / ints); keep: boolean mask; chrom_end(seqid) =
    chromosome length - 1."""
    out = []
    curchrom, first, end, prev = "", None, None, -1000000.0
    for i in np.flatnonzero(keep):
        if seqids[i] != curchrom or int(starts[i]) - window_size > prev:
            if curchrom != "":
                out.append((first, prev + window_size if prev + window_size < end else end))
            first, curchrom, end = int(i), seqids[i], chrom_end(seqids[i])
        prev = int(starts[i])
    if curchrom != "":
        out.append((first, prev + window_size if prev + window_size < end else end))
    return out


def parse_tabular(text, cols):
    """preProcessPvalues: (addr list, one float array per requested column)."""
    addr, vals = [], [[] for _ in cols]
    for line in text.split("\n"):
        if not line or line[0] == "#":
            continue
        c = line.split("\t")
        addr.append(c[0] + "\t" + c[1])
        for v, k in zip(vals, cols):
            v.append(float(c[k]))
    return addr, [np.asarray(v, dtype=np.float64) for v in vals]


def filter_fisher_scores_text(text, chrom_len, window_size=100000, normquantile=0.999, percentile=75.0):
    """The whole FilterFisherScores.execute output file (FilterFisherScores.py:69-115)."""
    addr, (fet, sd) = parse_tabular(text, (2, 3))
    limit = filter_limit(fet, sd, normquantile, percentile)[0]
    keep = fet >= limit
    head = ("##gtrack version: 1.0\n##track type: segments\n##uninterrupted data lines: true\n"
            "##sorted elements: false\n##no overlapping elements: true\n###seqid\tstart\tend\n")
    return head + _segments(addr, keep, window_size, chrom_len)


def significant_css_regions_text(text, chrom_len, fdr=None, num_top=None, window_size=2500):
    """The whole SignificantCSSRegions.execute output file (SignificantCSSRegions.py:86-154)."""
    addr, (scores, p) = parse_tabular(text, (2, 3))
    if fdr is not None:
        testp, k = bh_threshold(p, fdr)
        if k == 0:
            return "NONE found"
        keep = p <= testp
    else:
        keep = scores >= top_limit(scores, num_top)
    head = ("##gtrack version: 1.0\n##track type: segments\n##uninterrupted data lines: true\n"
            "##no overlapping elements: true\n###seqid\tstart\tend\n")
    return head + _segments(addr, keep, window_size, chrom_len)


def _py2_str(x):
    if isinstance(x, (int, np.integer)):
        return str(int(x))
    t = "%.12g" % x
    return t + ".0" if t.lstrip("-").isdigit() else t


def _segments(addr, keep, window_size, chrom_len):
    seq = [a.split("\t")[0] for a in addr]
    st = [a.split("\t")[1] for a in addr]
    regs = merge_regions(seq, st, keep, window_size, lambda s: int(chrom_len[s]) - 1)
    if not regs:  # the loop never opened a region: start "" and prevAddr = -1000000.
        return "\t" + _py2_str(-1000000.0 + window_size) + "\n"
    return "".join(addr[f] + "\t" + _py2_str(e) + "\n" for f, e in regs)
