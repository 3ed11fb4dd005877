"""Region filters after the scan: FilterFisherScores and
SignificantCSSRegions.

CPU tests pin the restatement (oracle/regions_oracle.py) -- scoreatpercentile against
the installed scipy, cmedian by a hand-computed case and the one-bin bound, BH against
an independent vectorised form, the merge against hand-made tracks -- and the native
tabular reader.  GPU tests compare the device path (gd_fet_region_limit,
gd_css_fdr_threshold, gd_css_top_limit, gd_merge_regions) with the restatement: all
outputs are exact (order statistics, integer merges; the limit formulas run the same
IEEE operations in the same order).
"""
import sys

import numpy as np
import pytest

from conftest import ORACLE_DIR

if str(ORACLE_DIR) not in sys.path:
    sys.path.insert(0, str(ORACLE_DIR))
import regions_oracle as ro  # noqa: E402


def rng(seed=1):
    return np.random.default_rng(seed)


# ----------------------------------------------------------------------- CPU: oracle pins
def test_scoreatpercentile_matches_scipy():
    from scipy import stats
    r = rng()
    for n in (1, 2, 7, 100, 1001):
        a = r.gamma(2.0, 1.0, n)
        for per in (0, 12.5, 50, 75, 99.9, 100):
            want = stats.scoreatpercentile(a, per)
            assert ro.scoreatpercentile(a, per) == pytest.approx(want, rel=1e-12, abs=1e-300)


def test_cmedian_hand_case():
    # values 0..4, numbins 5: s = 4/8 = .5, bins [-.5, 4.5] width 1; cumhist = 1 2 3 4 5;
    # n/2 = 2.5 -> cfbin 2, LRL 1.5, cfbelow 2, freq 1 -> 1.5 + 0.5 = 2.0
    assert ro.cmedian(np.arange(5.0), numbins=5) == 2.0
    # cfbin == 0 reads cumhist[-1] (Python indexing): two values a < b
    a, b = 1.0, 3.0
    s = (b - a) / (2 * 999.0)
    edges = np.linspace(a - s, b + s, 1001)
    assert ro.cmedian([a, b]) == (a - s) + ((1.0 - 2.0) / 1.0) * (edges[1] - edges[0])
    # LRL = smallest + binsize * cfbin, not bin_edges[cfbin] (scipy 0.9-0.11 steps)
    x = np.array([0.1, 0.7, 0.3, 0.9, 0.5])
    s = 0.8 / (2 * 999.0)
    hist, edges = np.histogram(x, 1000, range=(0.1 - s, 0.9 + s))
    cfbin = int(np.searchsorted(np.cumsum(hist), 2.5))
    bs = edges[1] - edges[0]
    assert ro.cmedian(x) == (0.1 - s) + bs * cfbin + ((2.5 - np.cumsum(hist)[cfbin - 1]) / 1.0) * bs
    # all values equal: numpy.histogram widens the range by 0.5 each side, smallest does not
    e = np.linspace(1.5, 2.5, 1001)
    bs = e[1] - e[0]
    assert ro.cmedian(np.full(4, 2.0)) == 2.0 + bs * 500 + (2.0 / 4.0) * bs


def test_cmedian_within_one_bin_of_median():
    r = rng(2)
    for n in (101, 1000, 50001):
        a = r.gamma(1.5, 2.0, n)
        bw = (a.max() - a.min()) / 999.0
        assert abs(ro.cmedian(a) - np.median(a)) <= bw


def bh_vectorised(p, fdr):
    p = np.asarray(p, np.float64)
    n = len(p)
    s = np.sort(p)  # NaN last
    ok = s <= (np.arange(1, n + 1) / float(n)) * fdr
    if not ok.any():
        return 0, 0
    k = int(np.flatnonzero(ok)[-1]) + 1
    return s[k - 1], k


def test_bh_loop_equals_step_up():
    r = rng(3)
    for n in (1, 5, 200, 3000):
        for fdr in (0.01, 0.05, 0.2):
            p = np.round(r.beta(0.3, 2.0, n), 3)  # ties
            if n > 4:
                p[::7] = np.nan
            assert ro.bh_threshold(p, fdr) == bh_vectorised(p, fdr)
    assert ro.bh_threshold(np.ones(10), 0.05) == (0, 0)


def test_merge_hand_case():
    seq = ["c1"] * 5 + ["c2"] * 3
    st = [0, 500, 5000, 5500, 9000, 0, 100, 200]
    keep = np.array([1, 1, 1, 0, 1, 1, 0, 1], bool)
    ends = {"c1": 9999, "c2": 1000}
    regs = ro.merge_regions(seq, st, keep, 2500, lambda s: ends[s] - 1)
    # c1: 0,500 -> [0, 3000]; 5000 (5000-2500 > 500) -> [5000, 7500]; 9000 -> [9000, min(11500, 9998)]
    # c2: 0,200 -> [0, min(2700, 999)]
    assert regs == [(0, 3000), (2, 7500), (4, 9998), (5, 999)]


def test_tool_text_empty_selection():
    text = "#seqid\tstart\tscore\tp\nc1\t0\t1.5\t0.5\n"
    out = ro.significant_css_regions_text(text, {"c1": 10000}, num_top=1, window_size=2500)
    assert out.endswith("c1\t0\t2500\n")
    assert ro.significant_css_regions_text(text, {"c1": 10000}, fdr=0.05) == "NONE found"


def test_tabular_reader(tmp_path):
    from gdscan.regions import read_tabular
    text = ("#seqid\tstart\tscore\tstddev\nchr1\t0\t1.25\t0.5\nchr1\t500\tnan\t2.0\r\n"
            "# comment\nchr2\t1000\t3.0\t-inf\nchr1\t1500\t1e-3\t7\n")
    f = tmp_path / "t.tabular"
    f.write_text(text)
    seqids, seq, start, c2, c3 = read_tabular(f)
    addr, (w2, w3) = ro.parse_tabular(text, (2, 3))
    assert [seqids[s] + "\t" + str(x) for s, x in zip(seq, start)] == addr
    np.testing.assert_array_equal(c2, w2)
    np.testing.assert_array_equal(c3, w3)
    bad = tmp_path / "bad.tabular"
    bad.write_text("chr1\t0\t1.0\n")
    from gdscan import GdError
    with pytest.raises(GdError):
        read_tabular(bad)


def test_tabular_reader_large_multithreaded(tmp_path):
    from gdscan.regions import read_tabular
    r = rng(4)
    n = 600_000
    seq = np.repeat(np.arange(6), n // 6)
    start = np.tile(np.arange(n // 6) * 500, 6)
    v = r.normal(size=n)
    lines = "".join(f"s{a}\t{b}\t{c!r}\t{c * 2!r}\n" for a, b, c in zip(seq.tolist(), start.tolist(), v.tolist()))
    f = tmp_path / "big.tabular"
    f.write_text("#seqid\tstart\tscore\tp\n" + lines)
    seqids, sq, st, c2, c3 = read_tabular(f)
    assert seqids == [f"s{k}" for k in range(6)]
    np.testing.assert_array_equal(sq, seq)
    np.testing.assert_array_equal(st, start)
    np.testing.assert_array_equal(c2, v)
    np.testing.assert_array_equal(c3, v * 2)


# ----------------------------------------------------------------------- GPU: device path
gpu = pytest.mark.gpu


@gpu
@pytest.mark.parametrize("n", [1, 2, 3, 10, 999, 100_003])
def test_fet_limit_matches_oracle(n):
    from gdscan.regions import fet_region_limit
    r = rng(10 + n)
    sc = r.gamma(2.0, 1.5, n)
    if n > 10:
        sc[::5] = np.round(sc[::5])  # values on bin edges / ties
    sd = r.gamma(1.2, 0.3, n)
    for q, per in ((0.999, 75.0), (0.95, 50.0), (0.5, 100.0), (0.999, 0.0), (0.99, 33.3)):
        got = fet_region_limit(sc, sd, q, per)
        want = ro.filter_limit(sc, sd, q, per)
        assert got[1] == want[1], (n, q, per)  # cmedian
        assert got[2] == want[2], (n, q, per)  # scoreatpercentile
        assert got[3] == want[3] and got[0] == want[0]


@gpu
def test_fet_limit_constant_and_bad():
    from gdscan import GdError
    from gdscan.regions import fet_region_limit
    sc = np.full(17, 2.5)
    got = fet_region_limit(sc, sc, 0.999, 75.0)
    assert got[:3] == ro.filter_limit(sc, sc, 0.999, 75.0)[:3]
    with pytest.raises(GdError):
        fet_region_limit(np.array([1.0, np.nan]), np.ones(2))
    with pytest.raises(GdError):
        fet_region_limit(np.zeros(0), np.zeros(0))
    with pytest.raises(GdError):
        fet_region_limit(np.ones(3), np.ones(3), 0.9, 101.0)


@gpu
@pytest.mark.parametrize("n", [0, 1, 7, 5000, 1_000_003])
def test_fdr_threshold_matches_oracle(n):
    from gdscan.regions import css_fdr_threshold
    r = rng(20 + n)
    p = np.round(r.beta(0.25, 3.0, n), 4)
    if n > 10:
        p[::11] = np.nan
        p[::13] = 1.0
    for fdr in (0.001, 0.05, 0.3):
        want = bh_vectorised(p, fdr) if n > 5000 else ro.bh_threshold(p, fdr)
        assert css_fdr_threshold(p, fdr) == (want[0], want[1]), (n, fdr)


@gpu
def test_top_limit_matches_oracle():
    from gdscan import GdError
    from gdscan.regions import css_top_limit
    r = rng(30)
    s = np.round(r.normal(size=20001), 2)
    s[::97] = np.nan
    s[5] = -0.0
    nn = int(np.isnan(s).sum())
    for k in (1, 2, nn, nn + 1, nn + 50, 1000, 20001, 0, -3):
        got, want = css_top_limit(s, k), ro.top_limit(s, k)
        assert (np.isnan(got) and np.isnan(want)) or got == want, k
    for k in (20002, -20001):
        with pytest.raises(GdError):
            css_top_limit(s, k)


def random_track(r, nseq=5, per=4000):
    seq = np.repeat(np.arange(nseq, dtype=np.int32), per)
    start = np.concatenate([np.sort(r.choice(per * 10, per, replace=False)) * 500 for _ in range(nseq)])
    return seq, start.astype(np.int64)


@gpu
@pytest.mark.parametrize("gap", [500, 2500, 100000])
def test_merge_matches_oracle(gap):
    from gdscan._lib import GD_SELECT_GE, GD_SELECT_LE
    from gdscan.regions import merge_regions
    r = rng(40 + gap)
    seq, start = random_track(r)
    vals = r.random(len(seq))
    ends = np.array([int(start[seq == k].max()) + r.integers(0, 3000) for k in range(5)], np.int64)
    names = [f"c{k}" for k in range(5)]
    for cmp, thr in ((GD_SELECT_GE, 0.9), (GD_SELECT_LE, 0.05), (GD_SELECT_GE, 0.0), (GD_SELECT_GE, 2.0)):
        keep = vals >= thr if cmp == GD_SELECT_GE else vals <= thr
        want = ro.merge_regions([names[k] for k in seq], start, keep, gap, lambda s: int(ends[int(s[1:])]))
        first, end, ns = merge_regions(vals, seq, start, cmp, thr, gap, ends)
        assert ns == int(keep.sum())
        assert list(zip(first.tolist(), end.tolist())) == want


@gpu
def test_merge_rejects_bad_seq():
    from gdscan import GdError
    from gdscan._lib import GD_SELECT_GE
    from gdscan.regions import merge_regions
    with pytest.raises(GdError):
        merge_regions(np.ones(3), np.array([0, 1, 2], np.int32), np.arange(3, dtype=np.int64), GD_SELECT_GE, 0.5,
                      10, np.array([100, 100], np.int64))


@gpu
def test_device_resident_track():
    """torch CUDA tensors go through in place (no host staging)."""
    import torch
    from gdscan._lib import GD_SELECT_LE
    from gdscan.regions import css_fdr_threshold, merge_regions
    r = rng(50)
    seq, start = random_track(r, 3, 20000)
    p = np.round(r.beta(0.2, 4.0, len(seq)), 5)
    ends = np.array([10 ** 8] * 3, np.int64)
    dev = lambda a: torch.from_numpy(a).cuda()
    testp, k = css_fdr_threshold(dev(p), 0.05)
    assert (testp, k) == bh_vectorised(p, 0.05)
    first, end, ns = merge_regions(dev(p), dev(seq), dev(start), GD_SELECT_LE, testp, 2500, dev(ends))
    want = ro.merge_regions(list(seq), start, p <= testp, 2500, lambda s: 10 ** 8)
    assert list(zip(first.tolist(), end.tolist())) == want


def write_track(path, header, seqids, lens, r, pcol):
    from gdscan.gtrack import write_tabular
    write_tabular(path, seqids[0], 500, np.zeros(0), np.zeros(0), header=header, append=False)
    for s, L in zip(seqids, lens):
        n = L // 500
        sc = np.where(r.random(n) < 0.1, 0.0, r.gamma(2.0, 1.0, n))
        other = r.beta(0.3, 3.0, n) if pcol else r.gamma(1.0, 0.2, n)
        write_tabular(path, s, 500, sc, other)


@gpu
def test_filter_fisher_scores_tool(tmp_path):
    from gdscan.regions import filter_fisher_scores
    r = rng(60)
    seqids, lens = ["chr1", "chr2", "chrX"], [2_000_000, 1_500_000, 900_000]
    src = tmp_path / "fet.tabular"
    write_track(src, "#seqid\tstart\tscore\tstddev", seqids, lens, r, False)
    cl = dict(zip(seqids, lens))
    for ws, q, per in ((100000, 0.999, 75.0), (2500, 0.9, 50.0), (500, 0.5, 10.0)):
        out = tmp_path / "fet.gtrack"
        filter_fisher_scores(src, out, cl, ws, q, per)
        assert out.read_text() == ro.filter_fisher_scores_text(src.read_text(), cl, ws, q, per)


@gpu
def test_significant_css_regions_tool(tmp_path):
    from gdscan.regions import significant_css_regions
    r = rng(70)
    seqids, lens = ["chr1", "chr2"], [3_000_000, 1_000_000]
    src = tmp_path / "css.tabular"
    write_track(src, "#seqid\tstart\tscore\tp", seqids, lens, r, True)
    cl = dict(zip(seqids, lens))
    text = src.read_text()
    for kw in ({"fdr": 0.05}, {"fdr": 0.2}, {"fdr": 1e-9}, {"num_top": 1}, {"num_top": 100}, {"num_top": 5000}):
        out = tmp_path / "css.gtrack"
        significant_css_regions(src, out, cl, window_size=2500, **kw)
        assert out.read_text() == ro.significant_css_regions_text(text, cl, window_size=2500, **kw), kw
