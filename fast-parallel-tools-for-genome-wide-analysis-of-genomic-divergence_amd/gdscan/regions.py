"""Divergent regions from a finished score track, on the device.

filter_fisher_scores     <- tools/FilterFisherScores.py:55-115 (execute)
significant_css_regions  <- tools/SignificantCSSRegions.py:78-154 (execute)

The statistics behind them are C-ABI calls (include/gdscan.h, csrc/gd_regions.hip):
fet_region_limit (cmedian + scoreatpercentile), css_fdr_threshold (Benjamini-Hochberg),
css_top_limit, merge_regions.  Their array arguments may be numpy arrays (staged
through the library) or CUDA torch tensors (used in place), so a track produced by
gd_*_scan_device never has to leave HBM.

The tools print progress to stdout; these functions return the same numbers instead.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import GD_SELECT_GE, GD_SELECT_LE, check, lib
from .gtrack import py2_str

FET_SEGMENTS_HEADER = ("##gtrack version: 1.0\n##track type: segments\n##uninterrupted data lines: true\n"
                       "##sorted elements: false\n##no overlapping elements: true\n###seqid\tstart\tend\n")
CSS_SEGMENTS_HEADER = ("##gtrack version: 1.0\n##track type: segments\n##uninterrupted data lines: true\n"
                       "##no overlapping elements: true\n###seqid\tstart\tend\n")


def _arg(x, dtype):
    """(pointer, n, keepalive) for a numpy array or a CUDA torch tensor."""
    if hasattr(x, "data_ptr") and hasattr(x, "is_cuda"):
        import torch
        tdt = {np.float64: torch.float64, np.int32: torch.int32, np.int64: torch.int64}[dtype]
        if x.dtype != tdt:
            raise ValueError(f"expected {tdt}, got {x.dtype}")
        x = x.contiguous()
        return x.data_ptr(), x.numel(), x
    a = np.ascontiguousarray(x, dtype=dtype)
    return a.ctypes.data, a.shape[0], a


def read_tabular(path):
    """The tools' result file -> (seqids, seq int32, start int64, col2 f64, col3 f64)."""
    t = lib.gd_tabular_read(str(path).encode())
    if not t:
        check(-1)
    try:
        n = lib.gd_tabular_rows(t)
        seqids = [lib.gd_tabular_seqid(t, s).decode() for s in range(lib.gd_tabular_nseq(t))]
        seq, start = np.empty(n, np.int32), np.empty(n, np.int64)
        c2, c3 = np.empty(n, np.float64), np.empty(n, np.float64)
        check(lib.gd_tabular_copy(t, seq.ctypes.data, start.ctypes.data, c2.ctypes.data, c3.ctypes.data))
    finally:
        lib.gd_tabular_free(t)
    return seqids, seq, start, c2, c3


def fet_region_limit(scores, stddev, normquantile=0.999, percentile=75.0, ctx=None, stream=None):
    """FilterFisherScores.py:84-87 -> (limit, median, upperquant, qnorm)."""
    from scipy import stats
    qnorm = float(stats.norm.ppf(normquantile))
    ps, n, k1 = _arg(scores, np.float64)
    pd, n2, k2 = _arg(stddev, np.float64)
    if n != n2:
        raise ValueError("scores and stddev differ in length")
    out = (C.c_double * 3)()
    check(lib.gd_fet_region_limit(ctx, ps, pd, n, qnorm, float(percentile), out, stream))
    return out[0], out[1], out[2], qnorm


def css_fdr_threshold(p, fdr, ctx=None, stream=None):
    """SignificantCSSRegions.py:104-114 -> (testp, k); k == 0: no window passes."""
    pp, n, keep = _arg(p, np.float64)
    testp, k = C.c_double(), C.c_int64()
    check(lib.gd_css_fdr_threshold(ctx, pp, n, float(fdr), C.byref(testp), C.byref(k), stream))
    return testp.value, k.value


def css_top_limit(scores, num_top, ctx=None, stream=None):
    """SignificantCSSRegions.py:125-126: the num_top-th highest score (NaN ranks first)."""
    ps, n, keep = _arg(scores, np.float64)
    lim = C.c_double()
    check(lib.gd_css_top_limit(ctx, ps, n, int(num_top), C.byref(lim), stream))
    return lim.value


def merge_regions(vals, seq, start, cmp, thr, max_gap, seq_end, ctx=None, stream=None):
    """Keep vals >= thr (cmp GD_SELECT_GE) or <= thr (GD_SELECT_LE) and merge into
    segments (FilterFisherScores.py:97-114) -> (first window index, end, n selected)."""
    pv, n, k1 = _arg(vals, np.float64)
    pq, n2, k2 = _arg(seq, np.int32)
    pst, n3, k3 = _arg(start, np.int64)
    pe, nseq, k4 = _arg(seq_end, np.int64)
    if not n == n2 == n3:
        raise ValueError("vals, seq and start differ in length")
    first, end = np.empty(max(n, 1), np.int64), np.empty(max(n, 1), np.int64)
    nr, ns = C.c_int64(), C.c_int64()
    check(lib.gd_merge_regions(ctx, pv, pq, pst, n, int(cmp), float(thr), int(max_gap), pe, nseq,
                               first.ctypes.data, end.ctypes.data, C.byref(nr), C.byref(ns), stream))
    return first[:nr.value], end[:nr.value], ns.value


def _seq_end(seqids, chrom_lengths):
    try:
        return np.array([int(chrom_lengths[s]) - 1 for s in seqids] or [0], np.int64)
    except KeyError as e:
        raise KeyError(f"no chromosome length for {e.args[0]!r}") from None


def _write_segments(out_path, header, seqids, seq, start, first, end, window_size):
    with open(out_path, "w") as f:
        f.write(header)
        if len(first) == 0:  # no window kept: the tools still close an empty region
            f.write("\t" + py2_str(-1000000.0 + window_size) + "\n")
            return
        f.write("".join(f"{seqids[seq[i]]}\t{start[i]}\t{e}\n" for i, e in zip(first.tolist(), end.tolist())))


def filter_fisher_scores(in_path, out_path, chrom_lengths, window_size=100000, normquantile=0.999, percentile=75.0):
    """FilterFisherScores.execute: FET result file -> GTrack segments of high-score windows.
    Returns {limit, median, upperquant, qnorm, windows, regions}."""
    seqids, seq, start, fet, sd = read_tabular(in_path)
    limit, med, upq, qnorm = fet_region_limit(fet, sd, normquantile, percentile)
    first, end, ns = merge_regions(fet, seq, start, GD_SELECT_GE, limit, window_size,
                                   _seq_end(seqids, chrom_lengths))
    _write_segments(out_path, FET_SEGMENTS_HEADER, seqids, seq, start, first, end, window_size)
    return {"limit": limit, "median": med, "upperquant": upq, "qnorm": qnorm, "windows": ns,
            "regions": len(first)}


def significant_css_regions(in_path, out_path, chrom_lengths, fdr=None, num_top=None, window_size=2500):
    """SignificantCSSRegions.execute: CSS result file -> GTrack segments, by a BH-FDR
    p threshold (fdr=...) or the num_top best scores (num_top=...).
    Returns {testp | limit, windows, regions}."""
    if (fdr is None) == (num_top is None):
        raise ValueError("give exactly one of fdr / num_top")
    seqids, seq, start, scores, p = read_tabular(in_path)
    if fdr is not None:
        testp, k = css_fdr_threshold(p, fdr)
        if k == 0:
            with open(out_path, "w") as f:
                f.write("NONE found")
            return {"testp": testp, "k": 0, "windows": 0, "regions": 0}
        first, end, ns = merge_regions(p, seq, start, GD_SELECT_LE, testp, window_size,
                                       _seq_end(seqids, chrom_lengths))
        info = {"testp": testp, "k": k, "false_discoveries": testp * len(p)}
    else:
        limit = css_top_limit(scores, num_top)
        first, end, ns = merge_regions(scores, seq, start, GD_SELECT_GE, limit, window_size,
                                       _seq_end(seqids, chrom_lengths))
        info = {"limit": limit}
    _write_segments(out_path, CSS_SEGMENTS_HEADER, seqids, seq, start, first, end, window_size)
    info.update(windows=ns, regions=len(first))
    return info
