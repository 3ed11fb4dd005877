"""End-to-end tools: two population GTrack files in, the HyperBrowser tools' tabular
result out, every chromosome scanned in one device batch.

fisher_exact_test_snp       <- tools/FisherExactTestSNPTool.py:140-189 (execute)
cluster_separation_score    <- tools/ClusterSeparationScore.py:150-205 (execute)

Differences from the Galaxy tools: chromosomes come in the order track A lists them
(HyperBrowser iterates the genome's chromosome list); the region of a chromosome is
[0, chrom_lengths[seqid]) when given, else [0, last position + 1) (HyperBrowser uses
the genome build's chromosome length).

Seeds: every chromosome's bootstrap / permutation stream derives from `seed` (default: the
calling thread's gd_set_seed value -- the library keeps one seed per thread, so a worker
thread that should follow the main thread's setting passes seed= explicitly).
"""
from __future__ import annotations

import numpy as np

from ._lib import GD_WINDOWS_THREADED, Chrom, check, lib
from .gtrack import read_gtrack, write_tabular


def _seed(seed):
    return lib.gd_get_seed() if seed is None else int(seed)


def _batch(track_a, track_b, wstep, chrom_lengths, seed=None):
    ta, tb = read_gtrack(track_a), read_gtrack(track_b)
    names = [s for s in ta if s in tb and len(ta[s][0]) > 0]
    chroms = (Chrom * max(len(names), 1))()
    av, bv, ap, bp = [], [], [], []
    off_a = off_b = w = 0
    for c, s in enumerate(names):
        (pa, va), (pb, vb) = ta[s], tb[s]
        regend = int(chrom_lengths[s]) if chrom_lengths and s in chrom_lengths else \
            int(max(pa[-1], pb[-1] if len(pb) else 0)) + 1
        chroms[c].a_off, chroms[c].b_off = off_a, off_b
        chroms[c].alen, chroms[c].blen = len(va), len(vb)
        chroms[c].regend, chroms[c].w_out = regend, w
        chroms[c].seed = _seed(seed)
        av.append(va); bv.append(vb); ap.append(pa); bp.append(pb)
        off_a += len(va); off_b += len(vb); w += regend // wstep
    cat = lambda xs, dt: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(0), dtype=dt)
    return names, chroms, cat(av, np.float64), cat(bv, np.float64), cat(ap, np.int32), cat(bp, np.int32), w


def _write(out_path, header, names, regends, wstep, s0, s1):
    write_tabular(out_path, names[0] if names else "", wstep, np.zeros(0), np.zeros(0), header=header, append=False)
    lo = 0
    for s, regend in zip(names, regends):
        n = regend // wstep
        write_tabular(out_path, s, wstep, s0[lo:lo + n], s1[lo:lo + n])
        lo += n


def _packed_pair(track_a, track_b, chrom_lengths, packed):
    """The pair read straight into packed chromosomes (packed.read_pair) when `packed` is
    True, or "auto" and both files have a packed form; None selects the reference layout."""
    if packed is False:
        return None
    if packed not in (True, "auto"):
        raise ValueError(f"packed must be True, False or 'auto', not {packed!r}")
    from .packed import read_pair
    try:
        return read_pair(track_a, track_b, chrom_lengths)
    except ValueError:
        if packed is True:
            raise
        return None


def _ptr(a, ct):
    import ctypes as C
    return a.ctypes.data_as(C.POINTER(ct))


def fisher_exact_test_snp(track_a, track_b, out_path, wsize=2500, wstep=500, percentile=0.95, chrom_lengths=None,
                          exact=None, packed="auto", seed=None):
    """packed: "auto" reads genotype tracks straight into 2-bit codes (gdscan.packed; same
    windows, scores and bootstrap streams) and falls back to the reference layout for
    tracks with no packed form; True requires the packed form, False never uses it.
    seed: the bootstrap seed (None: this thread's gd_set_seed value)."""
    import ctypes as C
    pair = _packed_pair(track_a, track_b, chrom_lengths, packed)
    if pair is not None:
        from . import packed as pk
        names, pcs = pair
        res = pk.fet_scan(pcs, wsize, wstep, percentile, seed=_seed(seed), exact=exact) if names else []
        scores = np.concatenate([r[0] for r in res]) if res else np.zeros(0)
        stddev = np.concatenate([r[1] for r in res]) if res else np.zeros(0)
        _write(out_path, "#seqid\tstart\tscore\tstddev", names, [p.regend for p in pcs], wstep, scores, stddev)
        return names, scores, stddev
    names, chroms, av, bv, ap, bp, w = _batch(track_a, track_b, wstep, chrom_lengths, seed)
    scores, stddev = np.zeros(w), np.zeros(w)
    if names:
        mode = lib.gd_get_fet_mode() if exact is None else int(bool(exact))  # GD_FET_REFERENCE / GD_FET_EXACT
        check(lib.gd_fet_scan_host_batch_ex(chroms, len(names), _ptr(av, C.c_double), _ptr(bv, C.c_double),
                                            _ptr(ap, C.c_int), _ptr(bp, C.c_int), int(wsize), int(wstep),
                                            float(percentile), mode, GD_WINDOWS_THREADED,
                                            _ptr(scores, C.c_double), _ptr(stddev, C.c_double)))
    _write(out_path, "#seqid\tstart\tscore\tstddev", names, [chroms[c].regend for c in range(len(names))], wstep,
           scores, stddev)
    return names, scores, stddev


# ClusterSeparationScore.py:167-173: the distance metric and MDS choices of the tool
COMPARE = {"count": 0, "Count individual SNP-differences in window": 0, "freq": 1}
MDS = {"classical": 0, "Classical MDS": 0, "smacof": 1, "SMACOF": 1, "smacof+cmds": 2}


def cluster_separation_score(track_a, track_b, out_path, wsize=2500, wstep=500, mc_treshold=10, mc_runs=0,
                             compare="count", mds="classical", chrom_lengths=None, packed="auto", seed=None):
    """compare: "count" (SNP differences) or "freq" (drosophila allele-frequency metric,
    one frequency track per population); mds: "classical", "smacof" or "smacof+cmds"
    (any other label selects SMACOF + classical, as the tool's else branch does);
    packed: as fisher_exact_test_snp (the count metric only: "freq" tracks hold
    frequencies, never genotype codes); seed: the permutation seed (None: this thread's
    gd_set_seed value)."""
    import ctypes as C
    if compare not in COMPARE:
        raise ValueError(f"unknown distance metric {compare!r}")
    dro, md = COMPARE[compare], MDS.get(mds, 2)
    pair = _packed_pair(track_a, track_b, chrom_lengths, packed) if dro == 0 else None
    if dro and packed is True:
        raise ValueError("the freq metric has no packed form")
    if pair is not None:
        from . import packed as pk
        names, pcs = pair
        res = pk.css_scan(pcs, wsize, wstep, mc_treshold, mc_runs, md, seed=_seed(seed)) if names else []
        scores = np.concatenate([r[0] for r in res]) if res else np.zeros(0)
        p = np.concatenate([r[1] for r in res]) if res else np.zeros(0)
        _write(out_path, "#seqid\tstart\tscore\tp", names, [c.regend for c in pcs], wstep, scores, p)
        return names, scores, p
    names, chroms, av, bv, ap, bp, w = _batch(track_a, track_b, wstep, chrom_lengths, seed)
    scores, p = np.zeros(w), np.zeros(w)
    if names:
        check(lib.gd_css_scan_host_batch_ex(chroms, len(names), _ptr(av, C.c_double), _ptr(bv, C.c_double),
                                            _ptr(ap, C.c_int), _ptr(bp, C.c_int), int(wsize), int(wstep),
                                            int(mc_treshold), int(mc_runs), dro, md, GD_WINDOWS_THREADED,
                                            _ptr(scores, C.c_double), _ptr(p, C.c_double)))
    _write(out_path, "#seqid\tstart\tscore\tp", names, [chroms[c].regend for c in range(len(names))], wstep,
           scores, p)
    return names, scores, p
