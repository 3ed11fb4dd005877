"""Packed genotype tracks: the four values VCFConvert.py:8-17
writes (3, 0, -3, -10000) as 2-bit codes, one position per SNP row.

A reference-layout chromosome (what HyperBrowser hands FisherExactScoreStat._compute:
float64 values and int32 positions per (SNP row, individual), SNP-major) packs into
``PackedChrom`` -- 2 bits per genotype + 4 bytes per row instead of 12 bytes per
genotype -- when its rows are whole (every individual of a row, A and B alike, at the
row's position) and every value is one of the four codes; anything else raises
ValueError and stays in the reference layout.  ``fet_scan`` / ``css_scan`` scan a list
of packed chromosomes on the GPU (libgdscan.so, gd_*_scan_packed_host) with exactly
the windows, scores and seeded bootstrap / permutation streams of the reference-layout
scans (gdscan.fet.scan / gdscan.css.scan) of the same tracks.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import GD_ERR_ARG, GD_FET_EXACT, GD_FET_REFERENCE, GD_OK, GD_WINDOWS_SERIAL, GD_WINDOWS_THREADED, \
    GdError, PChrom, check, lib

CODE_HET, CODE_MAJOR, CODE_MINOR, CODE_MISSING = 0, 1, 2, 3
VALUES = np.array([0.0, 3.0, -3.0, -10000.0])  # value of each code


def words(size):
    """uint64 words per row of one population (GD_PACK_WORDS)."""
    return (int(size) + 31) // 32


@dataclass
class PackedChrom:
    acodes: np.ndarray   # uint64 [nrows * words(asize)]
    bcodes: np.ndarray   # uint64 [nrows * words(bsize)]
    rowpos: np.ndarray   # int32 [nrows]
    asize: int
    bsize: int
    regend: int

    @property
    def nrows(self):
        return int(self.rowpos.shape[0])

    def unpack(self):
        """The reference layout back: (avals, bvals, apos, bpos)."""
        out = []
        for codes, size in ((self.acodes, self.asize), (self.bcodes, self.bsize)):
            w = codes.reshape(self.nrows, words(size))
            k = np.arange(size)
            c = (w[:, k // 32] >> (2 * (k % 32)).astype(np.uint64)) & np.uint64(3)
            out.append(VALUES[c.astype(np.int64)].ravel())
        return out[0], out[1], np.repeat(self.rowpos, self.asize), np.repeat(self.rowpos, self.bsize)


def shape(apos, bpos):
    """(asize, bsize, nrows): get_population_size() of both tracks and the whole rows both hold."""
    ap = np.ascontiguousarray(apos, dtype=np.int32)
    bp = np.ascontiguousarray(bpos, dtype=np.int32)
    a, b, n = C.c_int(), C.c_int(), C.c_int()
    ip = C.POINTER(C.c_int)
    st = lib.gd_pack_shape(ap.ctypes.data_as(ip), bp.ctypes.data_as(ip), ap.shape[0], bp.shape[0], C.byref(a),
                           C.byref(b), C.byref(n))
    if st == GD_ERR_ARG and n.value >= 0 and a.value > 0 and b.value > 0:
        raise ValueError("the tracks do not consist of whole rows of asize / bsize individuals "
                         f"({a.value} + {b.value} individuals, {ap.shape[0]} + {bp.shape[0]} elements)")
    check(st)
    return a.value, b.value, n.value


def pack(avals, bvals, apos, bpos, regend):
    """Pack one reference-layout chromosome (host, libgdscan's gd_pack_chrom)."""
    av = np.ascontiguousarray(avals, dtype=np.float64)
    bv = np.ascontiguousarray(bvals, dtype=np.float64)
    ap = np.ascontiguousarray(apos, dtype=np.int32)
    bp = np.ascontiguousarray(bpos, dtype=np.int32)
    asize, bsize, nrows = shape(ap, bp)
    if nrows * asize != av.shape[0] or nrows * bsize != bv.shape[0]:
        raise ValueError("the tracks do not consist of whole rows of asize / bsize individuals")
    ac = np.zeros(nrows * words(asize), dtype=np.uint64)
    bc = np.zeros(nrows * words(bsize), dtype=np.uint64)
    rp = np.zeros(nrows, dtype=np.int32)
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int)
    st = lib.gd_pack_chrom(av.ctypes.data_as(dp), bv.ctypes.data_as(dp), ap.ctypes.data_as(ip),
                           bp.ctypes.data_as(ip), asize, bsize, nrows, ac.ctypes.data, bc.ctypes.data, rp.ctypes.data)
    if st == GD_ERR_ARG:
        raise ValueError(lib.gd_last_error().decode(errors="replace"))
    check(st)
    return PackedChrom(ac, bc, rp, asize, bsize, int(regend))


def read_pair(track_a, track_b, chrom_lengths=None):
    """Two population GTrack files read straight into packed chromosomes
    (gtrack.read_gtrack_packed): (names, [PackedChrom]) for the sequences of A, in A's
    order, that B also holds -- the chromosomes gdscan.tools scans, region
    [0, chrom_lengths[seqid]) or [0, last position + 1).  ValueError when either file, or
    a shared sequence of the pair (different rows in A and B), has no packed form."""
    from .gtrack import read_gtrack_packed
    ta, tb = read_gtrack_packed(track_a), read_gtrack_packed(track_b)
    names, chroms = [], []
    for s, (pa, ca, na) in ta.items():
        if s not in tb or pa.shape[0] == 0:
            continue
        pb, cb, nb = tb[s]
        if pa.shape[0] != pb.shape[0] or not np.array_equal(pa, pb):
            raise ValueError(f"sequence {s}: the rows of A and B are not at the same positions "
                             f"({pa.shape[0]} and {pb.shape[0]} rows); the pair keeps the reference layout")
        regend = int(chrom_lengths[s]) if chrom_lengths and s in chrom_lengths else int(pa[-1]) + 1
        names.append(s)
        chroms.append(PackedChrom(ca, cb, pa, int(na), int(nb), regend))
    return names, chroms


def _batch(chroms, wstep, seed):
    """Concatenated codes / positions and the gd_pchrom descriptors; window outputs of
    chromosome c start at the running sum of regend // wstep."""
    n = len(chroms)
    desc = (PChrom * max(n, 1))()
    row = aw = bw = wo = 0
    for c, pc in enumerate(chroms):
        d = desc[c]
        d.row_off, d.a_word, d.b_word = row, aw, bw
        d.nrows, d.asize, d.bsize, d.regend = pc.nrows, pc.asize, pc.bsize, pc.regend
        d.w_out = wo
        d.seed = lib.gd_get_seed() if seed is None else int(seed)
        row += pc.nrows
        aw += pc.acodes.shape[0]
        bw += pc.bcodes.shape[0]
        wo += pc.regend // int(wstep)
    cat = lambda xs, t: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(1, t), dtype=t)
    return (desc, cat([p.acodes for p in chroms], np.uint64), cat([p.bcodes for p in chroms], np.uint64),
            cat([p.rowpos for p in chroms], np.int32), wo)


def _split(out, chroms, wstep):
    res, o = [], 0
    for pc in chroms:
        k = pc.regend // int(wstep)
        res.append(out[o:o + k])
        o += k
    return res


def fet_scan(chroms, wsize=2500, wstep=500, perc=0.95, seed=None, serial=False, exact=None):
    """FET scan of packed chromosomes -> [(scores, stddev)] per chromosome."""
    desc, ac, bc, rp, nw = _batch(chroms, wstep, seed)
    scores, stddev = np.zeros(max(nw, 1)), np.zeros(max(nw, 1))
    mode = lib.gd_get_fet_mode() if exact is None else (GD_FET_EXACT if exact else GD_FET_REFERENCE)
    dp = C.POINTER(C.c_double)
    check(lib.gd_fet_scan_packed_host(desc, len(chroms), ac.ctypes.data, bc.ctypes.data, rp.ctypes.data, int(wsize),
                                      int(wstep), float(perc), mode,
                                      GD_WINDOWS_SERIAL if serial else GD_WINDOWS_THREADED,
                                      scores.ctypes.data_as(dp), stddev.ctypes.data_as(dp)))
    return list(zip(_split(scores, chroms, wstep), _split(stddev, chroms, wstep)))


def css_scan(chroms, wsize=2500, wstep=500, treshold=10, runs=0, mds=0, seed=None, serial=False):
    """CSS scan (count metric) of packed chromosomes -> [(scores, p)] per chromosome."""
    desc, ac, bc, rp, nw = _batch(chroms, wstep, seed)
    scores, p = np.zeros(max(nw, 1)), np.zeros(max(nw, 1))
    dp = C.POINTER(C.c_double)
    check(lib.gd_css_scan_packed_host(desc, len(chroms), ac.ctypes.data, bc.ctypes.data, rp.ctypes.data, int(wsize),
                                      int(wstep), int(treshold), int(runs), int(mds),
                                      GD_WINDOWS_SERIAL if serial else GD_WINDOWS_THREADED,
                                      scores.ctypes.data_as(dp), p.ctypes.data_as(dp)))
    return list(zip(_split(scores, chroms, wstep), _split(p, chroms, wstep)))


__all__ = ["PackedChrom", "shape", "pack", "fet_scan", "css_scan", "words", "CODE_HET", "CODE_MAJOR", "CODE_MINOR",
           "CODE_MISSING", "GD_OK", "GdError"]
