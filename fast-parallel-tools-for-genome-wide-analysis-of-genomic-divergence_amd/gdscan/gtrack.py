"""HyperBrowser track I/O around the scan.

read_gtrack       GTrack "valued points" file -> per-seqid (starts int32, vals float64),
                  the arrays HyperBrowser's startsAsNumpyArray / valsAsNumpyArray give the
                  statistics (native parser in lib/libgdscan.so, gd_gtrack.cpp).
read_gtrack_packed  the same file parsed straight into packed genotype tracks (2-bit
                  codes, one position per row; gd_ptrack_read), no f64 intermediate.
write_tabular     the tools' result lines (FisherExactTestSNPTool.py:162-189,
                  ClusterSeparationScore.py:180-205), floats as Python 2 str() (Q11).
vcf_to_gtrack     restatement of tools/VCFConvert.py:2-86 (genotype -> 3 / 0 / -3 / -10000).
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np

from ._lib import GD_ERR_NOPACK, GdError, check, lib

# VCFConvert.py:9-18
GT_VALUES = {"./.": -10000, ".|.": -10000, "1/0": 0, "0/1": 0, "1|0": 0, "0|1": 0, "0/0": 3, "0|0": 3,
             "1/1": -3, "1|1": -3}


def read_gtrack(path) -> "OrderedDict[str, tuple[np.ndarray, np.ndarray]]":
    """seqid -> (starts int32, vals float64), sequences in first-seen order, lines in file order."""
    h = lib.gd_gtrack_read(str(path).encode())
    if not h:
        raise GdError(-1, lib.gd_last_error().decode(errors="replace"))
    try:
        out = OrderedDict()
        for s in range(lib.gd_gtrack_nseq(h)):
            n = lib.gd_gtrack_len(h, s)
            starts = np.empty(n, dtype=np.int32)
            vals = np.empty(n, dtype=np.float64)
            check(lib.gd_gtrack_copy(h, s, starts.ctypes.data, vals.ctypes.data))
            out[lib.gd_gtrack_seqid(h, s).decode()] = (starts, vals)
        return out
    finally:
        lib.gd_gtrack_free(h)


def read_gtrack_packed(path) -> "OrderedDict[str, tuple[np.ndarray, np.ndarray, int]]":
    """seqid -> (rowpos int32 [nrows], codes uint64 [nrows * words(size)], size): the
    packed form of read_gtrack's arrays (gdscan.packed layout).  ValueError for a track
    with no packed form (a value other than 3, 0, -3, -10000, or positions not in whole
    rows of get_population_size() individuals); GdError for an unreadable file."""
    h = lib.gd_ptrack_read(str(path).encode())
    if not h:
        msg = lib.gd_last_error().decode(errors="replace")
        st = lib.gd_last_status()
        if st == GD_ERR_NOPACK:  # readable, but no packed form: callers fall back to read_gtrack
            raise ValueError(msg)
        raise GdError(st, msg)
    try:
        out = OrderedDict()
        size, nrows = C.c_int32(), C.c_int64()
        for s in range(lib.gd_ptrack_nseq(h)):
            check(lib.gd_ptrack_shape(h, s, C.byref(size), C.byref(nrows)))
            rowpos = np.empty(nrows.value, dtype=np.int32)
            codes = np.empty(nrows.value * ((size.value + 31) // 32), dtype=np.uint64)
            check(lib.gd_ptrack_copy(h, s, codes.ctypes.data, rowpos.ctypes.data))
            out[lib.gd_ptrack_seqid(h, s).decode()] = (rowpos, codes, size.value)
        return out
    finally:
        lib.gd_ptrack_free(h)


def py2_str(x: float) -> str:
    """Python 2's str(float): '%.12g', '.0' appended to integral text."""
    buf = C.create_string_buffer(64)
    lib.gd_format_py2_float(float(x), buf, 64)
    return buf.value.decode()


def write_tabular(path, seqid, wstep, scores, other, header=None, append=True):
    """Append one chromosome's windows with score != 0 (optionally after a header line)."""
    scores = np.ascontiguousarray(scores, dtype=np.float64)
    other = np.ascontiguousarray(other, dtype=np.float64)
    if scores.shape != other.shape:
        raise ValueError("scores and the second column must have the same length")
    check(lib.gd_write_tabular(str(path).encode(), int(append), header.encode() if header else None,
                               str(seqid).encode(), int(wstep), scores.shape[0], scores.ctypes.data,
                               other.ctypes.data))


def gtrack_header(genome: str) -> str:
    """VCFConvert.addHeader (VCFConvert.py:53-57)."""
    return ("##gtrack version: 1.0\n##track type: valued points\n##value type: number\n"
            "###seqid\tstart\tvalue\tgenomeid\n####genome=%s\n" % genome)


def vcf_to_gtrack(vcf_text: str, pop, genome: str = "test") -> str:
    """VCFConvert.convertToGtrackFile + addHeader: one line per (SNP, individual of `pop`
    found in the #CHROM header), values from GT_VALUES.  Individuals missing from the
    header are dropped, as the reference does (VCFConvert.py:59-71)."""
    lines = vcf_text.strip().split("\n")
    idx = 0
    while not lines[idx].startswith("#CHROM"):
        idx += 1
    header = lines[idx].split("\t")
    chromidx, posidx, formatidx = header.index("#CHROM"), header.index("POS"), header.index("FORMAT")
    names = [p for p in pop if p in header]
    popidx = [header.index(p) for p in names]
    gtidx = lines[idx + 1].split("\t")[formatidx].split(":").index("GT")
    out = [gtrack_header(genome)]
    for line in lines[idx + 1:]:
        words = line.split("\t")
        for k, col in enumerate(popidx):
            gt = words[col].split(":")[gtidx]
            if gt not in GT_VALUES:
                raise ValueError(f"genotype {gt!r} has no GTrack value (VCFConvert.py:9-18)")
            out.append("%s\t%s\t%s\t%s\n" % (words[chromidx], words[posidx], GT_VALUES[gt], names[k]))
    return "".join(out)
