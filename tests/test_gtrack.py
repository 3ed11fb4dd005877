"""CPU: HyperBrowser track I/O (gdscan.gtrack).  The reference
ships no track files, so the conversions are checked against outputs derived by hand
from the reference's code (VCFConvert.py, the tools' write loops)."""
import math

import numpy as np
import pytest


def _py2(x):
    """Python 2.7 str(float) = PyOS_double_to_string(x, 'g', 12, Py_DTSF_ADD_DOT_0)."""
    if math.isnan(x):
        return "nan"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    s = "%.12g" % x
    return s if ("." in s or "e" in s) else s + ".0"


@pytest.mark.parametrize("x,want", [(3.0, "3.0"), (0.1, "0.1"), (1e16, "1e+16"), (2.8722813232690143, "2.87228132327"),
                                    (12345678901234.5, "1.23456789012e+13"), (-0.0, "-0.0"), (1e-5, "1e-05"),
                                    (float("nan"), "nan"), (float("inf"), "inf"), (-2.5, "-2.5"),
                                    (70.5975410337, "70.5975410337"), (0.0011410518554900925, "0.00114105185549")])
def test_py2_float_text(x, want):
    from gdscan.gtrack import py2_str
    assert py2_str(x) == want == _py2(x)


VCF = """##fileformat=VCFv4.1
##source=test
#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tind1\tind2\tind3
chrA\t101\t.\tA\tG\t50\tPASS\t.\tGT:DP\t0/0:10\t0/1:12\t1/1:7
chrA\t205\t.\tC\tT\t50\tPASS\t.\tGT:DP\t./.:0\t1|1:9\t0|0:3
chrB\t17\t.\tG\tA\t50\tPASS\t.\tGT:DP\t1|0:4\t0/0:8\t.|.:0
"""


def test_vcf_to_gtrack_matches_reference_encoding():
    from gdscan.gtrack import vcf_to_gtrack
    out = vcf_to_gtrack(VCF, ["ind3", "missing", "ind1"], genome="g1")
    want = ("##gtrack version: 1.0\n##track type: valued points\n##value type: number\n"
            "###seqid\tstart\tvalue\tgenomeid\n####genome=g1\n"
            "chrA\t101\t-3\tind3\nchrA\t101\t3\tind1\n"
            "chrA\t205\t3\tind3\nchrA\t205\t-10000\tind1\n"
            "chrB\t17\t-10000\tind3\nchrB\t17\t0\tind1\n")
    assert out == want


def test_read_gtrack_roundtrip(tmp_path):
    from gdscan import synth
    from gdscan.gtrack import gtrack_header, read_gtrack
    av, bv, ap, bp, regend = synth.chromosome(3, 2000, 5, 5)
    lines = [gtrack_header("g")]
    for chrom, (pos, val) in (("chr2", (ap[:5000], av[:5000])), ("chr10", (ap[5000:], av[5000:]))):
        for k in range(len(pos)):
            lines.append("%s\t%d\t%d\tind%d\n" % (chrom, pos[k], val[k], k % 5))
    f = tmp_path / "a.gtrack"
    f.write_text("".join(lines).replace("\n", "\r\n", 3))
    t = read_gtrack(f)
    assert list(t) == ["chr2", "chr10"]
    assert np.array_equal(t["chr2"][0], ap[:5000]) and np.array_equal(t["chr2"][1], av[:5000])
    assert t["chr10"][0].dtype == np.int32 and t["chr10"][1].dtype == np.float64
    assert np.array_equal(t["chr10"][0], ap[5000:]) and np.array_equal(t["chr10"][1], av[5000:])


def test_read_gtrack_column_order_and_floats(tmp_path):
    from gdscan.gtrack import read_gtrack
    f = tmp_path / "b.gtrack"
    f.write_text("##gtrack version: 1.0\n###value\tgenomeid\tstart\tseqid\n"
                 "1.5\tx\t10\tc1\n-3\ty\t10\tc1\n2e3\tx\t11\tc2\nnan\ty\t11\tc1\n")
    t = read_gtrack(f)
    assert np.array_equal(t["c1"][0], [10, 10, 11])
    v = t["c1"][1]
    assert v[0] == 1.5 and v[1] == -3 and np.isnan(v[2])
    assert t["c2"][1][0] == 2000.0


def test_read_gtrack_errors(tmp_path):
    from gdscan import GdError
    from gdscan.gtrack import read_gtrack
    with pytest.raises(GdError):
        read_gtrack(tmp_path / "nope.gtrack")
    f = tmp_path / "bad.gtrack"
    f.write_text("###seqid\tstart\tvalue\nc1\tten\t3\n")
    with pytest.raises(GdError):
        read_gtrack(f)


def _track_file(path, seqs, size):
    """seqs: [(name, positions per element, values per element)] -> a GTrack file"""
    from gdscan.gtrack import gtrack_header
    lines = [gtrack_header("g")]
    for name, pos, val in seqs:
        lines += ["%s\t%d\t%d\tind%d\n" % (name, pos[k], val[k], k % size) for k in range(len(pos))]
    path.write_text("".join(lines))
    return path


@pytest.mark.parametrize("chunk", [None, "4096", "777"])
@pytest.mark.parametrize("size", [5, 32, 33, 70])
def test_read_gtrack_packed_equals_pack_of_read_gtrack(tmp_path, monkeypatch, chunk, size):
    """gd_ptrack_read against gd_pack_chrom of gd_gtrack_read's arrays, with the file cut
    into many parser chunks (GD_GTRACK_CHUNK bytes per thread: rows and words split
    across chunks), sequences interleaved and revisited."""
    from gdscan import packed, synth
    from gdscan.gtrack import read_gtrack, read_gtrack_packed
    av, bv, ap, bp, _ = synth.chromosome(11, 600, size, size)
    n = len(ap)
    cut = (n // size // 3) * size
    seqs = [("chrX", ap[:cut], av[:cut]), ("chr7", bp[:cut], bv[:cut]), ("chrX", ap[cut:], av[cut:]),
            ("chr7", bp[cut:], bv[cut:])]
    f = _track_file(tmp_path / "t.gtrack", seqs, size)
    if chunk:
        monkeypatch.setenv("GD_GTRACK_CHUNK", chunk)
    ref, got = read_gtrack(f), read_gtrack_packed(f)
    assert list(got) == list(ref) == ["chrX", "chr7"]
    for s in ref:
        pos, val = ref[s]
        pc = packed.pack(val, val, pos, pos, int(pos[-1]) + 1)
        rowpos, codes, sz = got[s]
        assert sz == size and np.array_equal(rowpos, pc.rowpos) and np.array_equal(codes, pc.acodes)


def test_read_gtrack_packed_duplicate_positions_and_errors(tmp_path):
    """Two rows at one position stay two rows when the leading run is one row; the
    population size is the leading run of equal positions (get_population_size), so a
    track whose later run is not a multiple of it has no packed form (ValueError), and
    so has a value outside 3, 0, -3, -10000."""
    from gdscan import GdError, packed
    from gdscan.gtrack import read_gtrack, read_gtrack_packed
    vals = [3, 0, -3, -10000, 3, 3, 0, 0, -3]
    f = _track_file(tmp_path / "dup.gtrack", [("c", [5, 5, 5, 9, 9, 9, 9, 9, 9], vals)], 3)
    rowpos, codes, size = read_gtrack_packed(f)["c"]
    assert size == 3 and rowpos.tolist() == [5, 9, 9]
    pos, val = read_gtrack(f)["c"]
    assert np.array_equal(codes, packed.pack(val, val, pos, pos, 10).acodes)
    bad = _track_file(tmp_path / "ragged.gtrack", [("c", [5, 5, 9, 9, 9], [3, 3, 3, 3, 3])], 2)
    with pytest.raises(ValueError, match="whole rows"):
        read_gtrack_packed(bad)
    freq = _track_file(tmp_path / "freq.gtrack", [("c", [5, 5], [3, 2])], 2)
    with pytest.raises(ValueError, match="genotype codes"):
        read_gtrack_packed(freq)
    with pytest.raises(GdError):
        read_gtrack_packed(tmp_path / "nope.gtrack")
    assert len(read_gtrack_packed(_track_file(tmp_path / "empty.gtrack", [], 1))) == 0


def test_read_pair_checks_rows(tmp_path):
    from gdscan import packed
    a = _track_file(tmp_path / "a.gtrack", [("c1", [1, 1, 4, 4], [3, 0, 0, 3]), ("c2", [2, 2], [3, 3])], 2)
    b = _track_file(tmp_path / "b.gtrack", [("c2", [2, 2, 2], [0, 0, 0]), ("c1", [1, 1, 1, 4, 4, 4], [3] * 6)], 3)
    names, pcs = packed.read_pair(a, b, {"c1": 1000})
    assert names == ["c1", "c2"] and [p.regend for p in pcs] == [1000, 3]
    assert (pcs[0].asize, pcs[0].bsize, pcs[0].nrows) == (2, 3, 2)
    c = _track_file(tmp_path / "c.gtrack", [("c1", [1, 1, 1, 5, 5, 5], [3] * 6)], 3)
    with pytest.raises(ValueError, match="same positions"):
        packed.read_pair(a, c)


def test_write_tabular_matches_tool_loop(tmp_path):
    """FisherExactTestSNPTool.py:162-189: header, then windows with score != 0 at i*wStep."""
    from gdscan.gtrack import write_tabular
    f = tmp_path / "out.tabular"
    s1 = np.array([0.0, 1.5, -0.0, 3.0, 0.123456789012345, np.nan])
    d1 = np.array([9.0, 0.25, 1.0, 0.0, 2.8722813232690143, 1.0])
    write_tabular(f, "chr1", 500, s1, d1, header="#seqid\tstart\tscore\tstddev", append=False)
    write_tabular(f, "chr2", 500, np.array([7.0]), np.array([0.5]))
    want = "#seqid\tstart\tscore\tstddev\n"
    for i, (s, d) in enumerate(zip(s1, d1)):
        if s != 0:
            want += "%s\t%s\t%s\t%s\n" % ("chr1", i * 500, _py2(s), _py2(d))
    want += "chr2\t0\t7.0\t0.5\n"
    assert f.read_text() == want
