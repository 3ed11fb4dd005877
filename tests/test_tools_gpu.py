"""GPU: the end-to-end tools (two population GTrack files -> HyperBrowser tabular
result), every chromosome in one device batch, against per-chromosome oracle scans
written with the tools' own loop."""
import numpy as np
import pytest

from conftest import oracle_css_scan, oracle_fet_scan
from test_gtrack import _py2

pytestmark = pytest.mark.gpu


def _write_tracks(tmp_path, chroms, a, b):
    from gdscan.gtrack import gtrack_header
    fa, fb = tmp_path / "popA.gtrack", tmp_path / "popB.gtrack"
    la, lb = [gtrack_header("g")], [gtrack_header("g")]
    for name, (av, bv, ap, bp, regend) in chroms:
        for k in range(len(ap)):
            la.append("%s\t%d\t%d\ta%d\n" % (name, ap[k], av[k], k % a))
        for k in range(len(bp)):
            lb.append("%s\t%d\t%d\tb%d\n" % (name, bp[k], bv[k], k % b))
    fa.write_text("".join(la))
    fb.write_text("".join(lb))
    return fa, fb


def _expected(header, chroms, wstep, results):
    out = header + "\n"
    for (name, _), (s, o) in zip(chroms, results):
        for i in range(len(s)):
            if s[i] != 0:
                out += "%s\t%s\t%s\t%s\n" % (name, i * wstep, _py2(s[i]), _py2(o[i]))
    return out


def _chroms(a, b):
    from gdscan import synth
    data = [("chr1", synth.chromosome(60, 12_000, a, b)), ("chr2", synth.chromosome(61, 7_000, a, b))]
    return [(n, (av, bv, ap, bp, int(ap[-1]) + 1)) for n, (av, bv, ap, bp, _) in data]


@pytest.mark.parametrize("packed", [True, False])
def test_fisher_exact_test_snp_tool(oracle, tmp_path, packed):
    """packed=True reads the files straight into 2-bit codes (gd_ptrack_read) and scans
    them packed; the output file is the reference-layout path's byte for byte."""
    from gdscan import lib
    from gdscan.tools import fisher_exact_test_snp
    chroms = _chroms(6, 6)
    fa, fb = _write_tracks(tmp_path, chroms, 6, 6)
    out = tmp_path / "fet.tabular"
    lib.gd_set_seed(20261015)
    names, _, _ = fisher_exact_test_snp(fa, fb, out, packed=packed)
    assert names == ["chr1", "chr2"]
    res = [oracle_fet_scan(oracle, av, bv, ap, bp, regend) for _, (av, bv, ap, bp, regend) in chroms]
    assert out.read_text() == _expected("#seqid\tstart\tscore\tstddev", chroms, 500, res)


@pytest.mark.parametrize("packed", [True, False])
def test_cluster_separation_score_tool(oracle, tmp_path, packed):
    from gdscan import lib
    from gdscan.tools import cluster_separation_score
    chroms = _chroms(5, 7)
    fa, fb = _write_tracks(tmp_path, chroms, 5, 7)
    out = tmp_path / "css.tabular"
    lib.gd_set_seed(20261015)
    cluster_separation_score(fa, fb, out, mc_treshold=10, mc_runs=0, packed=packed)
    res = [oracle_css_scan(oracle, av, bv, ap, bp, regend) for _, (av, bv, ap, bp, regend) in chroms]
    got = out.read_text().splitlines()
    want = _expected("#seqid\tstart\tscore\tp", chroms, 500, res).splitlines()
    assert len(got) == len(want) and got[0] == want[0]
    # CSS scores agree to ~1e-13 (different eigen-solvers); compare numerically
    for g, w in zip(got[1:], want[1:]):
        gs, ws = g.split("\t"), w.split("\t")
        assert gs[:2] == ws[:2] and gs[3] == ws[3]
        assert abs(float(gs[2]) - float(ws[2])) <= 1e-9 * abs(float(ws[2])) + 1e-11


@pytest.mark.parametrize("runs", [0, 40])
def test_tools_packed_and_reference_layout_write_the_same_file(tmp_path, runs):
    """The packed reader path and the reference-layout path of both tools, same seed:
    identical files (FET bootstrap and CSS permutation streams included)."""
    from gdscan import lib
    from gdscan.tools import cluster_separation_score, fisher_exact_test_snp
    chroms = _chroms(7, 5)
    fa, fb = _write_tracks(tmp_path, chroms, 7, 5)
    for tool, kw in ((fisher_exact_test_snp, {}), (cluster_separation_score, {"mc_runs": runs, "mds": "smacof+cmds"})):
        outs = []
        for packed in (True, False):
            out = tmp_path / f"{tool.__name__}_{packed}.tabular"
            lib.gd_set_seed(77)
            tool(fa, fb, out, **kw, packed=packed)
            outs.append(out.read_text())
        assert outs[0] == outs[1] and outs[0].count("\n") > 20


def test_tools_fall_back_to_reference_layout(tmp_path):
    """A track with no packed form (a frequency value) runs the reference layout under
    packed="auto" and raises under packed=True."""
    from gdscan.tools import fisher_exact_test_snp
    chroms = _chroms(4, 4)
    fa, fb = _write_tracks(tmp_path, chroms, 4, 4)
    text = fb.read_text().splitlines(keepends=True)
    i = next(k for k, l in enumerate(text) if not l.startswith("#"))
    f = text[i].split("\t")
    text[i] = "\t".join([f[0], f[1], "0.5", f[3]])
    fb.write_text("".join(text))
    names, s, _ = fisher_exact_test_snp(fa, fb, tmp_path / "auto.tabular")
    assert names == ["chr1", "chr2"] and np.count_nonzero(s) > 0
    with pytest.raises(ValueError):
        fisher_exact_test_snp(fa, fb, tmp_path / "strict.tabular", packed=True)
