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


def test_fisher_exact_test_snp_tool(oracle, tmp_path):
    from gdscan import lib
    from gdscan.tools import fisher_exact_test_snp
    chroms = _chroms(6, 6)
    fa, fb = _write_tracks(tmp_path, chroms, 6, 6)
    out = tmp_path / "fet.tabular"
    lib.gd_set_seed(20261015)
    names, _, _ = fisher_exact_test_snp(fa, fb, out)
    assert names == ["chr1", "chr2"]
    res = [oracle_fet_scan(oracle, av, bv, ap, bp, regend) for _, (av, bv, ap, bp, regend) in chroms]
    assert out.read_text() == _expected("#seqid\tstart\tscore\tstddev", chroms, 500, res)


def test_cluster_separation_score_tool(oracle, tmp_path):
    from gdscan import lib
    from gdscan.tools import cluster_separation_score
    chroms = _chroms(5, 7)
    fa, fb = _write_tracks(tmp_path, chroms, 5, 7)
    out = tmp_path / "css.tabular"
    lib.gd_set_seed(20261015)
    cluster_separation_score(fa, fb, out, mc_treshold=10, mc_runs=0)
    res = [oracle_css_scan(oracle, av, bv, ap, bp, regend) for _, (av, bv, ap, bp, regend) in chroms]
    got = out.read_text().splitlines()
    want = _expected("#seqid\tstart\tscore\tp", chroms, 500, res).splitlines()
    assert len(got) == len(want) and got[0] == want[0]
    # CSS scores agree to ~1e-13 (different eigen-solvers); compare numerically
    for g, w in zip(got[1:], want[1:]):
        gs, ws = g.split("\t"), w.split("\t")
        assert gs[:2] == ws[:2] and gs[3] == ws[3]
        assert abs(float(gs[2]) - float(ws[2])) <= 1e-9 * abs(float(ws[2])) + 1e-11
