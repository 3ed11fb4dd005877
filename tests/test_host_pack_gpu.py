"""GPU: the reference-signature host entry points pack whole-row genotype tracks on host
threads (gd_pack_chrom_mt) and scan the packed form (gd_api.hip host_packed).  The packed
route must give the bit-identical outputs of the reference-layout route
(GD_HOST_NOPACK=1) and of the oracle, keep the caller's values at uncomputed windows, and
fall back to the reference layout whenever a value, a position or a row is off the packed
form (irregular values, A/B rows at different positions, partial rows, drosophila)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import close, oracle_css_scan

pytestmark = pytest.mark.gpu

C = ctypes
DPP = C.POINTER(C.c_double)
IPP = C.POINTER(C.c_int)


def _d(x):
    return x.ctypes.data_as(DPP)


def _i(x):
    return x.ctypes.data_as(IPP)


class nopack:
    """GD_HOST_NOPACK=1 for the calls inside (read by the library at every call)"""

    def __enter__(self):
        os.environ["GD_HOST_NOPACK"] = "1"

    def __exit__(self, *a):
        os.environ.pop("GD_HOST_NOPACK", None)


def _fet(av, bv, ap, bp, regend, seed=777, serial=False, fill=5.0):
    from gdscan import lib
    n = regend // 500
    s, d = np.full(n, fill), np.full(n, fill)
    fn = lib.gd_fet_scan_host
    st = fn(_d(av), _d(bv), _i(ap), _i(bp), regend, 2500, 500, len(av), len(bv), 0.95, seed, int(serial), _d(s), _d(d))
    assert st == 0, lib.gd_last_error()
    return s, d


def _css(av, bv, ap, bp, regend, runs=100, seed=777, drosophila=0, fill=5.0):
    from gdscan import lib
    n = regend // 500
    s, p = np.full(n, fill), np.full(n, fill)
    st = lib.gd_css_scan_host_ex(_d(av), _d(bv), _i(ap), _i(bp), regend, 2500, 500, len(av), len(bv), 10, runs,
                                 drosophila, 0, seed, 0, _d(s), _d(p))
    assert st == 0, lib.gd_last_error()
    return s, p


@pytest.mark.parametrize("a,b,nsnp", [(20, 20, 30000), (10, 13, 9000), (40, 40, 6000), (33, 64, 5000)])
def test_fet_packed_route_equals_reference_layout(oracle, a, b, nsnp):
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(61, nsnp, a, b)
    s1, d1 = _fet(av, bv, ap, bp, regend)
    with nopack():
        s2, d2 = _fet(av, bv, ap, bp, regend)
    assert np.array_equal(s1, s2, equal_nan=True) and np.array_equal(d1, d2, equal_nan=True)
    assert (s1 == 5.0).sum() > 0  # uncomputed windows keep the caller's values
    n = regend // 500
    s_ref, d_ref = np.full(n, 5.0), np.full(n, 5.0)
    oracle.orc_fet_scan(av, bv, ap, bp, regend, 2500, 500, len(av), len(bv), 0.95, 777, 0, s_ref, d_ref)
    assert close(s1, s_ref) and close(d1, d_ref)


def test_fet_packed_route_serial_window_set():
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(62, 8000, 20, 20)
    s1, d1 = _fet(av, bv, ap, bp, regend, serial=True)
    with nopack():
        s2, d2 = _fet(av, bv, ap, bp, regend, serial=True)
    assert np.array_equal(s1, s2, equal_nan=True) and np.array_equal(d1, d2, equal_nan=True)


@pytest.mark.parametrize("kind", ["value", "nan", "apos", "bpos", "partial"])
def test_fet_irregular_tracks_fall_back(oracle, kind):
    """anything off the packed form scans in the reference layout, with the oracle's outputs"""
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(63, 8000, 12, 9)
    av, bv, ap, bp = av.copy(), bv.copy(), ap.copy(), bp.copy()
    if kind == "value":
        av[12 * 3000 + 5] = 1.0
    elif kind == "nan":
        bv[9 * 4000 + 2] = np.nan
    elif kind == "apos":
        ap[12 * 2000 + 7] += 1  # an A individual off its row's position (positions stay sorted)
        ap[12 * 2000 + 8:12 * 2000 + 12] += 1
    elif kind == "bpos":
        bp[9 * 5000:9 * 5001] += 1  # B row 5000 at another position than A's row 5000
    else:
        av, ap = av[:-3], ap[:-3]  # a partial last A row
    s1, d1 = _fet(av, bv, ap, bp, regend)
    with nopack():
        s2, d2 = _fet(av, bv, ap, bp, regend)
    assert np.array_equal(s1, s2, equal_nan=True) and np.array_equal(d1, d2, equal_nan=True)
    n = regend // 500
    s_ref, d_ref = np.full(n, 5.0), np.full(n, 5.0)
    oracle.orc_fet_scan(av, bv, ap, bp, regend, 2500, 500, len(av), len(bv), 0.95, 777, 0, s_ref, d_ref)
    assert close(s1, s_ref) and close(d1, d_ref)


@pytest.mark.parametrize("a,b", [(20, 20), (40, 40), (7, 12)])
def test_css_packed_route_equals_reference_layout(a, b):
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(64, 6000, a, b)
    s1, p1 = _css(av, bv, ap, bp, regend)
    with nopack():
        s2, p2 = _css(av, bv, ap, bp, regend)
    assert np.array_equal(s1, s2, equal_nan=True) and np.array_equal(p1, p2, equal_nan=True)
    assert (s1 == 5.0).sum() > 0


def test_css_irregular_falls_back(oracle):
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(65, 6000, 15, 15)
    av = av.copy()
    av[15 * 1000 + 3] = 2.0
    s1, p1 = _css(av, bv, ap, bp, regend, runs=0)
    with nopack():
        s2, p2 = _css(av, bv, ap, bp, regend, runs=0)
    assert np.array_equal(s1, s2, equal_nan=True) and np.array_equal(p1, p2, equal_nan=True)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, treshold=10, runs=0, seed=777)
    comp = s_ref != 0
    assert close(s1[comp], s_ref[comp])


def test_fet_batch_packed_route():
    """gd_fet_scan_host_batch (the Galaxy tool's whole-genome call): several chromosomes, one
    packed scan, equal to the reference-layout batch"""
    from gdscan import synth
    from gdscan._lib import Chrom, lib
    parts = [synth.chromosome(70 + c, 5000 + 1000 * c, 20, 20) for c in range(3)]
    av = np.concatenate([p[0] for p in parts])
    bv = np.concatenate([p[1] for p in parts])
    ap = np.concatenate([p[2] for p in parts])
    bp = np.concatenate([p[3] for p in parts])
    ch = (Chrom * 3)()
    ao = bo = wo = 0
    for c, p in enumerate(parts):
        ch[c].a_off, ch[c].b_off, ch[c].alen, ch[c].blen = ao, bo, len(p[0]), len(p[1])
        ch[c].regend, ch[c].w_out, ch[c].seed = p[4], wo, 900 + c
        ao += len(p[0])
        bo += len(p[1])
        wo += p[4] // 500
    out = []
    for packed in (True, False):
        s, d = np.full(wo, 3.0), np.full(wo, 3.0)
        if not packed:
            os.environ["GD_HOST_NOPACK"] = "1"
        try:
            st = lib.gd_fet_scan_host_batch(ch, 3, _d(av), _d(bv), _i(ap), _i(bp), 2500, 500, 0.95, 0, _d(s), _d(d))
        finally:
            os.environ.pop("GD_HOST_NOPACK", None)
        assert st == 0, lib.gd_last_error()
        out.append((s, d))
    assert np.array_equal(out[0][0], out[1][0], equal_nan=True) and np.array_equal(out[0][1], out[1][1], equal_nan=True)


def _fet_status(av, bv, ap, bp, regend, seed=777, fill=5.0):
    from gdscan import lib
    n = regend // 500
    s, d = np.full(n, fill), np.full(n, fill)
    st = lib.gd_fet_scan_host(_d(av), _d(bv), _i(ap), _i(bp), regend, 2500, 500, len(av), len(bv), 0.95, seed, 0,
                              _d(s), _d(d))
    return st, s, d


def _css_status(av, bv, ap, bp, regend, runs=50, seed=777, fill=5.0):
    from gdscan import lib
    n = regend // 500
    s, p = np.full(n, fill), np.full(n, fill)
    st = lib.gd_css_scan_host_ex(_d(av), _d(bv), _i(ap), _i(bp), regend, 2500, 500, len(av), len(bv), 10, runs, 0, 0,
                                 seed, 0, _d(s), _d(p))
    return st, s, p


@pytest.mark.parametrize("kind", ["repeat", "decrease"])
@pytest.mark.parametrize("scan", ["fet", "css"])
def test_packed_route_row_positions(oracle, kind, scan):
    """Row positions the packer accepts (A and B rows share them) but slide_right sees as
    unusual: two consecutive rows at one position (k_bounds_rows' repeated run), and a
    decreasing position (the packed route's UNSORTED detection, not a fallback).  The packed
    route must give the reference-layout route's outputs and status."""
    from gdscan import synth
    a, b = 12, 9
    av, bv, ap, bp, regend = synth.chromosome(66, 8000, a, b)
    ap, bp = ap.copy(), bp.copy()
    r = 3000
    if kind == "repeat":
        ap[a * (r + 1):a * (r + 2)] = ap[a * r]
        bp[b * (r + 1):b * (r + 2)] = bp[b * r]
    else:
        ap[a * (r + 1):a * (r + 2)] = ap[a * r] - 1
        bp[b * (r + 1):b * (r + 2)] = bp[b * r] - 1
    run = _fet_status if scan == "fet" else _css_status
    st1, o1, q1 = run(av, bv, ap, bp, regend)
    with nopack():
        st2, o2, q2 = run(av, bv, ap, bp, regend)
    assert st1 == st2
    assert np.array_equal(o1, o2, equal_nan=True) and np.array_equal(q1, q2, equal_nan=True)
    if kind == "repeat":
        assert st1 == 0 and (o1 != 5.0).sum() > 0
        if scan == "fet":
            n = regend // 500
            s_ref, d_ref = np.full(n, 5.0), np.full(n, 5.0)
            oracle.orc_fet_scan(av, bv, ap, bp, regend, 2500, 500, len(av), len(bv), 0.95, 777, 0, s_ref, d_ref)
            assert close(o1, s_ref) and close(q1, d_ref)
    else:
        assert st1 != 0  # unsorted positions are reported on both routes
