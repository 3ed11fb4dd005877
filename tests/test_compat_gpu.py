"""GPU: INTEGRATION.md Route 2 end to end -- the compat libraries called through the
reference's own C signatures (threadfisher.h:33-34, cFisher.h:11-12, threadcss.h:36-37,
css.h:10-11), exactly as the unmodified .pyx files would call them, against the oracle."""
import ctypes

import numpy as np
import pytest

from conftest import assert_p_mismatches_are_ties, PKG, close, oracle_css_scan, oracle_fet_scan

pytestmark = pytest.mark.gpu

DP = np.ctypeslib.ndpointer(np.float64, flags="C")
IP = np.ctypeslib.ndpointer(np.int32, flags="C")


def _load(name, fet):
    import gdscan  # noqa: F401  (libgdscan.so first, RTLD_GLOBAL: one seed for both)
    lib = ctypes.CDLL(str(PKG / "lib" / name))
    C = ctypes
    if fet:
        sig = [DP, DP, IP, IP] + [C.c_int] * 6 + [C.c_double, DP, DP]
    else:
        sig = [DP, DP, IP, IP] + [C.c_int] * 10 + [DP, DP]
    for fn in (lib.threadcompute, lib.compute):
        fn.argtypes = sig
        fn.restype = None  # void, as in the reference
    return lib


@pytest.mark.parametrize("serial", [False, True])
def test_fisher_compat_symbols(oracle, serial):
    from gdscan import lib as gd, synth
    lib = _load("libgdscan_fisher.so", True)
    av, bv, ap, bp, regend = synth.chromosome(40, 8000, 12, 9)
    n = regend // 500
    s, d = np.full(n, 5.0), np.full(n, 5.0)
    gd.gd_set_seed(31337)
    fn = lib.compute if serial else lib.threadcompute
    fn(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 0.95, s, d)
    gd.gd_set_seed(20261015)
    s_ref, d_ref = np.full(n, 5.0), np.full(n, 5.0)
    oracle.orc_fet_scan(av, bv, ap, bp, regend, 2500, 500, len(av), len(bv), 0.95, 31337, int(serial), s_ref, d_ref)
    assert (s_ref != 5.0).sum() > 100
    assert close(s, s_ref) and close(d, d_ref)


@pytest.mark.parametrize("serial", [False, True])
def test_css_compat_symbols(oracle, serial):
    from gdscan import lib as gd, synth
    lib = _load("libgdscan_css.so", False)
    av, bv, ap, bp, regend = synth.chromosome(41, 8000, 10, 11)
    n = regend // 500
    s, p = np.zeros(n), np.full(n, -1.0)
    gd.gd_set_seed(4242)
    fn = lib.compute if serial else lib.threadcompute
    fn(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 10, 100, 0, 0, s, p)
    gd.gd_set_seed(20261015)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, treshold=10, runs=100, seed=4242, serial=serial)
    comp = s_ref != 0
    assert comp.sum() > 100
    assert np.array_equal(s != 0, comp)
    assert np.all(np.abs(s - s_ref) <= 1e-9 * np.abs(s_ref) + 1e-12)
    assert np.all(p[~comp] == -1.0)  # untouched at uncomputed windows
    # every p that differs from the oracle scan's is a near-tie on the device's coordinates
    assert_p_mismatches_are_ties(oracle, av, bv, ap, bp, regend, 10, 11, np.where(comp, p, 0.0),
                                 np.where(comp, p_ref, 0.0), 10, 100, 4242, serial=serial)
