"""CPU: the FET oracle against the reference's known answers (testFisher.c), the
golden fixtures produced by the reference's own C, and (dev container only) the
compiled reference itself."""
import ctypes

import numpy as np
import pytest

from conftest import GOLDEN, SCAN_FIXTURES, load_scan_fixture, oracle_fet_scan


def test_known_answers(oracle):
    # testFisher.c:410-414; the reference's overflow guard first returns 0 at C(68,31)
    assert oracle.orc_binomial(5, 3) == 10
    assert oracle.orc_binomial(40, 19) == 131282408400
    assert oracle.orc_binomial(67, 31) == 11923179284862717872
    assert oracle.orc_binomial(68, 31) == 0
    # testFisher.c:467-472
    assert abs(oracle.orc_fet_p(1, 9, 11, 3) - 0.001346076) < 1e-9
    assert abs(oracle.orc_fet_p(0, 10, 12, 2) - 0.000033652) < 1e-9
    assert abs(oracle.orc_fet_p(9, 3, 1, 6) - 0.0166706) < 1e-7
    # testFisher.c:474-500
    assert abs(oracle.orc_fet(2, 7, 8, 2) - 0.0230141) < 1e-7
    assert abs(oracle.orc_fet(2, 3, 6, 4) - 0.6083916) < 1e-7
    assert oracle.orc_fet(2, 2, 3, 3) == 1.0
    assert oracle.orc_fet(1, 3, 2, 3) == 1.0
    # testFisher.c:389-400 (the reference's own harness mis-declares percentile(); values measured)
    v = np.array([43, 54, 56, 61, 62, 66, 68, 69, 69, 70, 71, 72, 77, 78, 79, 85, 87, 88, 89, 93, 95, 96, 98, 99, 99],
                 np.float64)
    assert abs(oracle.orc_percentile(v, 25, 0.90) - 97.2) < 1e-12
    assert oracle.orc_percentile(np.arange(10, dtype=np.float64), 10, 0.5) == 4.5


def test_fetcount_known_answer(oracle):
    # testFisher.c:416-448: table 4|1 / 3|4
    av = np.array([3, 3, 0, -10000, 3, -3, 0, 0, 0, 3] * 2, np.float64)
    bv = np.array([-3, -3, 0, -10000, -3, -3, 3, 3, 3, 0] * 2, np.float64)
    f = (ctypes.c_int * 4)()
    oracle.orc_fet_counts.argtypes = [np.ctypeslib.ndpointer(np.float64, flags="C")] * 2 + \
        [ctypes.c_int] * 3 + [ctypes.c_int * 4]
    oracle.orc_fet_counts(av, bv, 0, 10, 10, f)
    assert list(f) == [4, 1, 3, 4]


def test_all_tables_match_reference_fixture(oracle):
    z = np.load(GOLDEN / "fet_tables.npz")
    t, p, s = z["tables"], z["p"], z["score"]
    po = np.array([oracle.orc_fet(*map(int, r)) for r in t])
    so = np.array([oracle.orc_fet_score(*map(int, r)) for r in t])
    assert np.array_equal(po, p, equal_nan=True)
    assert np.array_equal(so, s, equal_nan=True)
    binom = z["binom"]
    for n in range(81):
        for k in range(n + 1):
            assert oracle.orc_binomial(n, k) == int(binom[n, k])


def test_fet_differs_from_textbook_two_sided():
    """Quirk Q1: the Zar/Feldman-Klinger tail is not scipy's two-sided test."""
    from scipy.stats import fisher_exact
    z = np.load(GOLDEN / "fet_tables.npz")
    t, p = z["tables"][:4356 * 4], z["p"][:4356 * 4]
    diff = 0
    for r, pr in zip(t[::7], p[::7]):
        a, b, c, d = map(int, r)
        sp = fisher_exact([[a, b], [c, d]])[1]
        diff += abs(sp - pr) > 1e-9 * max(sp, pr)
    assert diff > 0


@pytest.mark.parametrize("name", SCAN_FIXTURES)
def test_oracle_scan_matches_reference_fixture(oracle, name):
    f = load_scan_fixture(name)
    s, d = oracle_fet_scan(oracle, f["av"], f["bv"], f["ap"], f["bp"], f["regend"], f["wsize"], f["wstep"],
                           f["perc"], f["seed"], f["serial"])
    assert np.array_equal(s, f["scores"]) and np.array_equal(d, f["stddev"])


def test_oracle_matches_live_reference(oracle, refc):
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(7, 20000, 10, 10)
    n = regend // 500
    s_ref, d_ref = np.zeros(n), np.zeros(n)
    refc.ref_fet_scan_seeded(av, bv, ap, bp, regend, 2500, 500, len(av), len(bv), 0.95, 77, 0, s_ref, d_ref)
    s, d = oracle_fet_scan(oracle, av, bv, ap, bp, regend, seed=77)
    assert np.array_equal(s, s_ref) and np.array_equal(d, d_ref)
    s_thr, d_thr = np.zeros(n), np.zeros(n)
    refc.threadcompute(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 0.95, s_thr, d_thr)
    assert np.array_equal(s, s_thr)


def test_window_sets(oracle):
    """Quirks Q2/Q3: threaded set = [0, end) with nothing when regend/wstep < 103;
    the library's pure window-count function agrees with the oracle."""
    from gdscan import fet
    for regend in (1000, 51_499, 51_500, 52_000, 123_456, 2_510_451, 25_000_000):
        for wsize, wstep in ((2500, 500), (1000, 500), (5000, 500), (2000, 1000), (500, 500)):
            assert fet.window_count(regend, wsize, wstep) == oracle.orc_threaded_window_end(regend, wsize, wstep)
            assert fet.window_count(regend, wsize, wstep, serial=True) == \
                oracle.orc_serial_window_end(regend, wsize, wstep)
    assert oracle.orc_threaded_window_end(51_499, 2500, 500) == 0
