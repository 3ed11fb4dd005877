"""CPU: the CSS oracle against the known answers of the reference's testcss.c and an
independent numpy/LAPACK restatement of classical MDS.  The reference CSS C needs
GSL, absent from this image, so no reference-built CSS fixtures exist."""
import ctypes

import numpy as np
import pytest

F64 = np.ctypeslib.ndpointer(np.float64, flags="C")
I32 = np.ctypeslib.ndpointer(np.int32, flags="C")


@pytest.fixture(scope="module")
def css(oracle):
    C = ctypes
    oracle.orc_css_compare_all.argtypes = [F64, F64, C.c_int, C.c_int, C.c_int, F64]
    oracle.orc_css_fill_averages.argtypes = [F64, C.c_int]
    oracle.orc_css_cmds.argtypes = [F64, C.c_int, F64, F64]
    oracle.orc_css_dist.argtypes = [F64, C.c_int, F64]
    oracle.orc_css_score.argtypes = [F64, C.c_int, I32, I32, C.c_int, C.c_int]
    oracle.orc_css_score.restype = C.c_double
    oracle.orc_css_window.argtypes = [F64, F64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                      C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int)]
    return oracle


def test_compare_all_kat(css):
    # testcss.c:369-420
    av = np.array([-3, 3, 0, 3], np.float64)
    bv = np.array([3, -3, -10000, 0], np.float64)
    D = np.full(16, -1.0)
    css.orc_css_compare_all(av, bv, 2, 2, 2, D)
    assert D.reshape(4, 4).tolist() == [[0, 1, 1, 0], [1, 0, 0, 1], [1, 0, 0, 1], [0, 1, 1, 0]]


def test_compare_all_is_PtN_plus_NtP(css):
    rng = np.random.default_rng(5)
    a, b, npos = 9, 14, 61
    av = rng.choice([3.0, 0.0, -3.0, -10000.0], (npos, a)).ravel()
    bv = rng.choice([3.0, 0.0, -3.0, -10000.0], (npos, b)).ravel()
    D = np.zeros((a + b) ** 2)
    css.orc_css_compare_all(av, bv, a, b, npos, D)
    V = np.concatenate([av.reshape(npos, a), bv.reshape(npos, b)], 1)
    P, N = (V == 3).astype(int), (V == -3).astype(int)
    ref = P.T @ N + N.T @ P
    np.fill_diagonal(ref, 0)
    assert np.array_equal(D.reshape(a + b, a + b), ref)


def test_fill_averages_kat(css):
    # testcss.c:422-473
    m = 5
    D = np.array([[0 if i == j else i + j for j in range(m)] for i in range(m)], np.float64).ravel()
    assert css.orc_css_fill_averages(D, m) == 1
    assert D[0] == 3.2 and D[6] == 3.2
    D = D.reshape(m, m)
    D[:, 0] = D[:, m - 1] = D[0, :] = 0
    np.fill_diagonal(D, 0)
    D = np.ascontiguousarray(D).ravel()
    assert css.orc_css_fill_averages(D, m) == 0


def test_calc_dist_kat(css):
    # testcss.c:475-510
    X = np.array([[0, 1], [1, 2]], np.float64).ravel()
    S = np.zeros(4)
    css.orc_css_dist(X, 2, S)
    assert np.allclose(S, [0, np.sqrt(2), np.sqrt(2), 0])


def test_cmds_kat(css):
    # testcss.c:569-620 (expected X printed to 2 decimals; columns up to sign)
    D = np.array([0, 4.05, 8.25, 5.57, 4.05, 0, 2.54, 2.69, 8.25, 2.54, 0, 2.11, 5.57, 2.69, 2.11, 0])
    X, e = np.zeros(8), np.zeros(2)
    css.orc_css_cmds(D, 4, X, e)
    X = X.reshape(4, 2)
    exp = np.array([[4.62, 0.07], [0.09, -1.11], [-3.63, -0.34], [-1.08, 1.38]])
    for c in range(2):
        s = np.sign(X[0, c]) * np.sign(exp[0, c])
        assert np.allclose(s * X[:, c], exp[:, c], atol=0.006)


def test_css_kat(css):
    # testcss.c:701-740
    m = 100
    X = np.array([[i, i + 1] for i in range(m)], np.float64).ravel()
    S = np.zeros(m * m)
    css.orc_css_dist(X, m, S)
    sc = css.orc_css_score(S, m, np.arange(50, dtype=np.int32), np.arange(50, 100, dtype=np.int32), 50, 50)
    assert abs(sc - 70.5975410337) < 1e-9


def numpy_cmds(D):
    m = len(D)
    Z = np.eye(m) - 1.0 / m
    B = -0.5 * Z @ (D * D) @ Z
    w, V = np.linalg.eigh(B)
    o = np.argsort(-w, kind="stable")[:2]
    return V[:, o] * np.sqrt(w[o])


@pytest.mark.parametrize("a,b", [(10, 10), (20, 20), (7, 13), (40, 40)])
def test_window_matches_lapack_restatement(css, a, b):
    """The Jacobi solver vs LAPACK: CSS depends only on distances in X (invariant to
    eigenvector sign), so the scores agree to ~1e-14 relative."""
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(11, 4000, a, b)
    for start in range(0, 3000, 97):
        npos = 50
        va = av[start * a:(start + npos) * a]
        vb = bv[start * b:(start + npos) * b]
        sc, p, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        ok = css.orc_css_window(np.ascontiguousarray(va), np.ascontiguousarray(vb), a, b, npos, 10, 0, 1,
                                ctypes.byref(sc), ctypes.byref(p), ctypes.byref(n))
        D = np.zeros((a + b) ** 2)
        css.orc_css_compare_all(np.ascontiguousarray(va), np.ascontiguousarray(vb), a, b, npos, D)
        ok2 = css.orc_css_fill_averages(D, a + b)
        assert ok == ok2
        if not ok:
            continue
        X = numpy_cmds(D.reshape(a + b, a + b))
        S = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)).ravel()
        ref = css.orc_css_score(np.ascontiguousarray(S), a + b, np.arange(a, dtype=np.int32),
                                np.arange(a, a + b, dtype=np.int32), a, b)
        assert p.value == 1.0 and n.value == 0
        assert abs(sc.value - ref) <= 1e-11 * abs(ref) + 1e-12


def test_significance_early_exit(css):
    """runs/treshold semantics: p = (hits+1)/(nscores+1), stop once hits == treshold."""
    from gdscan import synth
    av, bv, ap, bp, regend = synth.chromosome(2, 3000, 10, 10)
    npos = 50
    va, vb = np.ascontiguousarray(av[:npos * 10]), np.ascontiguousarray(bv[:npos * 10])
    sc, p, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    css.orc_css_window(va, vb, 10, 10, npos, 10, 1000, 12345, ctypes.byref(sc), ctypes.byref(p), ctypes.byref(n))
    hits = round(p.value * (n.value + 1)) - 1
    assert 1 <= n.value <= 1000
    assert hits == 10 or n.value == 1000
    assert abs(p.value - (hits + 1) / (n.value + 1)) < 1e-15
