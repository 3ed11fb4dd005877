"""CPU: the kernels' scalar building blocks (csrc/gd_common.h, compiled for the host)
against libc and the reference fixtures."""
import ctypes
import ctypes.util

import numpy as np

from conftest import GOLDEN


def test_lcg_matches_libc_nrand48(oracle, shim):
    for seed, w in ((1, 0), (20261015, 12345), (2**63 + 5, 10**7)):
        x0 = shim.shim_window_state(seed, 0, w)
        assert x0 == oracle.orc_window_state(seed, 0, w)
        ref = np.zeros(5000, np.int64)
        oracle.orc_nrand48_stream(x0, 5000, ref)
        ours = np.zeros(5000, np.uint32)
        shim.shim_stream(x0, 5000, ours)
        assert np.array_equal(ref, ours.astype(np.int64))
        # jump-ahead == stepping
        for k in (1, 63, 64, 1000, 4999):
            y = np.zeros(1, np.uint32)
            shim.shim_stream(shim.shim_jump(x0, k - 1), 1, y)
            assert y[0] == ours[k - 1]


def test_magic_modulo_exact(shim):
    rng = np.random.default_rng(1)
    for n in list(range(1, 300)) + [511, 512, 513, 1000, 2501, 65535, 1 << 20, 2**31 - 1]:
        rs = np.concatenate([rng.integers(0, 2**31, 4000, dtype=np.uint64).astype(np.uint32),
                             np.arange(0, 2 * n + 2, dtype=np.uint32)[:4000],
                             np.array([2**31 - 1, 2**31 - 2, n * (2**31 // max(n, 1)) - 1], np.uint32)])
        out = np.zeros(len(rs), np.uint32)
        shim.shim_mod(n, np.ascontiguousarray(rs), len(rs), out)
        assert np.array_equal(out, rs % np.uint32(n)), n
        assert shim.shim_limit(n) == 0x7FFFFFFF - (0x80000000 % n)


def test_fet_and_binomial_bit_exact(shim):
    z = np.load(GOLDEN / "fet_tables.npz")
    for r, p in zip(z["tables"], z["p"]):
        q = shim.shim_fet(*map(int, r))
        assert q == p or (np.isnan(q) and np.isnan(p))
    binom = z["binom"]
    for n in range(81):
        for k in range(n + 1):
            assert shim.shim_binomial(n, k) == int(binom[n, k])


def test_log10_reproduces_glibc(shim):
    """-log10 on the device: glibc's fdlibm formula over a correctly rounded log.
    Bit-identical to the reference's glibc log10 except where glibc's own log is
    not correctly rounded (<= 1 ulp, ~0.1% of arguments)."""
    z = np.load(GOLDEN / "fet_tables.npz")
    s = z["score"]
    ours = np.array([shim.shim_score(*map(int, r)) for r in z["tables"]])
    fin = np.isfinite(s)
    assert np.array_equal(np.isnan(ours), np.isnan(s))
    ulp = np.abs(ours[fin] - s[fin]) / np.spacing(np.maximum(np.abs(s[fin]), 1e-300))
    assert ulp.max() <= 1.0
    assert np.mean(ours[fin] == s[fin]) > 0.995
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.random(20000) ** rng.choice([1, 3, 10, 30], 20000), [1.0, 0.5, 2.0, 1e-300, 5e-324]])
    libm = ctypes.CDLL(ctypes.util.find_library("m"))  # the reference links glibc's log10, not numpy's
    libm.log10.argtypes, libm.log10.restype = [ctypes.c_double], ctypes.c_double
    ref = np.array([libm.log10(v) for v in x])
    mine = np.array([shim.shim_log10(v) for v in x])
    assert np.all(np.abs(mine - ref) <= np.spacing(np.abs(ref)))
    assert np.mean(mine == ref) > 0.998
    assert shim.shim_log10(0.0) == -np.inf and np.isnan(shim.shim_log10(-1.0))


def test_pair_index_is_dense(shim):
    for size in (1, 7, 20, 40):
        idx = [shim.shim_pair_index(a, b, size) for a in range(size + 1) for b in range(size + 1 - a)]
        assert idx == list(range((size + 1) * (size + 2) // 2))
