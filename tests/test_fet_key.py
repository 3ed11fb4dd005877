"""The FET window kernel's order key (gd_fet_fast.hip fw_key / fw_key_index).

The bootstrap loop never forms r mod n (random_int_nrand48, cFisher.c:547-554): it
keeps the top order statistics of key(u) = (M*u mod 2^64) >> 32, u = the high state
word (r = u >> 1), M = ceil(2^64 / 2n), and recovers r mod n = ((key + 1) * 2n) >> 33.
These checks pin the two properties the kernel relies on, for every n the fast path
takes (2..256): distinct residues u mod 2n order strictly by key, and the recovery is
exact."""
import numpy as np

MASK64 = (1 << 64) - 1


def key_np(u, n):
    D = 2 * n
    M = np.uint64(MASK64 // D + 1)
    return ((u * M) >> np.uint64(32)).astype(np.uint64)  # uint64 product wraps mod 2^64


def test_key_recovers_residue_and_orders():
    rng = np.random.default_rng(11)
    base = rng.integers(0, 1 << 32, 40000, dtype=np.uint64)
    for n in range(1, 257):
        D = 2 * n
        top = np.uint64((1 << 32) - 1)
        edges = np.array([0, 1, D - 1, D, D + 1], dtype=np.uint64)
        hi = top - np.arange(0, 3 * D, dtype=np.uint64)  # the top of the u range, every residue
        u = np.concatenate([base, edges, hi])
        k = key_np(u, n)
        res = u % np.uint64(D)
        got = ((k + np.uint64(1)) * np.uint64(D)) >> np.uint64(33)
        assert np.array_equal(got, res >> np.uint64(1)), n
        order = np.argsort(k, kind="stable")
        rs = res[order]
        assert np.all(np.diff(rs.astype(np.int64)) >= 0), n  # residues non-decreasing along keys
        # distinct residues: keys strictly separated
        kmax = np.zeros(D, dtype=np.int64) - 1
        kmin = np.full(D, 1 << 40, dtype=np.int64)
        np.maximum.at(kmax, res.astype(np.int64), k.astype(np.int64))
        np.minimum.at(kmin, res.astype(np.int64), k.astype(np.int64))
        seen = kmax >= 0
        assert np.all(kmax[seen][:-1] < kmin[seen][1:]), n


def test_key_matches_remainder_draws():
    """r mod n of real nrand48 draws (the oracle's random_int_nrand48) equals the recovery."""
    A, C = 0x5DEECE66D, 0xB
    x = 0x1234ABCD5678
    for n in (2, 3, 7, 50, 64, 100, 255, 256):
        D = 2 * n
        M = MASK64 // D + 1
        for _ in range(3000):
            x = (A * x + C) & ((1 << 48) - 1)
            u = x >> 16  # the high word of y = x << 16
            r = x >> 17
            key = ((M * u) & MASK64) >> 32
            assert ((key + 1) * D) >> 33 == r % n


def key16_np(u, n):
    """FW_KEY16: the low half of (M16 u mod 2^64) >> 32, M16 = ceil(M / 2^16) = ceil(2^48 / 2n)."""
    D = 2 * n
    M16 = np.uint64(((MASK64 // D + 1) + 0xFFFF) >> 16)
    return ((u * M16) >> np.uint64(32)) & np.uint64(0xFFFF)


def test_key16_recovers_residue_and_orders():
    rng = np.random.default_rng(12)
    base = rng.integers(0, 1 << 32, 40000, dtype=np.uint64)
    for n in range(1, 257):
        D = 2 * n
        top = np.uint64((1 << 32) - 1)
        edges = np.array([0, 1, D - 1, D, D + 1], dtype=np.uint64)
        hi = top - np.arange(0, 3 * D, dtype=np.uint64)
        u = np.concatenate([base, edges, hi])
        k = key16_np(u, n)
        res = u % np.uint64(D)
        idx = ((k + np.uint64(1)) * np.uint64(D)) >> np.uint64(17)
        assert np.array_equal(idx, res >> np.uint64(1)), n
        kmax = np.zeros(D, dtype=np.int64) - 1
        kmin = np.full(D, 1 << 40, dtype=np.int64)
        np.maximum.at(kmax, res.astype(np.int64), k.astype(np.int64))
        np.minimum.at(kmin, res.astype(np.int64), k.astype(np.int64))
        seen = kmax >= 0
        assert np.all(kmax[seen][:-1] < kmin[seen][1:]), n
        # pick_rix's packed form: ((key16 + 1) 256 n - base 2^24) mod 2^32, byte 3 = index - base
        for b in (0, 1, min(7, n - 1), n - 1):
            sel = (idx >= np.uint64(b))
            t = ((k[sel] * np.uint64(256 * n) + np.uint64((256 * n - (b << 24)) & 0xFFFFFFFF)) & np.uint64(0xFFFFFFFF))
            assert np.array_equal(t >> np.uint64(24), (idx[sel] - np.uint64(b)) & np.uint64(0xFF)), (n, b)
