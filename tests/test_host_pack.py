"""CPU: the host-thread packer behind the reference-signature entry points
(gd_pack_chrom_mt: pieces of rows on host threads, AVX2 + BMI2 where the CPU has them)
equals the scalar packer gd_pack_chrom word for word, and refuses what it refuses."""
import ctypes as C
import os

import numpy as np
import pytest


def _pack(fn, av, bv, ap, bp, a, b, nr):
    ac = np.zeros(nr * ((a + 31) // 32), np.uint64)
    bc = np.zeros(nr * ((b + 31) // 32), np.uint64)
    rp = np.zeros(nr, np.int32)
    st = fn(av.ctypes.data_as(C.POINTER(C.c_double)), bv.ctypes.data_as(C.POINTER(C.c_double)),
            ap.ctypes.data_as(C.POINTER(C.c_int)), bp.ctypes.data_as(C.POINTER(C.c_int)), a, b, nr,
            ac.ctypes.data, bc.ctypes.data, rp.ctypes.data)
    return st, ac, bc, rp


@pytest.mark.parametrize("a,b,threads", [(20, 20, "3"), (37, 20, "8"), (1, 3, "2"), (64, 65, "1"), (5, 5, "")])
def test_threaded_packer_matches_scalar(a, b, threads, monkeypatch):
    from gdscan import synth
    from gdscan._lib import lib
    if threads:
        monkeypatch.setenv("GD_HOST_THREADS", threads)
    nr = 7001
    av, bv, ap, bp, _ = synth.chromosome(66, nr, a, b)
    ref = _pack(lib.gd_pack_chrom, av, bv, ap, bp, a, b, nr)
    got = _pack(lib.gd_pack_chrom_mt, av, bv, ap, bp, a, b, nr)
    assert ref[0] == got[0] == 0
    assert all(np.array_equal(x, y) for x, y in zip(ref[1:], got[1:]))


@pytest.mark.parametrize("kind", ["value", "apos", "bpos", "minus_zero"])
def test_threaded_packer_refusals(kind):
    from gdscan import synth
    from gdscan._lib import lib
    nr, a, b = 3000, 20, 13
    av, bv, ap, bp, _ = synth.chromosome(67, nr, a, b)
    av, bv, ap, bp = av.copy(), bv.copy(), ap.copy(), bp.copy()
    if kind == "value":
        bv[13 * 2999 + 12] = 3.0000001
    elif kind == "apos":
        ap[20 * 1500 + 19] += 1
    elif kind == "bpos":
        bp[13 * 10] -= 1
    else:
        av[av == 0.0] = -0.0  # -0.0 == 0.0: the heterozygous code, as the reference's compares see it
    ref = _pack(lib.gd_pack_chrom, av, bv, ap, bp, a, b, nr)
    got = _pack(lib.gd_pack_chrom_mt, av, bv, ap, bp, a, b, nr)
    assert (ref[0] == 0) == (got[0] == 0) == (kind == "minus_zero")
    if kind == "minus_zero":
        assert all(np.array_equal(x, y) for x, y in zip(ref[1:], got[1:]))
