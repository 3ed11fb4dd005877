"""Fisher-exact-test window scan, reference-compatible entry points.

``fisher_exact_tester`` has the positional signature of the reference's Cython
function (statistics/fisher/fisher_cython_parallel.pyx:14) and its contract:
float64 avals/bvals, int32 apos/bpos (wrong dtype -> ValueError, as Cython's
typed buffers raise), outputs written in place at computed windows only.

The bootstrap seed of the reference-signature functions is per calling thread
(gd_set_seed in one thread does not reach another; include/gdscan.h): a worker thread
sets its own, or calls scan(..., seed=...).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import GD_FET_EXACT, GD_FET_REFERENCE, GD_WINDOWS_SERIAL, GD_WINDOWS_THREADED, check, lib

_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int)


def _arr(a, dtype, name):
    if not isinstance(a, np.ndarray) or a.ndim != 1:
        raise ValueError(f"{name}: expected a 1-d numpy array")
    if a.dtype != dtype:
        raise ValueError(f"Buffer dtype mismatch for {name}: expected {np.dtype(dtype).name}, got {a.dtype.name}")
    return a


def _ptrs(avals, bvals, apos, bpos, scores, other, other_name):
    avals = _arr(avals, np.float64, "avals")
    bvals = _arr(bvals, np.float64, "bvals")
    apos = _arr(apos, np.int32, "apos")
    bpos = _arr(bpos, np.int32, "bpos")
    scores = _arr(scores, np.float64, "scores")
    other = _arr(other, np.float64, other_name)
    for a, n in ((scores, "scores"), (other, other_name)):
        if not a.flags.c_contiguous or not a.flags.writeable:
            raise ValueError(f"{n} must be a writeable contiguous array")
    ins = [np.ascontiguousarray(x) for x in (avals, bvals, apos, bpos)]
    return ins, scores, other


def _run(fn, avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, perc, scores, stddev):
    (av, bv, ap, bp), scores, stddev = _ptrs(avals, bvals, apos, bpos, scores, stddev, "stddev")
    if alen > av.shape[0] or blen > bv.shape[0] or alen > ap.shape[0] or blen > bp.shape[0]:
        raise ValueError("alen/blen exceed the array lengths")
    nwin = int(regend) // int(wstep) if wstep > 0 else 0
    if scores.shape[0] < nwin or stddev.shape[0] < nwin:
        raise ValueError(f"output arrays must hold regend//wstep = {nwin} windows")
    check(fn(av.ctypes.data_as(_DP), bv.ctypes.data_as(_DP), ap.ctypes.data_as(_IP), bp.ctypes.data_as(_IP),
             int(regstart), int(regend), int(wsize), int(wstep), int(alen), int(blen), float(perc),
             scores.ctypes.data_as(_DP), stddev.ctypes.data_as(_DP)))


def fisher_exact_tester(avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, perc, scores,
                        stddev):
    """Drop-in for fisher_cython_parallel.fisher_exact_tester (threaded window set)."""
    _run(lib.gd_fet_threadcompute, avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, perc,
         scores, stddev)


def fisher_exact_tester_serial(avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, perc, scores,
                               stddev):
    """Drop-in for fisher_cython.fisher_exact_tester (serial compute() window set)."""
    _run(lib.gd_fet_compute, avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, perc, scores,
         stddev)


def _mode(exact):
    if exact is None:
        return lib.gd_get_fet_mode()
    return GD_FET_EXACT if exact else GD_FET_REFERENCE


def set_mode(exact):
    """Table probabilities of every call without an explicit mode, the reference-signature
    entry points included: exact=True evaluates them from ln k! (correct for >= 68
    individuals), False reproduces the reference's u64 binomials.  Returns the previous
    setting (True = exact)."""
    old = lib.gd_set_fet_mode(_mode(bool(exact)))
    check(min(old, 0))
    return old == GD_FET_EXACT


def scan(avals, bvals, apos, bpos, regend, wsize=2500, wstep=500, perc=0.95, seed=None, serial=False, exact=None):
    """Convenience: allocate zeroed outputs (regend//wstep) and run one chromosome.  exact:
    see set_mode (None follows it)."""
    nwin = int(regend) // int(wstep)
    scores = np.zeros(nwin)
    stddev = np.zeros(nwin)
    (av, bv, ap, bp), scores, stddev = _ptrs(avals, bvals, apos, bpos, scores, stddev, "stddev")
    s = lib.gd_get_seed() if seed is None else int(seed)
    check(lib.gd_fet_scan_host_ex(av.ctypes.data_as(_DP), bv.ctypes.data_as(_DP), ap.ctypes.data_as(_IP),
                                  bp.ctypes.data_as(_IP), int(regend), int(wsize), int(wstep), av.shape[0],
                                  bv.shape[0], float(perc), _mode(exact), s,
                                  GD_WINDOWS_SERIAL if serial else GD_WINDOWS_THREADED,
                                  scores.ctypes.data_as(_DP), stddev.ctypes.data_as(_DP)))
    return scores, stddev


def window_count(regend, wsize, wstep, serial=False):
    return lib.gd_window_count(int(regend), int(wsize), int(wstep), GD_WINDOWS_SERIAL if serial else
                               GD_WINDOWS_THREADED)
