"""Cluster-separation-score window scan, reference-compatible entry points.

``cluster_separation_scorer`` has the positional signature of the reference's
Cython function (statistics/css/css_cython_parallel.pyx:14).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import GD_WINDOWS_SERIAL, GD_WINDOWS_THREADED, check, lib
from .fet import _ptrs

_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int)


def _run(fn, avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, treshold, runs, drosophila, mds,
         scores, p):
    (av, bv, ap, bp), scores, p = _ptrs(avals, bvals, apos, bpos, scores, p, "p")
    if alen > av.shape[0] or blen > bv.shape[0] or alen > ap.shape[0] or blen > bp.shape[0]:
        raise ValueError("alen/blen exceed the array lengths")
    nwin = int(regend) // int(wstep) if wstep > 0 else 0
    if scores.shape[0] < nwin or p.shape[0] < nwin:
        raise ValueError(f"output arrays must hold regend//wstep = {nwin} windows")
    check(fn(av.ctypes.data_as(_DP), bv.ctypes.data_as(_DP), ap.ctypes.data_as(_IP), bp.ctypes.data_as(_IP),
             int(regstart), int(regend), int(wsize), int(wstep), int(alen), int(blen), int(treshold), int(runs),
             int(drosophila), int(mds), scores.ctypes.data_as(_DP), p.ctypes.data_as(_DP)))


def cluster_separation_scorer(avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, treshold, runs,
                              drosophila, mds, scores, p):
    """Drop-in for css_cython_parallel.cluster_separation_scorer (threaded window set)."""
    _run(lib.gd_css_threadcompute, avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, treshold,
         runs, drosophila, mds, scores, p)


def cluster_separation_scorer_serial(avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, treshold,
                                     runs, drosophila, mds, scores, p):
    """Drop-in for css_cython.cluster_separation_scorer (serial compute() window set)."""
    _run(lib.gd_css_compute, avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, treshold, runs,
         drosophila, mds, scores, p)


def scan(avals, bvals, apos, bpos, regend, wsize=2500, wstep=500, treshold=10, runs=0, seed=None, serial=False,
         drosophila=0, mds=0):
    """One chromosome; drosophila / mds as cluster_separation_scorer (css.c:181-223)."""
    nwin = int(regend) // int(wstep)
    scores = np.zeros(nwin)
    p = np.zeros(nwin)
    (av, bv, ap, bp), scores, p = _ptrs(avals, bvals, apos, bpos, scores, p, "p")
    s = lib.gd_get_seed() if seed is None else int(seed)
    check(lib.gd_css_scan_host_ex(av.ctypes.data_as(_DP), bv.ctypes.data_as(_DP), ap.ctypes.data_as(_IP),
                                  bp.ctypes.data_as(_IP), int(regend), int(wsize), int(wstep), av.shape[0],
                                  bv.shape[0], int(treshold), int(runs), int(drosophila), int(mds), s,
                                  GD_WINDOWS_SERIAL if serial else GD_WINDOWS_THREADED,
                                  scores.ctypes.data_as(_DP), p.ctypes.data_as(_DP)))
    return scores, p


def scan_coords(avals, bvals, apos, bpos, regend, wsize=2500, wstep=500, treshold=10, runs=100, seed=None,
                serial=False, mds=0):
    """Diagnostics (gd_css_coords_host): ``scan`` plus the coordinates the permutation test
    read, shape (regend // wstep, asize + bsize, 2); rows of uncomputed windows are zero."""
    nwin = int(regend) // int(wstep)
    scores = np.zeros(nwin)
    p = np.zeros(nwin)
    (av, bv, ap, bp), scores, p = _ptrs(avals, bvals, apos, bpos, scores, p, "p")
    # get_population_size (comparative.c:25-34): the leading run of pos[0]
    m = int(np.argmax(ap != ap[0]) or ap.shape[0]) + int(np.argmax(bp != bp[0]) or bp.shape[0])
    X = np.zeros((max(nwin, 1), m, 2))
    s = lib.gd_get_seed() if seed is None else int(seed)
    check(lib.gd_css_coords_host(av.ctypes.data_as(_DP), bv.ctypes.data_as(_DP), ap.ctypes.data_as(_IP),
                                 bp.ctypes.data_as(_IP), int(regend), int(wsize), int(wstep), av.shape[0],
                                 bv.shape[0], int(treshold), int(runs), int(mds), s,
                                 GD_WINDOWS_SERIAL if serial else GD_WINDOWS_THREADED,
                                 scores.ctypes.data_as(_DP), p.ctypes.data_as(_DP), X.ctypes.data_as(_DP)))
    X[:nwin][scores == 0] = 0.0
    return scores, p, X[:nwin]
