"""CPU experiment behind the eigenvector solver of the CSS MDS kernels:
twisted factorisations (Parlett & Dhillon), two rounds from a bisection shift, against two
pivoted-LU inverse-iteration solves (the previous kernels' method), both measured against
LAPACK's eigenvectors on the tridiagonal T of real synthetic windows.

For each window of the synthetic chromosome (gdscan.synth, the bench's generator) the count
distance matrix, fill_averages, B = -1/2 Z (D o D) Z and its Householder tridiagonal T
(scipy's hessenberg of the symmetric B) are formed as the kernels do; the shift of each of
the two largest eigenvalues is perturbed by up to TOL ||T|| / 2 (the bisection's stopping
width, CSS_BISECT_TOL), and the kernels' arithmetic is replayed in float64: the Sturm-form
chains (rescaled every 4 steps, e^2 floored at 1e-300), gamma, the twist, the products, the
Rayleigh shift.  Prints the worst |z - q| per round and of the inverse-iteration method.
usage: python tools/twist_accuracy.py [POP] [WINDOWS] [TOL]     (defaults 40 2000 1e-9)"""
import sys
from pathlib import Path

import numpy as np
import scipy.linalg as sl

sys.path.insert(0, str(Path(__file__).resolve().parent.parent /
                       "fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd"))
from gdscan import synth  # noqa: E402

POP = int(sys.argv[1]) if len(sys.argv) > 1 else 40
NWIN = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
TOL = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-9


def tridiagonals(a, nwin):
    av, bv, ap, bp, regend = synth.chromosome(3, 60000, a, a)
    m = 2 * a
    pos = ap[::a]
    G = np.concatenate([av.reshape(-1, a), bv.reshape(-1, a)], axis=1)
    out = []
    for st in range(0, regend - 2500, 500):
        lo, hi = np.searchsorted(pos, st), np.searchsorted(pos, st + 2500, side="right")
        if hi <= lo:
            continue
        g = G[lo:hi]
        P, N = (g == 3).astype(float), (g == -3).astype(float)
        D = P.T @ N + N.T @ P
        if (D < 1e-5).sum() > m * m // 2:
            continue
        D = np.where(D < 1e-5, D[D >= 1e-5].sum() / (m * m), D)
        Z = np.eye(m) - 1.0 / m
        H = sl.hessenberg(-0.5 * Z @ (D * D) @ Z)
        out.append((np.diag(H).copy(), np.diag(H, -1).copy()))
        if len(out) >= nwin:
            break
    return out


def pivots(a, e2):
    """D_k = p_k / p_{k-1} of the chain p_k = a_k p_{k-1} - e2_k p_{k-2}, rescaled every 4 steps"""
    D = np.empty(len(a))
    pm = pc = 1.0
    for k in range(len(a)):
        pn = a[k] * pc - e2[k] * pm
        D[k] = pn / pc
        pm, pc = pc, pn
        if k % 4 == 3:
            ex = np.frexp(max(abs(pm), abs(pc)))[1]
            pm, pc = np.ldexp(pm, -ex), np.ldexp(pc, -ex)
    return D


def twisted(d, e, sig):
    a = d - sig
    ee = np.maximum(e * e, 1e-300)
    Dp = pivots(a, np.concatenate([[0.0], ee]))
    Dm = pivots(a[::-1], np.concatenate([[0.0], ee[::-1]]))[::-1]
    g = Dp + Dm - a
    g = np.where(np.isfinite(g), np.abs(g), np.inf)
    r = int(np.argmin(g))
    z = np.zeros(len(d))
    z[r] = 1.0
    for k in range(r - 1, -1, -1):
        z[k] = -e[k] / Dp[k] * z[k + 1]
    for k in range(r + 1, len(d)):
        z[k] = -e[k - 1] / Dm[k] * z[k - 1]
    nz = z @ z
    return z / np.sqrt(nz), sig + (Dp[r] + Dm[r] - a[r]) / nz


def main():
    rng = np.random.default_rng(1)
    worst = [0.0, 0.0]
    worst_ii = 0.0
    T = tridiagonals(POP, NWIN)
    for d, e in T:
        m = len(d)
        M = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
        w, V = np.linalg.eigh(M)
        nT = max(abs(d).max() + 2 * abs(e).max(), 1e-300)
        for ei, idx in enumerate((m - 1, m - 2)):
            q = V[:, idx]
            sig0 = w[idx] + rng.uniform(-0.5, 0.5) * TOL * nT
            sig = sig0
            for rd in range(2):
                z, sig = twisted(d, e, sig)
                worst[rd] = max(worst[rd], np.linalg.norm(z - np.sign(z @ q) * q))
            k = np.arange(m)
            y = (1.0 if ei == 0 else np.where(k & 1, -1.0, 1.0)) * (0.5 + ((k * 40503 + 977 * (ei + 1)) & 1023) / 1024.0)
            lu = sl.lu_factor(M - sig0 * np.eye(m))
            for _ in range(2):
                y = sl.lu_solve(lu, y)
                y /= np.linalg.norm(y)
            worst_ii = max(worst_ii, np.linalg.norm(y - np.sign(y @ q) * q))
    print(f"{len(T)} windows, {POP}+{POP}, shift within {TOL:g} ||T||: twisted worst |z - q| round 1 {worst[0]:.2e}, "
          f"round 2 {worst[1]:.2e}; two pivoted-LU inverse-iteration solves {worst_ii:.2e}")


if __name__ == "__main__":
    main()
