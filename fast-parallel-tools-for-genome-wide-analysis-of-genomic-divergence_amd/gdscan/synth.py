"""Seeded synthetic SNP tracks, bit-identical to the
device generator ``gd_synth_*`` in csrc/gd_synth.hip.

A chromosome is two GTrack "valued points" tracks, one per population, laid out
exactly as HyperBrowser hands them to the statistic (FisherExactScoreStat.py:35-40,
VCFConvert.py:75-86): one entry per (SNP, individual), SNP-major, positions
repeated once per individual, values in {3, 0, -3, -10000}
(hom-major, het, hom-minor, missing).

Generator (all integer hashing; the few float ops are IEEE basic ops):
  h(c, s, tag)  = mix64(mix64(mix64(seed ^ c) ^ s) ^ tag)       (splitmix64 finaliser)
  gap_s         = 1 + h(c, s, GAP) % 99                         -> pos_s = cumsum(gap)
  q_A           = Q[h(c, s, FREQ) >> 52]                        Q = Beta(1/2,1/2) quantiles
  q_B           = clip(q_A + 0.2 * (sum_{t<12} u_t - 6), 0, 1)  Irwin-Hall normal noise
                  = 1 - q_A inside 5 "divergent islands" of 200 SNPs
  genotype      = -3 if u < q^2, 0 if u < q^2 + 2q(1-q), else 3; 2% set to -10000
"""
from __future__ import annotations

import numpy as np

MASTER_SEED = 20261015
TAG_GAP = 0x11
TAG_FREQ = 0x22
TAG_NOISE = 0x100  # + t, t < 12
TAG_ISLAND = 0x33
TAG_GENO = 0x1000000  # + (pop << 20) + individual
TAG_MISS = 0x2000000  # + (pop << 20) + individual
N_ISLANDS = 5
ISLAND_SNPS = 200
QTAB_BITS = 12

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix64(z):
    z = z ^ (z >> np.uint64(30))
    z = z * _M1
    z = z ^ (z >> np.uint64(27))
    z = z * _M2
    z = z ^ (z >> np.uint64(31))
    return z


def _h(seed, c, s, tag):
    with np.errstate(over="ignore"):
        x = _mix64(np.uint64(seed) ^ np.uint64(c))
        x = _mix64(x ^ np.asarray(s, dtype=np.uint64))
        return _mix64(x ^ np.asarray(tag, dtype=np.uint64))


def _unit(h):
    return (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def freq_table() -> np.ndarray:
    """Beta(1/2, 1/2) quantiles sin^2(pi u / 2) at u = (i + 0.5) / 4096."""
    n = 1 << QTAB_BITS
    u = (np.arange(n, dtype=np.float64) + 0.5) / n
    return np.sin(np.pi * u / 2.0) ** 2


def positions(c: int, nsnp: int, seed: int = MASTER_SEED) -> np.ndarray:
    """SNP positions of chromosome c (one per row), as chromosome() places them."""
    s = np.arange(nsnp, dtype=np.uint64)
    return np.cumsum(1 + (_h(seed, c, s, TAG_GAP) % np.uint64(99)).astype(np.int64))


def regend(c: int, nsnp: int, seed: int = MASTER_SEED) -> int:
    """chromosome(c, ...)[4] without generating the genotypes (last position + 1)."""
    return int(positions(c, nsnp, seed)[-1]) + 1


def chromosome(c: int, nsnp: int, asize: int, bsize: int, seed: int = MASTER_SEED):
    """Return (avals, bvals, apos, bpos, regend) for chromosome c."""
    s = np.arange(nsnp, dtype=np.uint64)
    pos = positions(c, nsnp, seed)
    if pos[-1] >= 2**31 - 1:
        raise ValueError("chromosome too long for int32 positions")
    qtab = freq_table()
    qa = qtab[(_h(seed, c, s, TAG_FREQ) >> np.uint64(64 - QTAB_BITS)).astype(np.int64)]
    acc = np.zeros(nsnp)
    for t in range(12):
        acc = acc + _unit(_h(seed, c, s, TAG_NOISE + t))
    qb = qa + 0.2 * (acc - 6.0)
    qb = np.minimum(np.maximum(qb, 0.0), 1.0)
    span = max(1, nsnp - ISLAND_SNPS)
    for k in range(N_ISLANDS):
        st = int(_h(seed, c, k, TAG_ISLAND) % np.uint64(span))
        sl = slice(st, min(nsnp, st + ISLAND_SNPS))
        qb[sl] = 1.0 - qa[sl]
    out = []
    for pop, (q, size) in enumerate(((qa, asize), (qb, bsize))):
        j = np.arange(size, dtype=np.uint64)
        tag_g = np.uint64(TAG_GENO) + (np.uint64(pop) << np.uint64(20)) + j
        tag_m = np.uint64(TAG_MISS) + (np.uint64(pop) << np.uint64(20)) + j
        u = _unit(_h(seed, c, s[:, None], tag_g[None, :]))
        qq = q[:, None]
        t1 = qq * qq
        t2 = t1 + (2.0 * qq) * (1.0 - qq)
        v = np.where(u < t1, -3.0, np.where(u < t2, 0.0, 3.0))
        miss = (_h(seed, c, s[:, None], tag_m[None, :]) % np.uint64(50)) == 0
        v[miss] = -10000.0
        out.append(np.ascontiguousarray(v.reshape(-1)))
    apos = np.repeat(pos.astype(np.int32), asize)
    bpos = np.repeat(pos.astype(np.int32), bsize)
    regend = int(pos[-1]) + 1
    return out[0], out[1], apos, bpos, regend
