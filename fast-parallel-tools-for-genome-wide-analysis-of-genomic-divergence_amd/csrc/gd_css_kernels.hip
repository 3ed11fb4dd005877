/*
 * gd_css_kernels.hip -- Cluster Separation Score scan (statistics/css/).
 *
 *   k_css_pack   genotype values -> per-individual SNP bit planes ("== 3", "== -3",
 *                and a per-row "irregular value" plane).  HBM-bound, reads every
 *                value once.
 *   k_css_mds    one workgroup per window: compare_all (css.c:277-327) as popcounts
 *                over the planes, fill_averages (css.c:337-366), double centering
 *                (cmds, css.c:505-530), Householder tridiagonalisation with the
 *                matrix rows held in VGPRs, bisection for the two largest
 *                eigenvalues, inverse iteration, back-transformation, X = Q sqrt(L)
 *                (css.c:533-560), calc_dist + css (css.c:573-647).
 *   k_css_perm   significance_treshold (css.c:727-752): the early-exit permutation
 *                test on the window's distance matrix, staged in LDS.
 *
 * compare_all counts SNPs with (int)v_i * v_j == -9.  For the genotype codes
 * {3, 0, -3, -10000} that is exactly "one is 3 and the other -3", i.e.
 * D = P^T N + N^T P over the window's SNPs, evaluated 64 SNPs per popcount.  A
 * window that holds any other value, or whose A/B slice does not start on a SNP
 * row, takes the literal path: the reference predicate evaluated per SNP with
 * x86 cvttsd2si semantics for the (int) cast.
 *
 * The eigen-solver is not GSL's (GSL is absent from the image).
 * CSS depends only on distances in X, which are invariant to eigenvector signs,
 * so any backward-stable solver agrees with the reference to ~1e-13 relative
 * except in (rare) windows whose second and third eigenvalues nearly coincide.
 */
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cstdlib>
#include <vector>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_internal.h"

namespace {

/* bits [bit, bit + 64) of a bit plane (planes carry 3 words of zero padding) */
__device__ __forceinline__ uint64_t plane_bits64(const uint32_t *pl, int64_t bit) {
  const int64_t w = bit >> 5;
  const int sh = (int)(bit & 31);
  const uint64_t lo = (uint64_t)pl[w] | ((uint64_t)pl[w + 1] << 32);
  const uint64_t hi = pl[w + 2];
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

/* Stops the scheduler from hoisting every LDS broadcast of an unrolled column
 * loop ahead of its FMAs (which would need 4 VGPRs per column on top of the
 * register-resident matrix row); loops issue their loads in groups of 8. */
#define CSS_GROUP_FENCE(j) \
  if (((j) & 7) == 7) asm volatile("" ::: "memory")

/* A copy of x the compiler cannot see through: per-column predicates built from it
 * (j < m, j vs lane) are materialised inside the loop that uses them instead of
 * being hoisted out of the window loop as one live SGPR mask per column. */
#define CSS_OPAQUE_S(x) asm volatile("" : "+s"(x))
#define CSS_OPAQUE_V(x) asm volatile("" : "+v"(x))

/* x86 cvttsd2si: NaN and out-of-range values give INT_MIN */
__device__ __forceinline__ double x86_int(double v) {
  return (v > -2147483649.0 && v < 2147483648.0) ? (double)(int)v : (double)INT_MIN;
}

/* wave64 reductions; the result is lane 0's, so every lane holds the same bits */
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return __shfl(v, 0);
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

/* block reductions over NW waves; red must hold NW doubles */
template <int NW>
__device__ __forceinline__ double block_sum(double v, double *red) {
  v = wave_sum(v);
  if constexpr (NW == 1) {
    return v;
  } else {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = red[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) s += red[k];
    return s;
  }
}
template <int NW>
__device__ __forceinline__ int block_sum_i(int v, double *red) {
  v = wave_sum_i(v);
  if constexpr (NW == 1) {
    return v;
  } else {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = (double)v;
    __syncthreads();
    int s = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += (int)red[k];
    return s;
  }
}
template <int NW>
__device__ __forceinline__ double block_min(double v, double *red) {
  v = wave_min(v);
  if constexpr (NW == 1) {
    return v;
  } else {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = red[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) s = fmin(s, red[k]);
    return s;
  }
}
template <int NW>
__device__ __forceinline__ double block_max(double v, double *red) {
  v = wave_max(v);
  if constexpr (NW == 1) {
    return v;
  } else {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = red[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) s = fmax(s, red[k]);
    return s;
  }
}

__device__ __forceinline__ int chrom_of(const gd_chrom_dev *ch, int nchrom, int64_t w) {
  int lo = 0, hi = nchrom - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ch[mid].w_base <= w)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ double xdist(const double *X, int i, int j) {
  const double dx = X[2 * i] - X[2 * j], dy = X[2 * i + 1] - X[2 * j + 1];
  return sqrt(dx * dx + dy * dy);
}

/* css() (css.c:608-647) for groups A = tracks[0..a), B = tracks[a..m).  The
 * between-group pairs are spread over the workgroup; both kernels call this with
 * the same NT, so the observed and the permuted scores are summed identically. */
template <int NW, class Dist>
__device__ __forceinline__ double css_score(const int *tracks, int a, int b, Dist dist, double *red) {
  constexpr int NT = 64 * NW;
  const int t = threadIdx.x, ab = a * b;
  const float invb = 1.0f / (float)b;
  double bet = 0;
  for (int q = t; q < ab; q += NT) {
    const int ii = (int)(((float)q + 0.5f) * invb); /* exact for q < 2^14 */
    const int jj = q - ii * b;
    bet += dist(tracks[ii], tracks[a + jj]);
  }
  const int m = a + b;
  double ad = 0, bd = 0;
  if (t < a - 1) ad = dist(tracks[t], tracks[t + 1]);
  if (t >= a && t < m - 1) bd = dist(tracks[t], tracks[t + 1]);
  bet = block_sum<NW>(bet, red);
  ad = block_sum<NW>(ad, red);
  bd = block_sum<NW>(bd, red);
  bet = bet / (a * b);
  if (a > 1) ad = ad / (a * a * (a - 1));
  if (b > 1) bd = bd / (b * b * (b - 1));
  return bet - (a + b) * (ad + bd);
}

}  // namespace

/* ------------------------------------------------------------------------ */
/* bit planes: thread (word w, individual i) packs rows [32w, 32w+32)          */
/* ------------------------------------------------------------------------ */
__global__ void __launch_bounds__(256) k_css_pack(const gd_chrom_dev *ch, const gd_css_planes *pl,
                                                  const double *avals, const double *bvals, uint32_t *planes) {
  const gd_chrom_dev &d = ch[blockIdx.y];
  const int pop = blockIdx.z;
  if (d.wend <= 0) return;
  const int s = pop ? d.bsize : d.asize;
  if (s <= 0) return;
  const int64_t rows = (pop ? d.blen : d.alen) / s;
  const double *v = pop ? bvals + d.b_off : avals + d.a_off;
  const gd_css_planes p = pl[blockIdx.y];
  const int64_t nw = pop ? p.wb : p.wa;
  uint32_t *base = planes + (pop ? p.pb : p.pa);
  const int64_t items = ((rows + 31) >> 5) * s;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < items; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = t / s;
    const int i = (int)(t - w * s);
    const int64_t r0 = w * 32;
    const int nb = (int)min<int64_t>(32, rows - r0);
    uint32_t P = 0, N = 0, X = 0;
    const double *src = v + r0 * s + i;
    for (int k = 0; k < nb; ++k) {
      const double x = src[(int64_t)k * s];
      P |= (uint32_t)(x == 3.0) << k;
      N |= (uint32_t)(x == -3.0) << k;
      X |= (uint32_t)(!(x == 3.0 || x == -3.0 || x == 0.0 || x == -10000.0)) << k;
    }
    base[(int64_t)(2 * i) * nw + w] = P;
    base[(int64_t)(2 * i + 1) * nw + w] = N;
    if (X) atomicOr(base + (int64_t)(2 * s) * nw + w, X);
  }
}

/* ------------------------------------------------------------------------ */
/* per-window classical MDS + CSS                                              */
/* ------------------------------------------------------------------------ */
template <int MP>
__global__ void __launch_bounds__(64 * ((MP + 63) / 64))
    k_css_mds(const gd_chrom_dev *ch, int nchrom, const gd_css_planes *pl, const uint32_t *planes,
              const int32_t *lo_a_, const int32_t *hi_a_, const int32_t *lo_b_, const double *avals,
              const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *pvals,
              double *xbuf, uint8_t *status, unsigned *flags) {
  constexpr int NW = (MP + 63) / 64;
  __shared__ double s_row[MP + 2];
  __shared__ double s_v[MP], s_w[MP];
  __shared__ double s_d[MP], s_e[MP], s_e2[MP], s_tau[MP];
  __shared__ uint64_t s_mask[2 * MP];
  __shared__ double s_vals[MP];
  __shared__ double s_y[2][MP];
  __shared__ double s_lu[2][3][MP];
  __shared__ uint8_t s_piv[2][MP];
  __shared__ double s_x[2 * MP];
  __shared__ int s_tr[MP];
  __shared__ double s_lam[2];
  __shared__ double s_red[NW];

  const int i = threadIdx.x;
  const int ii = i < MP ? i : MP - 1; /* clamped LDS index for lanes past MP */
  if (i < MP) s_tr[i] = i;

  for (int64_t w = blockIdx.x; w < wtotal; w += gridDim.x) {
    const int c = chrom_of(ch, nchrom, w);
    const gd_chrom_dev &d = ch[c];
    const int a = d.asize, b = d.bsize, m = a + b;
    const int64_t wl = w - d.w_base;
    const int32_t la = lo_a_[w], ha = hi_a_[w], lb = lo_b_[w];
    const int npos = (ha - la) / a;
    if (npos <= 0) continue;
    if ((int64_t)lb + (int64_t)npos * b > d.blen) {
      if (i == 0) atomicOr(flags, GD_FLAG_B_BOUNDS);
      continue;
    }
    if (m > MP) {
      if (i == 0) atomicOr(flags, GD_FLAG_BAD_SIZE);
      continue;
    }
    const bool row = i < m;
    const gd_css_planes P = pl[c];
    const uint32_t *pa = planes + P.pa, *pb = planes + P.pb;
    const int64_t ra = la / a, rb = lb / b;

    /* ---- regular window?  (rows aligned and no value outside {3,0,-3,-10000}) */
    bool literal = force_literal || (la % a) != 0 || (lb % b) != 0;
    if (!literal) {
      int irr = 0;
      for (int k = i; k * 64 < npos; k += 64 * NW) {
        const int nb = min(64, npos - 64 * k);
        const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
        const uint64_t xa = plane_bits64(pa + (int64_t)(2 * a) * P.wa, ra + 64 * k) & tail;
        const uint64_t xb = plane_bits64(pb + (int64_t)(2 * b) * P.wb, rb + 64 * k) & tail;
        irr |= (xa | xb) != 0;
      }
      literal = __syncthreads_or(irr);
    }

    /* ---- compare_all: D[i][j] in registers, lane i = row i */
    double A[MP];
    {
      int acc[MP];
#pragma unroll
      for (int j = 0; j < MP; ++j) acc[j] = 0;
      if (!literal) {
        for (int k = 0; k * 64 < npos; ++k) {
          const int nb = min(64, npos - 64 * k);
          const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
          __syncthreads();
          if (row) {
            const uint32_t *base = i < a ? pa + (int64_t)(2 * i) * P.wa : pb + (int64_t)(2 * (i - a)) * P.wb;
            const int64_t nw = i < a ? P.wa : P.wb;
            const int64_t r = (i < a ? ra : rb) + 64 * k;
            s_mask[2 * i] = plane_bits64(base, r) & tail;
            s_mask[2 * i + 1] = plane_bits64(base + nw, r) & tail;
          } else if (i < MP) {
            s_mask[2 * i] = 0;
            s_mask[2 * i + 1] = 0;
          }
          __syncthreads();
          const uint64_t Pi = s_mask[2 * ii], Ni = s_mask[2 * ii + 1];
#pragma unroll
          for (int j = 0; j < MP; ++j) {
            const uint64_t Pj = s_mask[2 * j], Nj = s_mask[2 * j + 1];
            acc[j] += __popcll(Pi & Nj) + __popcll(Ni & Pj);
            CSS_GROUP_FENCE(j);
          }
        }
      } else {
        const double *av = avals + d.a_off + la, *bv = bvals + d.b_off + lb;
        for (int k = 0; k < npos; ++k) {
          __syncthreads();
          if (row) s_vals[i] = i < a ? av[(int64_t)k * a + i] : bv[(int64_t)k * b + (i - a)];
          __syncthreads();
          const double vi = s_vals[ii];
          int io = i, mo = m, ao = a;
          CSS_OPAQUE_V(io);
          CSS_OPAQUE_S(mo);
          CSS_OPAQUE_S(ao);
#pragma unroll
          for (int j = 0; j < MP; ++j) {
            /* the diagonal never counts: (int)v * v >= 0 */
            if (j < mo) {
              const double vj = s_vals[j];
              /* the reference casts the row element of the larger index within a
               * population and the A element across populations (css.c:281-326) */
              const bool cast_i = ((io < ao) == (j < ao)) ? (io > j) : (io < ao);
              const double prod = cast_i ? x86_int(vi) * vj : x86_int(vj) * vi;
              acc[j] += prod == -9.0;
            }
          }
        }
      }
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int j = 0; j < MP; ++j) A[j] = (row && j < mo) ? (double)acc[j] : 0.0;
    }

    /* ---- fill_averages: entries < 1e-5 (diagonal included) count as unknown */
    {
      int unval = 0;
      double sum = 0;
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int j = 0; j < MP; ++j) {
        if (row && j < mo) {
          if (A[j] < 0.00001)
            ++unval;
          else
            sum += A[j];
        }
      }
      unval = block_sum_i<NW>(unval, s_red);
      sum = block_sum<NW>(sum, s_red); /* sums of integers: exact in any order */
      const int tot = m * m;
      if (unval > tot / 2) continue; /* discarded window: outputs untouched */
      const double avg = sum / tot;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int j = 0; j < MP; ++j)
        if (row && j < mo && A[j] < 0.00001) A[j] = avg;
    }

    /* ---- B = -1/2 Z (D o D) Z, Z = I - 11^T/m, by double centering */
    double zero_tol;
    {
      double rs = 0;
#pragma unroll
      for (int j = 0; j < MP; ++j) {
        A[j] = A[j] * A[j];
        rs += A[j];
      }
      const double ri = row ? rs / m : 0.0;
      __syncthreads();
      if (i < MP) s_v[i] = ri;
      const double g = block_sum<NW>(ri, s_red) / m;
      __syncthreads();
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int j = 0; j < MP; ++j) A[j] = (row && j < mo) ? -0.5 * ((A[j] - (ri + s_v[j])) + g) : 0.0;
      double f2 = 0;
#pragma unroll
      for (int j = 0; j < MP; ++j) f2 = fma(A[j], A[j], f2);
      /* eigenvalues within rounding of 0 count as 0 (oracle/css_oracle.c, cmds) */
      zero_tol = 64.0 * m * DBL_EPSILON * sqrt(block_sum<NW>(f2, s_red));
    }

    /* ---- Householder tridiagonalisation (LAPACK dsytd2, lower).  Column k of the
     * trailing matrix is read from row k (symmetry); after step k the dead column k
     * of each row holds that row's element of the reflector v_k. */
    for (int k = 0; k < m; ++k) {
      __syncthreads();
      if (i == k) {
#pragma unroll
        for (int j = 0; j < MP; ++j) s_row[j] = A[j];
      }
      __syncthreads();
      if (k >= m - 2) {
        if (i == 0) {
          s_d[k] = s_row[k];
          if (k == m - 2) s_e[k] = s_row[k + 1];
        }
        continue;
      }
      const double xi = (i > k + 1 && row) ? s_row[ii] : 0.0;
      const double alpha = s_row[k + 1];
      const double sigma = block_sum<NW>(xi * xi, s_red);
      double tau = 0.0, beta = alpha, scale = 0.0;
      if (sigma != 0.0) {
        beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
        tau = (beta - alpha) / beta;
        scale = 1.0 / (alpha - beta);
      }
      const double vi = (i == k + 1) ? 1.0 : xi * scale;
      if (i == 0) {
        s_d[k] = s_row[k];
        s_e[k] = beta;
        s_tau[k] = tau;
      }
      if (i < MP) s_v[i] = vi;
      __syncthreads();
      double p0 = 0, p1 = 0, p2 = 0, p3 = 0;
#pragma unroll
      for (int j = 0; j < MP; j += 4) {
        p0 = fma(A[j], s_v[j], p0);
        if (j + 1 < MP) p1 = fma(A[j + 1], s_v[j + 1], p1);
        if (j + 2 < MP) p2 = fma(A[j + 2], s_v[j + 2], p2);
        if (j + 3 < MP) p3 = fma(A[j + 3], s_v[j + 3], p3);
        CSS_GROUP_FENCE(j + 4);
      }
      const double pi = (i > k && row) ? tau * ((p0 + p1) + (p2 + p3)) : 0.0;
      const double K = -0.5 * tau * block_sum<NW>(pi * vi, s_red);
      const double wi = pi + K * vi;
      if (i < MP) s_w[i] = wi;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < MP; ++j) {
        A[j] = fma(-vi, s_w[j], fma(-wi, s_v[j], A[j]));
        CSS_GROUP_FENCE(j);
      }
#pragma unroll
      for (int j = 0; j < MP; ++j) A[j] = (j == k) ? vi : A[j];
    }
    __syncthreads();

    /* ---- the two largest eigenvalues of T: Gershgorin bounds, then 33-section
     * Sturm-count bisection, one half-wave per eigenvalue */
    double glo, ghi, pivmin;
    {
      double lo = DBL_MAX, hi = -DBL_MAX, e2m = 0;
      if (row) {
        const double r = (i > 0 ? fabs(s_e[i - 1]) : 0.0) + (i < m - 1 ? fabs(s_e[i]) : 0.0);
        lo = s_d[i] - r;
        hi = s_d[i] + r;
        if (i < m - 1) {
          const double e2 = s_e[i] * s_e[i];
          s_e2[i] = e2;
          e2m = e2;
        }
      }
      glo = block_min<NW>(lo, s_red);
      ghi = block_max<NW>(hi, s_red);
      e2m = block_max<NW>(e2m, s_red);
      pivmin = DBL_MIN * fmax(1.0, e2m);
      const double tn = fmax(fabs(glo), fabs(ghi));
      glo -= 2.0 * DBL_EPSILON * tn * m + 2.0 * pivmin;
      ghi += 2.0 * DBL_EPSILON * tn * m + 2.0 * pivmin;
    }
    __syncthreads();
    if (i < 64) {
      const int h = i >> 5, j = i & 31;
      const int target = m - 1 - h; /* ascending index of the eigenvalue */
      double l = glo, u = ghi;
      for (int it = 0; it < 80; ++it) {
        const double x = l + (u - l) * ((double)(j + 1) * (1.0 / 33.0));
        int cnt = 0;
        double q = s_d[0] - x;
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
        for (int k = 1; k < m; ++k) {
          q = (s_d[k] - x) - s_e2[k - 1] / q;
          if (fabs(q) < pivmin) q = -pivmin;
          cnt += q < 0.0;
        }
        double nl = cnt <= target ? x : l;
        double nu = cnt <= target ? u : x;
#pragma unroll
        for (int o = 16; o >= 1; o >>= 1) {
          nl = fmax(nl, __shfl_xor(nl, o));
          nu = fmin(nu, __shfl_xor(nu, o));
        }
        nl = __shfl(nl, i & 32);
        nu = __shfl(nu, i & 32);
        const bool same = (nl == l && nu == u);
        l = nl;
        u = nu;
        const bool conv = same || (u - l) <= 2.0 * DBL_EPSILON * fmax(fabs(l), fabs(u)) + pivmin;
        if (__all(conv)) break;
      }
      if (j == 0) {
        const double lam = 0.5 * (l + u);
        s_lam[h] = fabs(lam) <= zero_tol ? 0.0 : lam;
      }
    }
    __syncthreads();

    /* ---- eigenvectors of T by inverse iteration (partial-pivot LU of T - lam I),
     * lane 0 for the largest, lane 1 for the second */
    if (i < 2) {
      const double sig = s_lam[i];
      const double tiny = DBL_EPSILON * fmax(fmax(fabs(glo), fabs(ghi)), DBL_MIN);
      double *U0 = s_lu[i][0], *U1 = s_lu[i][1], *U2 = s_lu[i][2];
      double *y = s_y[i];
      double *ml = s_x + i * MP; /* elimination multipliers; s_x is free until X is formed */
      uint8_t *pv = s_piv[i];
      double c0 = s_d[0] - sig, c1 = m > 1 ? s_e[0] : 0.0;
      for (int k = 0; k < m - 1; ++k) {
        const double n0 = s_e[k], n1 = s_d[k + 1] - sig, n2 = (k + 2 < m) ? s_e[k + 1] : 0.0;
        if (fabs(c0) >= fabs(n0)) {
          const double t = (c0 != 0.0) ? n0 / c0 : 0.0;
          U0[k] = c0;
          U1[k] = c1;
          U2[k] = 0.0;
          ml[k] = t;
          pv[k] = 0;
          c0 = n1 - t * c1;
          c1 = n2;
        } else {
          const double t = c0 / n0;
          U0[k] = n0;
          U1[k] = n1;
          U2[k] = n2;
          ml[k] = t;
          pv[k] = 1;
          c0 = c1 - t * n1;
          c1 = -t * n2;
        }
      }
      U0[m - 1] = c0;
      for (int k = 0; k < m; ++k)
        if (U0[k] == 0.0) U0[k] = tiny;
      /* start vector: deterministic, not orthogonal to anything in practice */
      for (int k = 0; k < m; ++k) {
        const double f = (double)((k * 40503u + 977u * (unsigned)(i + 1)) & 1023u) / 1024.0;
        y[k] = (i == 0 ? 1.0 : ((k & 1) ? -1.0 : 1.0)) * (0.5 + f);
      }
      for (int itn = 0; itn < 3; ++itn) {
        for (int k = 0; k < m - 1; ++k) {
          if (pv[k]) {
            const double t = y[k];
            y[k] = y[k + 1];
            y[k + 1] = t;
          }
          y[k + 1] -= ml[k] * y[k];
        }
        y[m - 1] = y[m - 1] / U0[m - 1];
        if (m > 1) y[m - 2] = (y[m - 2] - U1[m - 2] * y[m - 1]) / U0[m - 2];
        for (int k = m - 3; k >= 0; --k) y[k] = (y[k] - U1[k] * y[k + 1] - U2[k] * y[k + 2]) / U0[k];
        double mx = 0;
        for (int k = 0; k < m; ++k) mx = fmax(mx, fabs(y[k]));
        const double inv = mx > 0 ? 1.0 / mx : 1.0;
        double nrm = 0;
        for (int k = 0; k < m; ++k) {
          y[k] *= inv;
          nrm += y[k] * y[k];
        }
        const double r = 1.0 / sqrt(nrm);
        for (int k = 0; k < m; ++k) y[k] *= r;
      }
    }
    __syncthreads();
    /* orthogonalise the second vector against the first (close eigenvalues) */
    double y1 = row ? s_y[0][ii] : 0.0, y2 = row ? s_y[1][ii] : 0.0;
    {
      const double dt = block_sum<NW>(y1 * y2, s_red);
      y2 -= dt * y1;
      const double n2 = block_sum<NW>(y2 * y2, s_red);
      y2 *= 1.0 / sqrt(n2);
    }

    /* ---- back-transformation y <- H_0 H_1 ... H_{m-3} y */
#pragma unroll
    for (int k = MP - 3; k >= 0; --k) {
      if (k <= m - 3) {
        const double vk = row ? A[k] : 0.0;
        const double t = s_tau[k];
        const double d1 = block_sum<NW>(vk * y1, s_red);
        const double d2 = block_sum<NW>(vk * y2, s_red);
        y1 -= (t * d1) * vk;
        y2 -= (t * d2) * vk;
      }
    }

    /* ---- X = Q sqrt(L) (css.c:545-556), then calc_dist + css on identity groups */
    {
      const double L1 = sqrt(s_lam[0]), L2 = sqrt(s_lam[1]);
      __syncthreads();
      if (row) {
        s_x[2 * i] = y1 * L1 + y2 * 0.0;
        s_x[2 * i + 1] = y1 * 0.0 + y2 * L2;
      }
      __syncthreads();
    }
    const double score = css_score<NW>(s_tr, a, b, [&](int p, int q) { return xdist(s_x, p, q); }, s_red);
    if (score == -1.0) continue; /* the reference's "discarded" marker (css.c:127) */
    if (i == 0) {
      scores[d.w_out + wl] = score;
      if (!want_x) pvals[d.w_out + wl] = 1.0; /* runs == 0: p = (0 + 1) / (0 + 1) */
    }
    if (want_x) {
      if (i < 2 * MP) xbuf[w * 2 * MP + i] = (i < 2 * m) ? s_x[i] : 0.0;
      if (i + 64 * NW < 2 * MP) xbuf[w * 2 * MP + i + 64 * NW] = (i + 64 * NW < 2 * m) ? s_x[i + 64 * NW] : 0.0;
      if (i == 0) status[w] = 1;
    }
  }
}

/* ------------------------------------------------------------------------ */
/* significance_treshold: early-exit Monte-Carlo p on the window's S matrix   */
/* ------------------------------------------------------------------------ */
template <int MP>
__global__ void __launch_bounds__(64 * ((MP + 63) / 64))
    k_css_perm(const gd_chrom_dev *ch, int nchrom, const double *xbuf, const uint8_t *status, int64_t wtotal, int treshold, int runs, double *pvals) {
  constexpr int NW = (MP + 63) / 64, NT = 64 * NW;
  __shared__ double s_S[MP * MP];
  __shared__ double s_x[2 * MP];
  __shared__ int s_tr[MP];
  __shared__ gd_randint s_rd[MP + 1];
  __shared__ double s_red[NW];
  const int i = threadIdx.x;
  for (int n = i; n <= MP; n += NT) s_rd[n] = gd_randint_make(n < 1 ? 1u : (uint32_t)n);

  for (int64_t w = blockIdx.x; w < wtotal; w += gridDim.x) {
    if (!status[w]) continue;
    const int c = chrom_of(ch, nchrom, w);
    const gd_chrom_dev &d = ch[c];
    const int a = d.asize, b = d.bsize, m = a + b;
    const int64_t wl = w - d.w_base;
    __syncthreads();
    if (i < 2 * MP) s_x[i] = xbuf[w * 2 * MP + i];
    if (i + NT < 2 * MP) s_x[i + NT] = xbuf[w * 2 * MP + i + NT];
    if (i < m) s_tr[i] = i;
    __syncthreads();
    for (int e = i; e < m * m; e += NT) {
      const int r = e / m, q = e - r * m;
      s_S[e] = xdist(s_x, r, q);
    }
    __syncthreads();
    auto dist = [&](int p, int q) { return s_S[p * m + q]; };
    /* the observed score, summed exactly as the permuted ones */
    const double score = css_score<NW>(s_tr, a, b, dist, s_red);
    uint64_t x = gd_window_state(d.seed, GD_STREAM_CSS, wl);
    int hits = 0, nscores = 0;
    while (hits < treshold && nscores < runs) {
      __syncthreads();
      if (i == 0) {
        for (int k = m - 1; k > 0; --k) {
          const gd_randint rd = s_rd[k + 1];
          uint32_t r;
          do {
            x = gd_lcg_next(x);
            r = gd_lcg_value(x);
          } while (r > rd.limit);
          const int idx = (int)gd_randint_mod(&rd, r);
          const int t = s_tr[k];
          s_tr[k] = s_tr[idx];
          s_tr[idx] = t;
        }
      }
      __syncthreads();
      const double ps = css_score<NW>(s_tr, a, b, dist, s_red);
      hits += ps >= score;
      ++nscores;
    }
    if (i == 0) pvals[d.w_out + wl] = (hits + 1) * 1.0 / (nscores + 1);
  }
}

/* ------------------------------------------------------------------------ */
int gd_css_tier(int m) {
  static const int tiers[] = {24, 40, 64, 80, 96};
  for (int t : tiers)
    if (m <= t) return t;
  return 0;
}

template <int MP>
static int launch_tier(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                       const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                       const double *bvals, int64_t wtotal, int treshold, int runs, double *scores, double *p,
                       double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s) {
  constexpr int NT = 64 * ((MP + 63) / 64);
  const int want_x = (runs > 0 && treshold > 0) ? 1 : 0;
  const unsigned gx = (unsigned)std::min<int64_t>(wtotal, 256 * 32);
  const char *fl = getenv("GD_CSS_FORCE_LITERAL"); /* diagnostics: per-SNP predicate for every window */
  const int force_literal = (fl && fl[0] == '1') ? 1 : 0;
  hipLaunchKernelGGL(k_css_mds<MP>, dim3(gx), dim3(NT), 0, s, d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals,
                     bvals, wtotal, want_x, force_literal, scores, p, xbuf, status, flags);
  if (hipGetLastError() != hipSuccess) return GD_ERR_HIP;
  if (want_x) {
    hipLaunchKernelGGL(k_css_perm<MP>, dim3(gx), dim3(NT), 0, s, d_ch, nchrom, xbuf, status, wtotal,
                       treshold, runs, p);
    if (hipGetLastError() != hipSuccess) return GD_ERR_HIP;
  }
  return GD_OK;
}

int gd_css_launch(int mp, const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, uint32_t *planes,
                  const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                  const double *bvals, int64_t wtotal, int64_t max_rows_words, int treshold, int runs,
                  double *scores, double *p, double *xbuf, uint8_t *status, unsigned *flags,
                  hipStream_t s) {
  {
    const unsigned gx = (unsigned)std::min<int64_t>((max_rows_words * 8 + 255) / 256, std::max(1, 16384 / nchrom));
    hipLaunchKernelGGL(k_css_pack, dim3(std::max(1u, gx), nchrom, 2), dim3(256), 0, s, d_ch, d_pl, avals, bvals,
                       planes);
    if (hipGetLastError() != hipSuccess) return GD_ERR_HIP;
  }
  switch (mp) {
    case 24:
      return launch_tier<24>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, treshold, runs,
                             scores, p, xbuf, status, flags, s);
    case 40:
      return launch_tier<40>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, treshold, runs,
                             scores, p, xbuf, status, flags, s);
    case 64:
      return launch_tier<64>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, treshold, runs,
                             scores, p, xbuf, status, flags, s);
    case 80:
      return launch_tier<80>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, treshold, runs,
                             scores, p, xbuf, status, flags, s);
    case 96:
      return launch_tier<96>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, treshold, runs,
                             scores, p, xbuf, status, flags, s);
  }
  return GD_ERR_SIZE;
}
