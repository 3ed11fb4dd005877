/*
 * gd_css_smacof.hip -- the CSS options beside classical MDS on the count metric
 * (SURVEY.md 8(f) rank 3):
 *
 *   k_css_smacof    SMACOF multidimensional scaling (css.c:767-938): mds = 1 runs
 *                   smacof_runs (css.c:807-835, 4 runs from drand48 starts), mds = 2
 *                   one run started from the classical-MDS coordinates k_css_mds (or
 *                   k_css_freq_cmds) leaves in xbuf (css.c:211-213); on the count
 *                   metric or the drosophila allele-frequency metric
 *   k_css_freq_cmds compare_freq (css.c:245-264) + fill_averages + classical MDS of
 *                   the 2 x 2 dissimilarity matrix + css, one lane per window (mds = 0)
 *
 * SMACOF follows the reference's evaluation order -- smacof / guttman_transform /
 * stress (css.c:855-938, 767-787) with the dgemm of css.c:421-430 as GSL's cblas
 * row-major loop -- so a literal CPU restatement (oracle/css_options_oracle.c)
 * reproduces the iteration count and the coordinates bit for bit.  One workgroup per
 * window, lane i = individual i; a pass over a configuration Z (double-buffered in
 * LDS) computes
 *   pass A  j = m-1 .. 0 (j != i): d_ij = |z_i - z_j|, b_ij = d_ij < 1e-5 ? 0 :
 *           -delta_ij / d_ij summed in that order for b_ii, and for j < i the stress
 *           term (d_ij - delta_ij)^2 into a packed triangle
 *   pass B  k = 0 .. m-1: x_i += b_ik z_k, terms with b_ik == 0 skipped as the cblas
 *           loop skips them; b_ik is recomputed (bit-identical) instead of stored
 *   stress  one lane sums the triangle in the reference's (i desc, j desc) order
 * i.e. the stress of Z and the Guttman transform of Z in one pass; the loop keeps
 * the reference's exit test (sigma_prev - sigma > 1e-6 && k <= 300).  The
 * dissimilarities are the window's integer counts (zero entries read as the
 * fill_averages mean) held in LDS as 16-bit counts.
 *
 * Documented deviations: the drand48 starts come from the window's own
 * stream (seed, window, stream 2) instead of the time-seeded global drand48; when no
 * run reaches stress < 99999 the reference keeps X from an earlier window (its per-call
 * scratch), here the run of least stress is used.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdint>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_internal.h"

#define SM_MAX_ITERS 300   /* css.c:211, 213 */
#define SM_EPS 0.000001    /* css.c:211, 213 */
#define SM_NINIT 4         /* css.c:211 */
#define SM_SIGMA0 99999.0  /* smacof_runs' initial sigma_best, css.c:816 */

namespace {

__device__ __forceinline__ int sm_chrom_of(const gd_chrom_dev *ch, int nchrom, int64_t w) {
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

/* bits [bit, bit + 64) of a bit plane (planes carry 3 words of zero padding) */
__device__ __forceinline__ uint64_t sm_plane_bits64(const uint32_t *pl, int64_t bit) {
  const int64_t w = bit >> 5;
  const int sh = (int)(bit & 31);
  const uint64_t lo = (uint64_t)pl[w] | ((uint64_t)pl[w + 1] << 32);
  const uint64_t hi = pl[w + 2];
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

/* x86 cvttsd2si: NaN and out-of-range values give INT_MIN */
__device__ __forceinline__ double sm_x86_int(double v) {
  return (v > -2147483649.0 && v < 2147483648.0) ? (double)(int)v : (double)INT_MIN;
}

/* calc_dist (css.c:573-587) of two points */
__device__ __forceinline__ double sm_dist(double xi0, double xi1, double xj0, double xj1) {
  const double dx = xi0 - xj0, dy = xi1 - xj1;
  return sqrt(dx * dx + dy * dy);
}

/* dabs (css.c:229-234) */
__device__ __forceinline__ double sm_dabs(double x) { return x < 0 ? -1 * x : x; }

/* css() (css.c:608-647) of X (m x 2, row-major) on the identity groups, serial in the
 * reference's loop order */
__device__ double sm_css_serial(const double *X, int a, int b) {
  double bet = 0.0, ad = 0.0, bd = 0.0;
  for (int i = a; i--;)
    for (int j = b; j--;) bet += sm_dist(X[2 * (a + j)], X[2 * (a + j) + 1], X[2 * i], X[2 * i + 1]);
  bet = bet / (a * b);
  if (a > 1) {
    for (int i = a - 1; i--;) ad += sm_dist(X[2 * (i + 1)], X[2 * (i + 1) + 1], X[2 * i], X[2 * i + 1]);
    ad = ad / (a * a * (a - 1));
  }
  if (b > 1) {
    for (int i = b - 1; i--;)
      bd += sm_dist(X[2 * (a + i + 1)], X[2 * (a + i + 1) + 1], X[2 * (a + i)], X[2 * (a + i) + 1]);
    bd = bd / (b * b * (b - 1));
  }
  return bet - (a + b) * (ad + bd);
}

/* the k-th drand48() value of a stream (k >= 1): advance k steps, then state / 2^48
 * (glibc erand48_r) */
__device__ __forceinline__ double sm_drand48_at(uint64_t x0, uint64_t k) {
  return (double)gd_affine_apply(gd_lcg_jump(k), x0) * (1.0 / 281474976710656.0);
}

}  // namespace

/* ------------------------------------------------------------------------ */
/* compare_freq + classical MDS of the 2 x 2 matrix + css, one lane per window */
/* (drosophila metric, asize = bsize = 1).  B = -1/2 Z (D o D) Z by the two     */
/* naive products of cmds (css.c:505-530); its eigenpairs in closed form;       */
/* |lambda| <= 64 m eps ||B||_F counts as 0 (as k_css_mds).                      */
/* ------------------------------------------------------------------------ */
__global__ void __launch_bounds__(256)
    k_css_freq_cmds(const gd_chrom_dev *ch, int nchrom, const int32_t *lo_a_, const int32_t *hi_a_,
                    const int32_t *lo_b_, const double *avals, const double *bvals, int64_t wtotal, int want_x,
                    int xstride, double *scores, double *pvals, double *xbuf, uint8_t *status, unsigned *flags) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= wtotal) return;
  const int c = sm_chrom_of(ch, nchrom, w);
  const gd_chrom_dev &d = ch[c];
  const int64_t wl = w - d.w_base;
  const int32_t la = lo_a_[w], ha = hi_a_[w], lb = lo_b_[w];
  const int a = d.asize, b = d.bsize;
  if (a != 1 || b != 1) {
    atomicOr(flags, GD_FLAG_BAD_SIZE);
    return;
  }
  const int npos = ha - la;
  if (npos <= 0) return;
  if ((int64_t)lb + npos > d.blen) {
    atomicOr(flags, GD_FLAG_B_BOUNDS);
    return;
  }
  const double *av = avals + d.a_off + la, *bv = bvals + d.b_off + lb;
  double f = 0.0;
  for (int k = npos; k--;) f += sm_dabs(av[k] - bv[k]);
  f = f / npos;
  /* fill_averages on [[0, f], [f, 0]]: the diagonal is unknown, f too if < 1e-5 */
  const int unval = 2 + (f < 0.00001 ? 2 : 0);
  if (unval > 4 / 2) return;
  const double avg = (f + f) / 4;
  double D[4] = {avg, f, f, avg}, Bm[4], T[4];
  const double Z[4] = {(2 - 1) / (2 * 1.0), -1.0 / 2, -1.0 / 2, (2 - 1) / (2 * 1.0)};
  for (int e = 0; e < 4; ++e) Bm[e] = D[e] * D[e];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) T[2 * i + j] = Z[2 * i] * Bm[j] + Z[2 * i + 1] * Bm[2 + j];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) D[2 * i + j] = -0.5 * (T[2 * i] * Z[j] + T[2 * i + 1] * Z[2 + j]);
  /* symmetric 2 x 2 eigenpairs: p, q, r = B00, B01, B11 */
  const double p = D[0], q = 0.5 * (D[1] + D[2]), r = D[3];
  const double hm = 0.5 * (p + r), hd = 0.5 * (p - r);
  const double rad = sqrt(hd * hd + q * q);
  const double zero_tol = 64.0 * 2 * DBL_EPSILON * sqrt(p * p + 2 * q * q + r * r);
  double l1 = hm + rad, l2 = hm - rad;
  if (fabs(l1) <= zero_tol) l1 = 0.0;
  if (fabs(l2) <= zero_tol) l2 = 0.0;
  /* eigenvector of l1: the longer of (q, l1 - p) and (l1 - r, q), normalised */
  double v0, v1;
  {
    const double a0 = q, a1 = l1 - p, b0 = l1 - r, b1 = q;
    const double na = a0 * a0 + a1 * a1, nb = b0 * b0 + b1 * b1;
    if (na >= nb && na > 0) {
      v0 = a0 / sqrt(na);
      v1 = a1 / sqrt(na);
    } else if (nb > 0) {
      v0 = b0 / sqrt(nb);
      v1 = b1 / sqrt(nb);
    } else {
      v0 = 1.0;
      v1 = 0.0;
    }
  }
  const double L1 = sqrt(l1), L2 = sqrt(l2);
  /* X = Q sqrt(L) (css.c:545-556); the second eigenvector is (-v1, v0) */
  const double X[4] = {v0 * L1 + (-v1) * 0.0, v0 * 0.0 + (-v1) * L2, v1 * L1 + v0 * 0.0, v1 * 0.0 + v0 * L2};
  const double score = sm_css_serial(X, 1, 1);
  if (score == -1.0) return; /* the reference's "discarded" marker (css.c:127) */
  scores[d.w_out + wl] = score;
  if (want_x) {
    for (int e = 0; e < xstride; ++e) xbuf[w * xstride + e] = e < 4 ? X[e] : 0.0;
    status[w] = 1;
  } else {
    pvals[d.w_out + wl] = 1.0;
  }
}

/* ------------------------------------------------------------------------ */
/* SMACOF (mds = 1: smacof_runs; mds = 2: one run from the cmds coordinates)   */
/* ------------------------------------------------------------------------ */
/* BIG (the general path, m above the register tiers): the counts and the stress triangle
 * live in the workgroup's global-memory slab (tri first, mpb (mpb - 1) / 2 doubles for the
 * batch's tier mpb, then the counts at column stride ld) and the workgroups loop over
 * windows; otherwise both are in LDS, one workgroup per window. */
/* threads of a tier: one per individual up to 1024, two individuals per thread above */
template <int MP>
constexpr int sm_nt() { return MP > 1024 ? 1024 : 64 * ((MP + 63) / 64); }
template <int MP, bool FREQ, bool BIG>
__global__ void __launch_bounds__(sm_nt<MP>())
    k_css_smacof(const gd_chrom_dev *ch, int nchrom, const gd_css_planes *pl, const uint32_t *planes,
                 const int32_t *lo_a_, const int32_t *hi_a_, const int32_t *lo_b_, const double *avals,
                 const double *bvals, int64_t wtotal, int mds, int want_x, int force_literal, int xstride,
                 double *scores, double *pvals, double *xbuf, uint8_t *status, unsigned *flags, double *slab,
                 int64_t slab_per_wg, int mpb, int ld) {
  constexpr int NT = sm_nt<MP>(), NW = NT / 64, SR = (MP + NT - 1) / NT; /* SR individuals per thread */
  constexpr int NTRI = MP * (MP - 1) / 2;
  __shared__ uint16_t s_cnt_l[BIG ? 1 : MP * MP]; /* count D[i][j] at j*cs + i */
  __shared__ double s_tri_l[BIG ? 1 : NTRI];      /* stress terms, (i, j < i) at i(i-1)/2 + j */
  double *const s_tri = BIG ? slab + (int64_t)blockIdx.x * slab_per_wg : s_tri_l;
  uint16_t *const s_cnt =
      BIG ? reinterpret_cast<uint16_t *>(s_tri + (int64_t)mpb * (mpb - 1) / 2 + 8) : s_cnt_l;
  const int cs = BIG ? ld : MP; /* count column stride */
  __shared__ double s_z[2][2 * MP];   /* configurations, row-major m x 2 */
  __shared__ double s_best[2 * MP];
  __shared__ uint64_t s_mask[2 * MP];
  __shared__ double s_vals[MP];
  __shared__ double s_red[2 * NW];
  __shared__ double s_sig, s_f;
  __shared__ int s_irr;

  const int tid = threadIdx.x;
  for (int64_t w = blockIdx.x; w < wtotal; w += BIG ? (int64_t)gridDim.x : wtotal) {
  if (BIG) __syncthreads(); /* the previous window's readers are done */
  if (mds == 2 && !status[w]) continue; /* discarded in the classical stage */
  const int c = sm_chrom_of(ch, nchrom, w);
  const gd_chrom_dev &d = ch[c];
  const int a = d.asize, b = d.bsize, m = a + b;
  const int64_t wl = w - d.w_base;
  const int32_t la = lo_a_[w], ha = hi_a_[w], lb = lo_b_[w];
  const int npos = (ha - la) / a;
  if (npos <= 0) continue;
  if ((int64_t)lb + (int64_t)npos * b > d.blen) {
    if (tid == 0) atomicOr(flags, GD_FLAG_B_BOUNDS);
    continue;
  }
  if (m > MP || (FREQ && (a != 1 || b != 1)) || (!FREQ && npos > 65535)) {
    if (tid == 0) atomicOr(flags, GD_FLAG_BAD_SIZE);
    continue;
  }
  /* individual i = tid + rr NT of this thread, rr < SR */
#define SM_ROWS(i) \
  _Pragma("unroll") for (int rr_ = 0, i = tid; rr_ < SR; ++rr_, i += NT) if (i < m)

  /* ---- dissimilarities + fill_averages */
  double avg = 0.0, fdel = 0.0;
  if constexpr (FREQ) {
    if (tid == 0) {
      const double *av = avals + d.a_off + la, *bv = bvals + d.b_off + lb;
      double f = 0.0;
      for (int k = npos; k--;) f += sm_dabs(av[k] - bv[k]);
      s_f = f / npos;
    }
    __syncthreads();
    fdel = s_f;
    if (2 + (fdel < 0.00001 ? 2 : 0) > 2) continue;
  } else {
    const gd_css_planes P = pl[c];
    const uint32_t *pa = planes + P.pa, *pb = planes + P.pb;
    const int64_t ra = la / a, rb = lb / b;
    bool literal = force_literal || (la % a) != 0 || (lb % b) != 0;
    if (tid == 0) s_irr = 0;
    for (int e = tid; e < (BIG ? cs * m : MP * MP); e += NT) s_cnt[e] = 0;
    __syncthreads();
    if (!literal) {
      int irr = 0;
      for (int k = tid; k * 64 < npos; k += NT) {
        const int nb = min(64, npos - 64 * k);
        const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
        const uint64_t xa = sm_plane_bits64(pa + (int64_t)(2 * a) * P.wa, ra + 64 * k) & tail;
        const uint64_t xb = sm_plane_bits64(pb + (int64_t)(2 * b) * P.wb, rb + 64 * k) & tail;
        irr |= (xa | xb) != 0;
      }
      if (irr) s_irr = 1;
      __syncthreads();
      literal = s_irr != 0;
    }
    if (!literal) {
      for (int k = 0; k * 64 < npos; ++k) {
        const int nb = min(64, npos - 64 * k);
        const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
        __syncthreads();
        SM_ROWS(i) {
          const uint32_t *base = i < a ? pa + (int64_t)(2 * i) * P.wa : pb + (int64_t)(2 * (i - a)) * P.wb;
          const int64_t nw = i < a ? P.wa : P.wb;
          const int64_t r = (i < a ? ra : rb) + 64 * k;
          s_mask[2 * i] = sm_plane_bits64(base, r) & tail;
          s_mask[2 * i + 1] = sm_plane_bits64(base + nw, r) & tail;
        }
        __syncthreads();
        SM_ROWS(i) {
          const uint64_t Pi = s_mask[2 * i], Ni = s_mask[2 * i + 1];
          for (int j = 0; j < m; ++j) {
            const uint64_t Pj = s_mask[2 * j], Nj = s_mask[2 * j + 1];
            s_cnt[j * cs + i] = (uint16_t)(s_cnt[j * cs + i] + __popcll(Pi & Nj) + __popcll(Ni & Pj));
          }
        }
      }
    } else {
      const double *av = avals + d.a_off + la, *bv = bvals + d.b_off + lb;
      for (int k = 0; k < npos; ++k) {
        __syncthreads();
        SM_ROWS(i) s_vals[i] = i < a ? av[(int64_t)k * a + i] : bv[(int64_t)k * b + (i - a)];
        __syncthreads();
        SM_ROWS(i) {
          const double vi = s_vals[i];
          for (int j = 0; j < m; ++j) {
            if (j == i) continue; /* (int)v * v >= 0 never counts */
            const double vj = s_vals[j];
            /* the reference casts the row element of the larger index within a population
             * and the A element across populations (css.c:281-326) */
            const bool cast_i = ((i < a) == (j < a)) ? (i > j) : (i < a);
            const double prod = cast_i ? sm_x86_int(vi) * vj : sm_x86_int(vj) * vi;
            if (prod == -9.0) s_cnt[j * cs + i] = (uint16_t)(s_cnt[j * cs + i] + 1);
          }
        }
      }
    }
    __syncthreads();
    /* fill_averages (css.c:337-366): zero counts, the diagonal included, are unknown */
    double unv = 0.0, sum = 0.0;
    SM_ROWS(i) {
      for (int j = 0; j < m; ++j) {
        const int cj = s_cnt[j * cs + i];
        if (cj == 0)
          unv += 1.0;
        else
          sum += (double)cj;
      }
    }
    /* sums of integers: exact in any order */
    for (int o = 32; o > 0; o >>= 1) {
      unv += __shfl_xor(unv, o);
      sum += __shfl_xor(sum, o);
    }
    if ((tid & 63) == 0) {
      s_red[tid >> 6] = unv;
      s_red[NW + (tid >> 6)] = sum;
    }
    __syncthreads();
    unv = 0.0;
    sum = 0.0;
    for (int k = 0; k < NW; ++k) {
      unv += s_red[k];
      sum += s_red[NW + k];
    }
    const int tot = m * m;
    if ((int)unv > tot / 2) continue; /* discarded window: outputs untouched */
    avg = sum / tot;
  }
  /* delta(i, j), i != j */
  auto delta = [&](int i, int j) -> double {
    if constexpr (FREQ) {
      (void)i;
      (void)j;
      return fdel;
    } else {
      const int cij = s_cnt[j * cs + i];
      return cij == 0 ? avg : (double)cij;
    }
  };

  /* one pass over configuration cur: returns the stress of s_z[cur] and leaves its
   * Guttman transform in s_z[cur ^ 1] */
  auto pass = [&](int cur) -> double {
    const double *Z = s_z[cur];
    double *Xn = s_z[cur ^ 1];
    SM_ROWS(i) {
      const double zi0 = Z[2 * i], zi1 = Z[2 * i + 1];
      const int tb = i * (i - 1) / 2;
      double dsum = 0.0;
      for (int j = m - 1; j >= 0; --j) {
        if (j == i) continue;
        const double dij = sm_dist(zi0, zi1, Z[2 * j], Z[2 * j + 1]);
        const double del = delta(i, j);
        const double bij = dij < 0.00001 ? 0.0 : -1 * del / dij;
        dsum += bij;
        if (j < i) {
          const double e = dij - del;
          s_tri[tb + j] = e * e;
        }
      }
      double x0 = 0.0, x1 = 0.0;
      for (int k = 0; k < m; ++k) {
        double bik;
        if (k == i) {
          bik = -1 * dsum;
        } else {
          const double dik = sm_dist(zi0, zi1, Z[2 * k], Z[2 * k + 1]);
          bik = dik < 0.00001 ? 0.0 : -1 * delta(i, k) / dik;
        }
        if (bik != 0.0) {
          x0 = x0 + bik * Z[2 * k];
          x1 = x1 + bik * Z[2 * k + 1];
        }
      }
      Xn[2 * i] = x0 / m;
      Xn[2 * i + 1] = x1 / m;
    }
    __syncthreads();
    if (tid == 0) {
      double s = 0.0;
      for (int e = m * (m - 1) / 2; e--;) s += s_tri[e];
      s_sig = s;
    }
    __syncthreads();
    return s_sig;
  };

  /* smacof (css.c:855-938) from s_z[0]: returns the final stress, *fin = buffer of X */
  auto smacof = [&](int *fin) -> double {
    int cur = 0;
    double sigma = pass(cur), sprev;
    int k = 0;
    do {
      sprev = sigma;
      ++k;
      cur ^= 1;
      sigma = pass(cur);
    } while ((sprev - sigma) > SM_EPS && k <= SM_MAX_ITERS);
    *fin = cur;
    return sigma;
  };

  const double *Xf;
  if (mds == 2) {
    SM_ROWS(i) {
      s_z[0][2 * i] = xbuf[w * xstride + 2 * i];
      s_z[0][2 * i + 1] = xbuf[w * xstride + 2 * i + 1];
    }
    __syncthreads();
    int fin;
    smacof(&fin);
    Xf = s_z[fin];
  } else {
    /* smacof_runs (css.c:807-835) */
    const uint64_t x0 = gd_window_state(d.seed, GD_STREAM_SMACOF, wl + d.w_first);
    double best = SM_SIGMA0, fallback = 0.0;
    bool have = false;
    for (int r = 0; r < SM_NINIT; ++r) {
      __syncthreads();
      SM_ROWS(i) {
        const uint64_t k = (uint64_t)r * 2 * m + 2 * i; /* draws before this individual's two */
        s_z[0][2 * i] = sm_drand48_at(x0, k + 1);
        s_z[0][2 * i + 1] = sm_drand48_at(x0, k + 2);
      }
      __syncthreads();
      int fin;
      const double sigma = smacof(&fin);
      const bool take = sigma < best || (!have && (r == 0 || sigma < fallback));
      if (take) {
        SM_ROWS(i) {
          s_best[2 * i] = s_z[fin][2 * i];
          s_best[2 * i + 1] = s_z[fin][2 * i + 1];
        }
        if (sigma < best) {
          best = sigma;
          have = true;
        } else {
          fallback = sigma;
        }
      }
    }
    __syncthreads();
    Xf = s_best;
  }

  /* ---- calc_dist + css on the identity groups (serial, the reference's order) */
  if (tid == 0) s_sig = sm_css_serial(Xf, a, b);
  __syncthreads();
  const double score = s_sig;
  if (score == -1.0) { /* the reference's "discarded" marker (css.c:127) */
    if (tid == 0 && want_x) status[w] = 0;
    continue;
  }
  if (tid == 0) {
    scores[d.w_out + wl] = score;
    if (!want_x) pvals[d.w_out + wl] = 1.0;
  }
  if (want_x) {
    for (int e = tid; e < xstride; e += NT) xbuf[w * xstride + e] = (e < 2 * m) ? Xf[e] : 0.0;
    if (tid == 0) status[w] = 1;
  }
  }
}

#undef SM_ROWS

template <int MP, bool FREQ, bool BIG = false>
static int launch_smacof(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                         const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                         const double *bvals, int64_t wtotal, int mds, int want_x, int force_literal, int xstride,
                         double *scores, double *p, double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s,
                         double *slab = nullptr, int mpb = 0) {
  const int64_t grid = BIG ? gd_css_big_grid(wtotal, mpb) : wtotal;
  hipLaunchKernelGGL((k_css_smacof<MP, FREQ, BIG>), dim3((unsigned)grid), dim3(sm_nt<MP>()), 0, s, d_ch,
                     nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, mds, want_x, force_literal,
                     xstride, scores, p, xbuf, status, flags, slab, BIG ? gd_css_big_slab_per_wg(mpb) : 0, mpb,
                     BIG ? gd_css_big_ld(mpb) : 0);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

/* mds = 1 / 2 stage of a CSS scan; xbuf rows are 2 * mp doubles */
int gd_css_smacof_launch(int mp, bool freq, const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl,
                         const uint32_t *planes, const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b,
                         const double *avals, const double *bvals, int64_t wtotal, int mds, int want_x,
                         int force_literal, double *scores, double *p, double *xbuf, uint8_t *status,
                         unsigned *flags, double *slab, hipStream_t s) {
  const int xs = 2 * mp;
#define SM_CASE(T)                                                                                          \
  case T:                                                                                                   \
    return launch_smacof<T, false>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, mds, \
                                   want_x, force_literal, xs, scores, p, xbuf, status, flags, s);
  if (freq)
    return launch_smacof<24, true>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, mds, want_x,
                                   force_literal, xs, scores, p, xbuf, status, flags, s);
  switch (mp) {
    SM_CASE(24)
    SM_CASE(40)
    SM_CASE(64)
    SM_CASE(80)
    SM_CASE(96)
    SM_CASE(128)
    default:
      if (mp > GD_CSS_TIER_MAX && mp <= 256)
        return launch_smacof<256, false, true>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, mds,
                                               want_x, force_literal, xs, scores, p, xbuf, status, flags, s, slab, mp);
      if (mp > 256 && mp <= 512)
        return launch_smacof<512, false, true>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, mds,
                                               want_x, force_literal, xs, scores, p, xbuf, status, flags, s, slab, mp);
      if (mp > 512 && mp <= 1024)
        return launch_smacof<1024, false, true>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal,
                                                mds, want_x, force_literal, xs, scores, p, xbuf, status, flags, s, slab,
                                                mp);
      if (mp > 1024 && mp <= GD_CSS_SMACOF_MAX)
        return launch_smacof<2048, false, true>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal,
                                                mds, want_x, force_literal, xs, scores, p, xbuf, status, flags, s, slab,
                                                mp);
  }
#undef SM_CASE
  return GD_ERR_SIZE;
}

/* mds = 0 with the drosophila metric */
int gd_css_freq_cmds_launch(int mp, const gd_chrom_dev *d_ch, int nchrom, const int32_t *lo_a, const int32_t *hi_a,
                            const int32_t *lo_b, const double *avals, const double *bvals, int64_t wtotal,
                            int want_x, double *scores, double *p, double *xbuf, uint8_t *status, unsigned *flags,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_css_freq_cmds, dim3((unsigned)((wtotal + 255) / 256)), dim3(256), 0, s, d_ch, nchrom, lo_a,
                     hi_a, lo_b, avals, bvals, wtotal, want_x, 2 * mp, scores, p, xbuf, status, flags);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}
