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
 *   (the 80 tier: gd_css_t80.hip; the 25..40 tier: gd_css_h40.hip; the general path
 *   above 128 individuals: gd_css_big.hip; the permutation test, significance_treshold,
 *   is in gd_css_perm.hip; device helpers in gd_css_common.h)
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
#include "gd_css_common.h"


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
/* per-window classical MDS + CSS.  Matrix row i lives in the VGPRs of G lanes  */
/* (t = G*i + h holds columns [h*CP, (h+1)*CP), CP = MP/G): G = 1 up to 64      */
/* individuals, G = 2 above (half the registers per lane, 3x the occupancy).    */
/* Row-level values (row sums, x_i, p_i, v_i, w_i, y_i) are replicated in the G */
/* lanes of a row and counted once ("lead" lane) in block reductions.           */
/* ------------------------------------------------------------------------ */
template <int MP, int G>
struct CssShape {
  static constexpr int CP = MP / G;
  static constexpr int NT = 64 * ((MP * G + 63) / 64);
  static constexpr int NW = NT / 64;
};

/* sum over the G lanes of a row (adjacent lanes) */
template <int G>
__device__ __forceinline__ double pair_sum(double x) {
  if constexpr (G == 1)
    return x;
  else
    return x + dpp64<0xB1, 0xF>(x, 0.0); /* quad_perm [1,0,3,2]: the partner lane */
}

/* One Householder step with the column index K known at compile time (single-wave
 * tiers up to 40 individuals): block skipping, the dead-column stash and the reads
 * of x, d_K and A e_{K+1} all resolve to fixed registers -- no per-column selects. */
template <int MP, int K>
__device__ __forceinline__ void hh_step_static(double (&A)[MP], int m, double *s_row, double *s_v, double *s_w,
                                               double *s_d, double *s_e, double *s_tau) {
  const int i = css_lane_now(), tid = i, ii = i < MP ? i : MP - 1; /* one wave: row = lane */
  const bool row = i < m;
  __syncthreads();
  if (i == K) {
#pragma unroll
    for (int jb = 0; jb < MP / 8; ++jb)
      if (8 * jb + 7 >= K) {
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
          const int j = 8 * jb + u;
          *reinterpret_cast<double2 *>(s_row + j) = make_double2(j > K ? A[j] : 0.0, j + 1 > K ? A[j + 1] : 0.0);
        }
      }
    s_d[K] = A[K];
  }
  __syncthreads();
  if constexpr (K >= MP - 2) {
    if (tid == 0 && K == m - 2) s_e[K] = s_row[K + 1];
    return;
  }
  /* K >= m - 2 (below MP - 2) runs the general step on the zero padding: x = 0, so
   * sigma = 0, tau = 0, beta = alpha (= e_{m-2} at K = m - 2) and the update adds
   * exact zeros -- the same values as an early exit, without a join point per step
   * (each one cost a block of register moves) */
  const double xi = (i > K + 1 && row) ? s_row[ii] : 0.0;
  const double alpha = s_row[K + 1];
  double p0 = 0, p1 = 0;
#pragma unroll
  for (int jb = 0; jb < MP / 8; ++jb) {
    if (8 * jb + 7 > K) {
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        if (8 * jb + u > K) p0 = fma(A[8 * jb + u], s_row[8 * jb + u], p0);
        if (8 * jb + u + 1 > K) p1 = fma(A[8 * jb + u + 1], s_row[8 * jb + u + 1], p1);
      }
      CSS_PIN(p0);
      CSS_PIN(p1);
    }
  }
  const double ak1 = A[K + 1 < MP ? K + 1 : K]; /* K >= MP - 2 returned above */
  const double praw = p0 + p1;
  /* one reduction for |x|^2 and q = r^T A r (r: row K right of the diagonal, r_{K+1} =
   * alpha): with v = scale (r - beta e_{K+1}), v^T p = tau scale^2 (q - 2 beta (A r)_{K+1}
   * + beta^2 A_{K+1,K+1}), so no second reduction waits on beta */
  double sigma = xi * xi, q = ((i > K && row) ? s_row[ii] : 0.0) * praw;
  wave_sum2(sigma, q);
  const double pr1 = readlane_f64(praw, K + 1), a11 = readlane_f64(ak1, K + 1);
  double tau = 0.0, beta = alpha, scale = 0.0;
  if (sigma != 0.0) {
    beta = -copysign(sqrt_pos(alpha * alpha + sigma), alpha);
    const double r = fast_rcp(beta * (alpha - beta)); /* 1/beta and 1/(alpha - beta) from one reciprocal */
    tau = -(alpha - beta) * (alpha - beta) * r;
    scale = beta * r;
  }
  const double vi = (i == K + 1) ? 1.0 : xi * scale;
  const double pi = (i > K && row) ? (tau * scale) * fma(-beta, ak1, praw) : 0.0;
  const double Kc = -0.5 * tau * (tau * scale * scale) * fma(beta, fma(beta, a11, -2.0 * pr1), q);
  const double wi = fma(Kc, vi, pi);
  if (tid == 0) {
    s_e[K] = beta;
    s_tau[K] = tau;
  }
  if (i < MP) {
    s_v[i] = vi;
    s_w[i] = wi;
  }
  __syncthreads();
#pragma unroll
  for (int jb = 0; jb < MP / 8; ++jb) {
    if (8 * jb + 7 > K) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = 8 * jb + u;
        if (j > K) A[j] = fma(-vi, s_w[j], fma(-wi, s_v[j], A[j]));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) CSS_PIN(A[8 * jb + u]);
    }
  }
  A[K] = vi; /* stash v_K in the dead column K */
}

template <int MP, int K>
struct HhStatic {
  static __device__ __forceinline__ void run(double (&A)[MP], int m, double *s_row, double *s_v, double *s_w,
                                             double *s_d, double *s_e, double *s_tau) {
    if ((K & 7) == 0 && K >= m) return; /* exits only at block boundaries (see above) */
    hh_step_static<MP, K>(A, m, s_row, s_v, s_w, s_d, s_e, s_tau);
    HhStatic<MP, K + 1>::run(A, m, s_row, s_v, s_w, s_d, s_e, s_tau);
  }
};
template <int MP>
struct HhStatic<MP, MP> {
  static __device__ __forceinline__ void run(double (&)[MP], int, double *, double *, double *, double *, double *,
                                             double *) {}
};

/* The compile-time-K step for the two-lanes-per-row tiers (G = 2): lane part h holds
 * columns [h*CP, (h+1)*CP).  Block skipping is uniform over both parts (a block is
 * skipped when it is dead in part 1), column K+1 and the dead column K sit at fixed
 * registers of a fixed part, so reading A e_{K+1} and stashing v_K cost one select
 * each instead of one per column. */
template <int MP, int G, int K, int PART>
__device__ __forceinline__ void hh_publish_part(const double (&A)[MP / G], double *s_row, double *s_d) {
  constexpr int CP = MP / G, C0 = PART * CP;
#pragma unroll
  for (int jb = 0; jb < CP / 8; ++jb)
    if ((G - 1) * CP + 8 * jb + 7 > K - 1) {
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        const int j = C0 + 8 * jb + u;
        *reinterpret_cast<double2 *>(s_row + j) =
            make_double2(j > K ? A[8 * jb + u] : 0.0, j + 1 > K ? A[8 * jb + u + 1] : 0.0);
      }
    }
  if constexpr (K >= C0 && K < C0 + CP) s_d[K] = A[K - C0];
}

template <int MP, int G, int K>
__device__ __forceinline__ void hh_step_static_g(double (&A)[MP / G], int m, int wave, double *s_row, double *s_v,
                                                 double *s_w, double *s_d, double *s_e, double *s_tau,
                                                 double *s_red) {
  constexpr int CP = MP / G, NW = CssShape<MP, G>::NW;
  const int lane = css_lane_now(), tid = wave * 64 + lane;
  const int i = tid / G, h = tid % G, ii = i < MP ? i : MP - 1;
  const bool row = i < m, lead = h == 0;
  const int c0 = h * CP;
  /* No barrier ahead of the publish: every read of s_row by step K-1 happened before
   * its v/w barrier, which every wave has passed by now.  The reduction slots alternate
   * between two banks by step parity, so their writes need no barrier of their own.
   * (Step MP-2 reads s_row after its publish without a later barrier: step MP-1 keeps it.) */
  if constexpr (K == 0 || K == MP - 1) __syncthreads();
  double *red = s_red + (K & 1) * (2 * NW + 2);
  if (i == K) {
    if constexpr (G == 1)
      hh_publish_part<MP, G, K, 0>(A, s_row, s_d);
    else if (h == 0)
      hh_publish_part<MP, G, K, 0>(A, s_row, s_d);
    else
      hh_publish_part<MP, G, K, 1>(A, s_row, s_d);
  }
  __syncthreads();
  if constexpr (K >= MP - 2) {
    if (tid == 0 && K == m - 2) s_e[K] = s_row[K + 1];
    return;
  } else {
    /* K >= m - 2 below MP - 2: a no-op reflector on the zero padding (hh_step_static) */
    const double xi = (i > K + 1 && row) ? s_row[ii] : 0.0;
    const double alpha = s_row[K + 1];
    double p0 = 0, p1 = 0;
#pragma unroll
    for (int jb = 0; jb < CP / 8; ++jb) {
      if ((G - 1) * CP + 8 * jb + 7 > K) {
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
          p0 = fma(A[8 * jb + u], s_row[c0 + 8 * jb + u], p0);
          p1 = fma(A[8 * jb + u + 1], s_row[c0 + 8 * jb + u + 1], p1);
        }
        CSS_PIN(p0);
        CSS_PIN(p1);
      }
    }
    constexpr int HK1 = (K + 1) / CP, LK1 = K + 1 - HK1 * CP;
    const double ak1 = pair_sum<G>(h == HK1 ? A[LK1] : 0.0);
    const double praw = pair_sum<G>(p0 + p1);
    /* one reduction for |x|^2 and r^T A r (hh_step_static); (A r)_{K+1} and A_{K+1,K+1}
     * travel from row K+1 through the two LDS slots behind the reduction's */
    static_assert(NW > 1, "block_sum2 synchronises the slots only across waves");
    double sigma = lead ? xi * xi : 0.0, q = (lead && i > K && row) ? s_row[ii] * praw : 0.0;
    if (lead && i == K + 1) {
      red[2 * NW] = praw;
      red[2 * NW + 1] = ak1;
    }
    wave_sum2(sigma, q);
    if (lane == 0) {
      red[wave] = sigma;
      red[NW + wave] = q;
    }
    __syncthreads();
    sigma = red[0];
    q = red[NW];
#pragma unroll
    for (int k = 1; k < NW; ++k) {
      sigma += red[k];
      q += red[NW + k];
    }
    const double pr1 = red[2 * NW], a11 = red[2 * NW + 1];
    double tau = 0.0, beta = alpha, scale = 0.0;
    if (sigma != 0.0) {
      beta = -copysign(sqrt_pos(alpha * alpha + sigma), alpha);
      const double r = fast_rcp(beta * (alpha - beta));
      tau = -(alpha - beta) * (alpha - beta) * r;
      scale = beta * r;
    }
    const double vi = (i == K + 1) ? 1.0 : xi * scale;
    const double pi = (i > K && row) ? (tau * scale) * fma(-beta, ak1, praw) : 0.0;
    const double Kc = -0.5 * tau * (tau * scale * scale) * fma(beta, fma(beta, a11, -2.0 * pr1), q);
    const double wi = fma(Kc, vi, pi);
    if (tid == 0) {
      s_e[K] = beta;
      s_tau[K] = tau;
    }
    if (lead && i < MP) {
      s_v[i] = vi;
      s_w[i] = wi;
    }
    __syncthreads();
#pragma unroll
    for (int jb = 0; jb < CP / 8; ++jb) {
      if ((G - 1) * CP + 8 * jb + 7 > K) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = c0 + 8 * jb + u;
          A[8 * jb + u] = fma(-vi, s_w[j], fma(-wi, s_v[j], A[8 * jb + u]));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) CSS_PIN(A[8 * jb + u]);
      }
    }
    constexpr int HK = K / CP, LK = K - HK * CP;
    if (h == HK) A[LK] = vi; /* stash v_K in the dead column K */
  }
}

template <int MP, int G, int K>
struct HhStaticG {
  static __device__ __forceinline__ void run(double (&A)[MP / G], int m, int wave, double *s_row, double *s_v,
                                             double *s_w, double *s_d, double *s_e, double *s_tau, double *s_red) {
    if ((K & 7) == 0 && K >= m) return;
    hh_step_static_g<MP, G, K>(A, m, wave, s_row, s_v, s_w, s_d, s_e, s_tau, s_red);
    HhStaticG<MP, G, K + 1>::run(A, m, wave, s_row, s_v, s_w, s_d, s_e, s_tau, s_red);
  }
};
template <int MP, int G>
struct HhStaticG<MP, G, MP> {
  static __device__ __forceinline__ void run(double (&)[MP / G], int, int, double *, double *, double *, double *,
                                             double *, double *, double *) {}
};

template <int MP, int G>
__global__ void __launch_bounds__((CssShape<MP, G>::NT), CSS_MDS_WAVES(MP, G))
    k_css_mds(const gd_chrom_dev *ch, int nchrom, const gd_css_planes *pl, const uint32_t *planes,
              const int32_t *lo_a_, const int32_t *hi_a_, const int32_t *lo_b_, const double *avals,
              const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *pvals,
              double *xbuf, uint8_t *status, unsigned *flags) {
  constexpr int CP = CssShape<MP, G>::CP, NT = CssShape<MP, G>::NT, NW = CssShape<MP, G>::NW;
  __shared__ double s_row[MP + 2];
  __shared__ double s_v[MP], s_w[MP];
  __shared__ __attribute__((aligned(16))) double s_d[MP + 4];
  __shared__ __attribute__((aligned(16))) double s_e2[MP + 4];
  __shared__ double s_e[MP], s_tau[MP];
  __shared__ uint64_t s_mask[2 * MP];
  __shared__ double s_vals[MP];
  __shared__ double s_y[2][MP];
  __shared__ double s_lu[2][3][MP];
  __shared__ uint8_t s_piv[2][MP];
  __shared__ double s_x[2 * MP];
  __shared__ int s_tr[MP];
  __shared__ double s_lam[2];
  __shared__ double s_red[2 * (2 * NW + 2)]; /* block sums; [2NW], [2NW+1]: row K+1 in a Householder step
                                                (two banks, alternating by step in the G = 2 steps) */

  const int tid = threadIdx.x;
  const int i = tid / G, h = tid % G; /* row, column part */
  const int c0 = h * CP;              /* first column held by this lane */
  const bool lead = h == 0;
  const int ii = i < MP ? i : MP - 1; /* clamped LDS index for lanes past MP */
  if (tid < MP) s_tr[tid] = tid;

  /* one workgroup per window (no persistent loop: hoisting per-lane invariants out of
   * a window loop costs ~100 VGPRs and halves the occupancy) */
  for (int64_t w = blockIdx.x; w < wtotal; w += wtotal) {
    CSS_PROF_INIT;
    const int c = chrom_of(ch, nchrom, w);
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
    if (m > MP) {
      if (tid == 0) atomicOr(flags, GD_FLAG_BAD_SIZE);
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
      for (int k = tid; k * 64 < npos; k += NT) {
        const int nb = min(64, npos - 64 * k);
        const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
        const uint64_t xa = plane_bits64(pa + (int64_t)(2 * a) * P.wa, ra + 64 * k) & tail;
        const uint64_t xb = plane_bits64(pb + (int64_t)(2 * b) * P.wb, rb + 64 * k) & tail;
        irr |= (xa | xb) != 0;
      }
      literal = __syncthreads_or(irr);
    }

    /* ---- compare_all: D[i][c0 + jj] in registers */
    double A[CP];
    {
      int acc[CP];
#pragma unroll
      for (int jj = 0; jj < CP; ++jj) acc[jj] = 0;
      if (!literal) {
        for (int k = 0; k * 64 < npos; ++k) {
          const int nb = min(64, npos - 64 * k);
          const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
          __syncthreads();
          if (lead && row) {
            const uint32_t *base = i < a ? pa + (int64_t)(2 * i) * P.wa : pb + (int64_t)(2 * (i - a)) * P.wb;
            const int64_t nw = i < a ? P.wa : P.wb;
            const int64_t r = (i < a ? ra : rb) + 64 * k;
            s_mask[2 * i] = plane_bits64(base, r) & tail;
            s_mask[2 * i + 1] = plane_bits64(base + nw, r) & tail;
          } else if (lead && i < MP) {
            s_mask[2 * i] = 0;
            s_mask[2 * i + 1] = 0;
          }
          __syncthreads();
          const uint64_t Pi = s_mask[2 * ii], Ni = s_mask[2 * ii + 1];
#pragma unroll
          for (int jj = 0; jj < CP; ++jj) {
            const int j = c0 + jj;
            const uint64_t Pj = s_mask[2 * j], Nj = s_mask[2 * j + 1];
            acc[jj] += __popcll(Pi & Nj) + __popcll(Ni & Pj);
            if ((jj & 7) == 7) {
#pragma unroll
              for (int u = jj - 7; u <= jj; ++u) CSS_PIN(acc[u]);
            }
          }
        }
      } else {
        const double *av = avals + d.a_off + la, *bv = bvals + d.b_off + lb;
        for (int k = 0; k < npos; ++k) {
          __syncthreads();
          if (lead && row) s_vals[i] = i < a ? av[(int64_t)k * a + i] : bv[(int64_t)k * b + (i - a)];
          __syncthreads();
          const double vi = s_vals[ii];
          int io = i, mo = m, ao = a, co = c0;
          CSS_OPAQUE_V(io);
          CSS_OPAQUE_V(co);
          CSS_OPAQUE_S(mo);
          CSS_OPAQUE_S(ao);
#pragma unroll
          for (int jj = 0; jj < CP; ++jj) {
            const int j = co + jj;
            /* the diagonal never counts: (int)v * v >= 0 */
            if (j < mo) {
              const double vj = s_vals[j];
              /* the reference casts the row element of the larger index within a
               * population and the A element across populations (css.c:281-326) */
              const bool cast_i = ((io < ao) == (j < ao)) ? (io > j) : (io < ao);
              const double prod = cast_i ? x86_int(vi) * vj : x86_int(vj) * vi;
              acc[jj] += prod == -9.0;
            }
          }
        }
      }
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int jj = 0; jj < CP; ++jj) A[jj] = (row && c0 + jj < mo) ? (double)acc[jj] : 0.0;
    }

    CSS_PROF(0);
    /* ---- fill_averages: entries < 1e-5 (diagonal included) count as unknown */
    {
      int unval = 0;
      double sum = 0;
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int jj = 0; jj < CP; ++jj) {
        if (row && c0 + jj < mo) {
          if (A[jj] < 0.00001)
            ++unval;
          else
            sum += A[jj];
        }
      }
      double unv = (double)unval;
      block_sum2<NW>(unv, sum, s_red); /* sums of integers: exact in any order */
      unval = (int)unv;
      const int tot = m * m;
      if (unval > tot / 2) continue; /* discarded window: outputs untouched */
      const double avg = sum / tot;
      /* D holds non-negative integer counts, so "< 1e-5" is "== 0" and the fill is
       * A + avg (1 - min(A, 1)), exact and mask-free (no per-column compare results
       * kept alive across the reduction); padding columns are re-zeroed below */
      CSS_OPAQUE_ROW(A);
#pragma unroll
      for (int jj = 0; jj < CP; ++jj) A[jj] = fma(avg, 1.0 - fmin(A[jj], 1.0), A[jj]);
    }

    /* ---- B = -1/2 Z (D o D) Z, Z = I - 11^T/m, by double centering */
    double zero_tol;
    {
      double rs = 0;
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int jj = 0; jj < CP; ++jj) {
        A[jj] = (row && c0 + jj < mo) ? A[jj] * A[jj] : 0.0;
        rs += A[jj];
      }
      rs = pair_sum<G>(rs);
      const double ri = row ? rs / m : 0.0;
      __syncthreads();
      if (lead && i < MP) s_v[i] = ri;
      const double g = block_sum<NW>(lead ? ri : 0.0, s_red) / m;
      __syncthreads();
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int jj = 0; jj < CP; ++jj) {
        A[jj] = (row && c0 + jj < mo) ? -0.5 * ((A[jj] - (ri + s_v[c0 + jj])) + g) : 0.0;
        if ((jj & 7) == 7) {
#pragma unroll
          for (int u = jj - 7; u <= jj; ++u) CSS_PIN(A[u]);
        }
      }
      double f2 = 0;
#pragma unroll
      for (int jj = 0; jj < CP; ++jj) f2 = fma(A[jj], A[jj], f2);
      /* eigenvalues within rounding of 0 count as 0 (oracle/css_oracle.c, cmds) */
      zero_tol = 64.0 * m * DBL_EPSILON * sqrt(block_sum<NW>(f2, s_red));
    }

    CSS_PROF(1);
    /* ---- Householder tridiagonalisation (LAPACK dsytd2, lower).  Column k of the
     * trailing matrix is read from row k (symmetry); after step k the dead column k
     * of each row holds that row's element of the reflector v_k.  Columns are
     * handled in blocks of 8; a block dead in every column part (v, w and x are 0
     * left of k) is skipped by a uniform branch. */
    if constexpr (G == 1 && MP <= CSS_STATIC_G1_MAX) {
#ifndef GD_CSS_SKIP_TRIDIAG
      HhStatic<MP, 0>::run(A, m, s_row, s_v, s_w, s_d, s_e, s_tau);
#endif
    } else if constexpr ((G == 2 || MP > 64) && MP <= CSS_STATIC_G2_MAX) {
      HhStaticG<MP, G, 0>::run(A, m, __builtin_amdgcn_readfirstlane(tid >> 6), s_row, s_v, s_w, s_d, s_e, s_tau,
                               s_red);
    } else
    for (int k = 0; k < m; ++k) {
      __syncthreads();
      /* row k's lanes publish x = row k right of the diagonal (zeros at j <= k) and d_k */
      if (i == k) {
#pragma unroll
        for (int jb = 0; jb < CP / 8; ++jb)
          if ((G - 1) * CP + 8 * jb + 7 >= k) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int j = c0 + 8 * jb + u;
              s_row[j] = j > k ? A[8 * jb + u] : 0.0;
              if (j == k) s_d[k] = A[8 * jb + u];
            }
          }
      }
      __syncthreads();
      if (k >= m - 2) {
        if (tid == 0 && k == m - 2) s_e[k] = s_row[k + 1];
        continue;
      }
      const double xi = (i > k + 1 && row) ? s_row[ii] : 0.0;
      const double alpha = s_row[k + 1];
      /* A x and A e_{k+1} need only x, so they overlap the norm reduction */
      const int lk1 = k + 1 - c0; /* column k+1 in this lane's part, if there */
      double p0 = 0, p1 = 0, ak1 = 0;
#pragma unroll
      for (int jb = 0; jb < CP / 8; ++jb) {
        if ((G - 1) * CP + 8 * jb + 7 > k) {
#pragma unroll
          for (int u = 0; u < 8; u += 2) {
            p0 = fma(A[8 * jb + u], s_row[c0 + 8 * jb + u], p0);
            p1 = fma(A[8 * jb + u + 1], s_row[c0 + 8 * jb + u + 1], p1);
          }
          CSS_PIN(p0);
          CSS_PIN(p1);
        }
        if ((lk1 >> 3) == jb) {
#pragma unroll
          for (int u = 0; u < 8; ++u) ak1 = (8 * jb + u == lk1) ? A[8 * jb + u] : ak1;
        }
      }
      const double praw = pair_sum<G>(p0 + p1);
      ak1 = pair_sum<G>(ak1);
      /* |x|^2 and r^T A r in one reduction (hh_step_static) */
      double sigma = lead ? xi * xi : 0.0, q = (lead && i > k && row) ? s_row[ii] * praw : 0.0;
      double pr1, a11;
      if constexpr (NW == 1) {
        static_assert(G == 1, "one wave holds whole rows");
        wave_sum2(sigma, q);
        pr1 = readlane_f64(praw, k + 1);
        a11 = readlane_f64(ak1, k + 1);
      } else {
        if (lead && i == k + 1) {
          s_red[2 * NW] = praw;
          s_red[2 * NW + 1] = ak1;
        }
        block_sum2<NW>(sigma, q, s_red);
        pr1 = s_red[2 * NW];
        a11 = s_red[2 * NW + 1];
      }
      double tau = 0.0, beta = alpha, scale = 0.0;
      if (sigma != 0.0) {
        beta = -copysign(sqrt_pos(alpha * alpha + sigma), alpha);
        const double r = fast_rcp(beta * (alpha - beta));
        tau = -(alpha - beta) * (alpha - beta) * r;
        scale = beta * r;
      }
      /* v = scale (x - beta e_{k+1}), v_{k+1} = 1;  p = tau A v */
      const double vi = (i == k + 1) ? 1.0 : xi * scale;
      const double pi = (i > k && row) ? (tau * scale) * fma(-beta, ak1, praw) : 0.0;
      const double K = -0.5 * tau * (tau * scale * scale) * fma(beta, fma(beta, a11, -2.0 * pr1), q);
      const double wi = fma(K, vi, pi);
      if (tid == 0) {
        s_e[k] = beta;
        s_tau[k] = tau;
      }
      if (lead && i < MP) {
        s_v[i] = vi;
        s_w[i] = wi;
      }
      __syncthreads();
      const int lk = k - c0; /* the dead column k in this lane's part, if there */
#pragma unroll
      for (int jb = 0; jb < CP / 8; ++jb) {
        if ((G - 1) * CP + 8 * jb + 7 > k) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int j = c0 + 8 * jb + u;
            A[8 * jb + u] = fma(-vi, s_w[j], fma(-wi, s_v[j], A[8 * jb + u]));
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) CSS_PIN(A[8 * jb + u]);
        }
        /* stash v_k in the dead column k */
        if ((lk >> 3) == jb) {
#pragma unroll
          for (int u = 0; u < 8; ++u) A[8 * jb + u] = (8 * jb + u == lk) ? vi : A[8 * jb + u];
        }
      }
    }
    __syncthreads();

    CSS_PROF(2);
    /* ---- the two largest eigenvalues of T: Gershgorin bounds, then 33-section
     * bisection, one half-wave per eigenvalue.  Sturm counts come from the sign
     * changes of the leading principal minors p_k(x) (three-term recurrence,
     * rescaled every 4 steps): no division on the serial chain. */
    double glo, ghi;
    {
      double lo = DBL_MAX, hi = -DBL_MAX;
      if (lead && row) {
        const double r = (i > 0 ? fabs(s_e[i - 1]) : 0.0) + (i < m - 1 ? fabs(s_e[i]) : 0.0);
        lo = s_d[i] - r;
        hi = s_d[i] + r;
      }
      if (tid < MP + 4) {
        /* Sturm arrays: s_e2[k] = e_{k-1}^2 (s_e2[0] = 0); entries m..m4 are a
         * decoupled tail far above the spectrum (no sign changes) */
        s_e2[tid] = (tid >= 1 && tid < m) ? s_e[tid - 1] * s_e[tid - 1] : 0.0;
      }
      glo = block_reduce<NW, OpMin>(lo, s_red);
      ghi = block_reduce<NW, OpMax>(hi, s_red);
      const double pad = 2.0 * DBL_EPSILON * fmax(fabs(glo), fabs(ghi)) * m + DBL_MIN;
      glo -= pad;
      ghi += pad;
      if (tid >= m && tid < MP + 4) s_d[tid] = 2.0 * fabs(ghi) + 2.0 * fabs(glo) + 1.0;
    }
    const double bis_tol = CSS_BISECT_TOL * fmax(fabs(glo), fabs(ghi)) + DBL_MIN;
    __syncthreads();
    if (tid < 64) bisect_top2(m, glo, ghi, bis_tol, s_d, s_e2, s_lam, tid);
    __syncthreads();

    CSS_PROF(3);
    /* ---- eigenvectors of T: two steps of inverse iteration with a partial-pivot
     * LU of T - lam I (thread 0: largest, thread 1: second).  The serial chains carry
     * their running values in registers; LDS holds only read-once factors. */
    if (tid < 2) invit_factor<MP>(m, tid, s_d, s_e, s_lam, s_lu, s_x, s_piv, s_y);
    __syncthreads();
    if (tid < m) {
      /* reciprocal pivots, in parallel (zero pivots -> tiny) */
      const double tiny = DBL_EPSILON * fmax(fmax(fabs(glo), fabs(ghi)), DBL_MIN);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double u0 = s_lu[e][0][tid];
        s_lu[e][0][tid] = fast_rcp(u0 == 0.0 ? tiny : u0);
      }
    }
    double y1 = 0.0, y2 = 0.0;
#ifdef GD_CSS_SKIP_INVIT
    for (int itn = 0; itn < 0; ++itn) {
#else
    for (int itn = 0; itn < 2; ++itn) {
#endif
      __syncthreads();
      if (tid < 2) invit_solve<MP>(m, tid, s_lu, s_x, s_piv, s_y);
      __syncthreads();
      y1 = row ? s_y[0][ii] : 0.0;
      y2 = row ? s_y[1][ii] : 0.0;
      double n1 = lead ? y1 * y1 : 0.0, n2 = lead ? y2 * y2 : 0.0;
      block_sum2<NW>(n1, n2, s_red);
      y1 *= 1.0 / sqrt(n1);
      y2 *= 1.0 / sqrt(n2);
      __syncthreads();
      if (itn == 0 && lead && row) {
        s_y[0][i] = y1;
        s_y[1][i] = y2;
      }
    }
    /* orthogonalise the second vector against the first (close eigenvalues) */
    {
      double dt = lead ? y1 * y2 : 0.0, zero = 0.0;
      block_sum2<NW>(dt, zero, s_red);
      y2 = fma(-dt, y1, y2);
      double n2 = lead ? y2 * y2 : 0.0;
      zero = 0.0;
      block_sum2<NW>(n2, zero, s_red);
      y2 *= 1.0 / sqrt(n2);
    }
    /* eigenvalues = Rayleigh quotients y^T T y of the unit vectors (error ~ the
     * squared eigenvector error, far below rounding) */
    {
      __syncthreads();
      if (lead && row) {
        s_y[0][i] = y1;
        s_y[1][i] = y2;
      }
      __syncthreads();
      double t1 = 0.0, t2 = 0.0;
      if (lead && row) {
        const double el = i > 0 ? s_e[i - 1] : 0.0, er = i + 1 < m ? s_e[i] : 0.0;
        const int il = i > 0 ? i - 1 : 0, ir = i + 1 < m ? i + 1 : i;
        t1 = y1 * (s_d[i] * y1 + el * s_y[0][il] + er * s_y[0][ir]);
        t2 = y2 * (s_d[i] * y2 + el * s_y[1][il] + er * s_y[1][ir]);
      }
      block_sum2<NW>(t1, t2, s_red);
      if (tid == 0) {
        s_lam[0] = fabs(t1) <= zero_tol ? 0.0 : t1;
        s_lam[1] = fabs(t2) <= zero_tol ? 0.0 : t2;
      }
      __syncthreads();
    }

    CSS_PROF(4);
    /* ---- back-transformation y <- H_0 H_1 ... H_{m-3} y; v_k sits in column k,
     * i.e. in part k / CP of the row */
#pragma unroll
#ifdef GD_CSS_SKIP_BACK
    for (int k = -1; k >= 0; --k) {
#else
    for (int k = MP - 3; k >= 0; --k) {
#endif
      if (k <= m - 3) {
        constexpr int dummy = 0;
        (void)dummy;
        const int hk = k / CP, lk = k - hk * CP;
        const double vk = pair_sum<G>((row && h == hk) ? A[lk] : 0.0);
        const double t = s_tau[k];
        double d1 = lead ? vk * y1 : 0.0, d2 = lead ? vk * y2 : 0.0;
        block_sum2<NW>(d1, d2, s_red);
        y1 = fma(-(t * d1), vk, y1);
        y2 = fma(-(t * d2), vk, y2);
        asm volatile("" ::: "memory"); /* one s_tau load in flight, not MP */
      }
    }

    CSS_PROF(5);
    /* ---- X = Q sqrt(L) (css.c:545-556), then calc_dist + css on identity groups */
    {
      const double L1 = sqrt(s_lam[0]), L2 = sqrt(s_lam[1]);
      __syncthreads();
      if (lead && row) {
        s_x[2 * i] = y1 * L1 + y2 * 0.0;
        s_x[2 * i + 1] = y1 * 0.0 + y2 * L2;
      }
      __syncthreads();
    }
    const double score = css_score<NW>(s_tr, a, b, [&](int p, int q) { return xdist(s_x, p, q); }, s_red);
    CSS_PROF(6);
    if (score == -1.0) continue; /* the reference's "discarded" marker (css.c:127) */
    if (tid == 0) {
      scores[d.w_out + wl] = score;
      if (!want_x) pvals[d.w_out + wl] = 1.0; /* runs == 0: p = (0 + 1) / (0 + 1) */
    }
    if (want_x) {
      for (int e = tid; e < 2 * MP; e += NT) xbuf[w * 2 * MP + e] = (e < 2 * m) ? s_x[e] : 0.0;
      if (tid == 0) status[w] = 1;
    }
  }
}

/* the other stages of a scan (gd_css_perm.hip, gd_css_smacof.hip, gd_packed.hip) */
int gd_packed_css_planes_launch(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl,
                                const int64_t *word_off, const uint64_t *acodes, const uint64_t *bcodes,
                                int64_t max_rows_words, uint32_t *planes, hipStream_t s);
int gd_css_perm_launch(int mp, const gd_chrom_dev *d_ch, int nchrom, const double *xbuf, const uint8_t *status,
                       int64_t wtotal, int treshold, int runs, double *p, unsigned *wq, double *slab, hipStream_t s);
int gd_css_smacof_launch(int mp, bool freq, const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl,
                         const uint32_t *planes, const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b,
                         const double *avals, const double *bvals, int64_t wtotal, int mds, int want_x,
                         int force_literal, double *scores, double *p, double *xbuf, uint8_t *status,
                         unsigned *flags, double *slab, hipStream_t s);
int gd_css_freq_cmds_launch(int mp, const gd_chrom_dev *d_ch, int nchrom, const int32_t *lo_a, const int32_t *hi_a,
                            const int32_t *lo_b, const double *avals, const double *bvals, int64_t wtotal,
                            int want_x, double *scores, double *p, double *xbuf, uint8_t *status, unsigned *flags,
                            hipStream_t s);

/* the MDS tiers in their own translation units (gd_css_t80.hip, gd_css_h40.hip, gd_css_big.hip) */
int gd_css_launch_t80(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s);
int gd_css_launch_p40(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s);
int gd_css_launch_big(int mp, const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, double *slab, hipStream_t s);

/* ------------------------------------------------------------------------ */
int gd_css_tier(int m) {
  static const int tiers[] = {24, 40, 64, 80, 96, 128};
  for (int t : tiers)
    if (m <= t) return t;
  /* the general path: any tier value above GD_CSS_TIER_MAX, the xbuf row width / 2 */
  if (m <= GD_CSS_BIG_MAX) return (m + 7) & ~7;
  return 0;
}

template <int MP, int G>
static int launch_tier(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                       const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                       const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                       double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s) {
  constexpr int NT = CssShape<MP, G>::NT;
  CSS_PROF_LAUNCH(s);
  hipLaunchKernelGGL((k_css_mds<MP, G>), dim3((unsigned)wtotal), dim3(NT), 0, s, d_ch, nchrom, d_pl, planes, lo_a,
                     hi_a, lo_b, avals, bvals, wtotal, want_x, force_literal, scores, p, xbuf, status, flags);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

/* One CSS scan after the window bounds: bit planes, the scores of the chosen metric
 * and MDS (cluster_separation_scorer, css.c:181-223), the permutation test.
 *   mds 0: k_css_mds (count metric) or k_css_freq_cmds (drosophila)
 *   mds 1: k_css_smacof from drand48 starts
 *   mds 2: the classical stage, then k_css_smacof from its coordinates (xbuf)
 * xbuf/status carry the coordinates between stages when runs > 0 or mds == 2. */
/* acodes != NULL: a packed batch; its bit planes come from the codes (never irregular,
 * rows always aligned, so the literal per-SNP path and the raw values are never read) */
int gd_css_launch(int mp, int drosophila, int mds, const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl,
                  uint32_t *planes, const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b,
                  const double *avals, const double *bvals, const int64_t *word_off, const uint64_t *acodes,
                  const uint64_t *bcodes, int64_t wtotal, int64_t max_rows_words, int treshold, int runs,
                  double *scores, double *p, double *xbuf, uint8_t *status, unsigned *flags, double *slab,
                  hipStream_t s, hipEvent_t ev_perm) {
  const bool perms = runs > 0 && treshold > 0;
  const int want_x1 = (perms || mds == 2) ? 1 : 0; /* coordinates out of the classical stage */
  const char *fl = getenv("GD_CSS_FORCE_LITERAL"); /* diagnostics: per-SNP predicate for every window */
  const int force_literal = (fl && fl[0] == '1' && !acodes) ? 1 : 0;
  if (acodes) {
    const int st = gd_packed_css_planes_launch(d_ch, nchrom, d_pl, word_off, acodes, bcodes, max_rows_words, planes, s);
    if (st) return st;
  } else if (!drosophila) {
    const unsigned gx = (unsigned)std::min<int64_t>((max_rows_words * 8 + 255) / 256, std::max(1, 16384 / nchrom));
    hipLaunchKernelGGL(k_css_pack, dim3(std::max(1u, gx), nchrom, 2), dim3(256), 0, s, d_ch, d_pl, avals, bvals,
                       planes);
    if (hipGetLastError() != hipSuccess) return GD_ERR_HIP;
  }
  int st = GD_OK;
  if (mds != 1) {
    if (drosophila) {
      st = gd_css_freq_cmds_launch(mp, d_ch, nchrom, lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x1, scores, p, xbuf,
                                   status, flags, s);
    } else {
#define CSS_TIER(T, G)                                                                                          \
  case T:                                                                                                       \
    st = launch_tier<T, G>(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x1,         \
                           force_literal, scores, p, xbuf, status, flags, s);                                   \
    break;
      switch (mp) {
        CSS_TIER(24, 1)
#if CSS_P40
        case 40:
          st = gd_css_launch_p40(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x1, force_literal,
                          scores, p, xbuf, status, flags, s);
          break;
#else
        CSS_TIER(40, 1)
#endif
        CSS_TIER(64, 1)
#if CSS_T80
        case 80:
          st = gd_css_launch_t80(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x1, force_literal,
                          scores, p, xbuf, status, flags, s);
          break;
#else
        CSS_TIER(80, CSS_G80)
#endif
        CSS_TIER(96, 2)
        CSS_TIER(128, 2)
        default:
          if (mp <= GD_CSS_TIER_MAX || mp > GD_CSS_BIG_MAX) return GD_ERR_SIZE;
          st = gd_css_launch_big(mp, d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x1, force_literal,
                          scores, p, xbuf, status, flags, slab, s);
      }
#undef CSS_TIER
    }
    if (st) return st;
  }
  if (mds != 0) {
    st = gd_css_smacof_launch(mp, drosophila != 0, d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal,
                              mds, perms ? 1 : 0, force_literal, scores, p, xbuf, status, flags, slab, s);
    if (st) return st;
  }
  if (ev_perm && hipEventRecord(ev_perm, s) != hipSuccess) return GD_ERR_HIP; /* end of the MDS stage */
  if (perms) st = gd_css_perm_launch(mp, d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, flags + 8, slab, s);
  return st;
}
