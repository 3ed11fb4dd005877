/*
 * gd_css_big.hip -- the CSS MDS general path above 128 individuals (k_css_mds_big; css.c:181-223, 277-366, 505-647; threadcss.c:207-215)
 */
#include "gd_css_common.h"

/* ------------------------------------------------------------------------ */
/* The general path: cohorts above the register tiers (GD_CSS_TIER_MAX < m <=  */
/* GD_CSS_BIG_MAX; the reference scores any m, threadcss.c:191,207-215).  The    */
/* same algorithm as k_css_mds -- compare_all by popcounts (literal predicate for */
/* irregular windows), fill_averages, double centering, Householder (dsytd2,      */
/* lower), bisection for the top two eigenvalues, inverse iteration, back-        */
/* transformation, X, css -- with thread t owning rows t, t + NT, .. (R rows,      */
/* NT = MP / R threads) and the matrix in a global-memory slab of the workgroup's */
/* own, column-major (element (i, j) at j ld + i): every sweep over a column      */
/* touches one contiguous 8 m-byte run, so a wave's loads coalesce.  The          */
/* workgroups loop over windows (grid = the device's resident capacity,           */
/* gd_css_big_grid).  Above 512 individuals (R = 2) the inverse-iteration factors */
/* live in the slab behind the matrix instead of LDS.                             */
/* ------------------------------------------------------------------------ */
template <int MP, int R>
__global__ void __launch_bounds__(MP / R)
    k_css_mds_big(const gd_chrom_dev *ch, int nchrom, const gd_css_planes *pl, const uint32_t *planes,
                  const int32_t *lo_a_, const int32_t *hi_a_, const int32_t *lo_b_, const double *avals,
                  const double *bvals, int64_t wtotal, int want_x, int force_literal, int xstride, double *scores,
                  double *pvals, double *xbuf, uint8_t *status, unsigned *flags, double *slab, int64_t slab_per_wg,
                  int ld) {
  constexpr int NT = MP / R, NW = NT / 64;
  constexpr bool LUG = R > 1;      /* inverse-iteration factors in the slab (LDS budget) */
  constexpr bool GSL = MP > 1024;  /* the 2048 tier: masks, iterates and coordinates in the slab too */
  static_assert(!LUG || MP == 1024 || MP == 2048, "the slab tail is sized for the 1024 and 2048 tiers");
  constexpr int64_t LU_D = MP > 1024 ? GD_CSS_BIG_LU_DOUBLES_2K : GD_CSS_BIG_LU_DOUBLES;
  constexpr int64_t GX_D = GSL ? GD_CSS_BIG_GX_DOUBLES_2K : 0;
  __shared__ double s_row[MP + 2];
  __shared__ double s_v[MP], s_w[MP];
  __shared__ __attribute__((aligned(16))) double s_d[MP + 4];
  __shared__ __attribute__((aligned(16))) double s_e2[MP + 4];
  __shared__ double s_e[MP], s_tau[MP];
  __shared__ uint64_t s_mask_l[GSL ? 1 : 2 * MP];
  __shared__ double s_y_l[2][GSL ? 1 : MP];
  __shared__ double s_lu_l[2][3][LUG ? 1 : MP];
  __shared__ uint8_t s_piv_l[2][LUG ? 1 : MP];
  __shared__ double s_x_l[GSL ? 1 : 2 * MP];
  __shared__ int s_tr[MP];
  __shared__ double s_lam[2];
  __shared__ double s_red[2 * (2 * NW + 2)];

  const int tid = threadIdx.x;
  double *A = slab + (int64_t)blockIdx.x * slab_per_wg;
  /* the slab's tail (gd_css_big_slab_per_wg): the factors, then (2048 tier) the vectors */
  double *lug = A + slab_per_wg - (LUG ? LU_D : 0) - GX_D;
  double *gx = A + slab_per_wg - GX_D;
  double(*s_lu)[3][MP] = LUG ? reinterpret_cast<double(*)[3][MP]>(lug)
                             : reinterpret_cast<double(*)[3][MP]>(&s_lu_l[0][0][0]);
  uint8_t(*s_piv)[MP] = LUG ? reinterpret_cast<uint8_t(*)[MP]>(lug + 6 * MP)
                            : reinterpret_cast<uint8_t(*)[MP]>(&s_piv_l[0][0]);
  uint64_t *s_mask = GSL ? reinterpret_cast<uint64_t *>(gx) : &s_mask_l[0];
  double(*s_y)[MP] = GSL ? reinterpret_cast<double(*)[MP]>(gx + 2 * MP) : reinterpret_cast<double(*)[MP]>(&s_y_l[0][0]);
  double *s_x = GSL ? gx + 4 * MP : &s_x_l[0];
  auto at = [&](int r, int c) -> double & { return A[(int64_t)c * ld + r]; };
  for (int t = tid; t < MP; t += NT) s_tr[t] = t;

  for (int64_t w = blockIdx.x; w < wtotal; w += gridDim.x) {
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
    if (m > MP || m > ld) {
      if (tid == 0) atomicOr(flags, GD_FLAG_BAD_SIZE);
      continue;
    }
    const gd_css_planes P = pl[c];
    const uint32_t *pa = planes + P.pa, *pb = planes + P.pb;
    const int64_t ra = la / a, rb = lb / b;
    __syncthreads(); /* the previous window's readers of s_x / s_tr are done */

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

    /* ---- compare_all into column-major A (counts as doubles; the diagonal is 0) */
    if (!literal) {
      for (int k = 0; k * 64 < npos; ++k) {
        const int nb = min(64, npos - 64 * k);
        const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
        __syncthreads();
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
          const int i = tid + rr * NT;
          if (i < m) {
            const uint32_t *base = i < a ? pa + (int64_t)(2 * i) * P.wa : pb + (int64_t)(2 * (i - a)) * P.wb;
            const int64_t nw = i < a ? P.wa : P.wb;
            const int64_t r = (i < a ? ra : rb) + 64 * k;
            s_mask[2 * i] = plane_bits64(base, r) & tail;
            s_mask[2 * i + 1] = plane_bits64(base + nw, r) & tail;
          }
        }
        __syncthreads();
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
          const int i = tid + rr * NT;
          if (i < m) {
            const uint64_t Pi = s_mask[2 * i], Ni = s_mask[2 * i + 1];
            for (int j = 0; j < m; ++j) {
              const double cnt = (double)(__popcll(Pi & s_mask[2 * j + 1]) + __popcll(Ni & s_mask[2 * j]));
              at(i, j) = k == 0 ? cnt : at(i, j) + cnt;
            }
          }
        }
      }
    } else {
      const double *av = avals + d.a_off + la, *bv = bvals + d.b_off + lb;
      auto val = [&](int r, int k) { return r < a ? av[(int64_t)k * a + r] : bv[(int64_t)k * b + (r - a)]; };
#pragma unroll 1
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m)
          for (int j = 0; j < m; ++j) {
            int cnt = 0;
            /* the reference casts the row element of the larger index within a population and
             * the A element across populations (css.c:281-326); the diagonal never counts */
            const bool cast_i = ((i < a) == (j < a)) ? (i > j) : (i < a);
            if (j != i)
              for (int k = 0; k < npos; ++k) {
                const double vi = val(i, k), vj = val(j, k);
                const double prod = cast_i ? x86_int(vi) * vj : x86_int(vj) * vi;
                cnt += prod == -9.0;
              }
            at(i, j) = (double)cnt;
          }
      }
    }

    /* ---- fill_averages: entries < 1e-5 (diagonal included) count as unknown */
    double zero_tol;
    {
      double unv = 0.0, sum = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m)
          for (int j = 0; j < m; ++j) {
            const double x = at(i, j);
            if (x < 0.00001)
              unv += 1.0;
            else
              sum += x;
          }
      }
      block_sum2<NW>(unv, sum, s_red); /* sums of integers: exact in any order */
      const int tot = m * m;
      if ((int)unv > tot / 2) continue; /* discarded window: outputs untouched */
      const double avg = sum / tot;
      /* B = -1/2 Z (D o D) Z by double centering, as k_css_mds */
      double ri[R], rsum = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        double rs = 0.0;
        if (i < m)
          for (int j = 0; j < m; ++j) {
            double x = at(i, j);
            x = fma(avg, 1.0 - fmin(x, 1.0), x);
            x = x * x;
            at(i, j) = x;
            rs += x;
          }
        ri[rr] = i < m ? rs / m : 0.0;
        if (i < MP) s_v[i] = ri[rr];
        rsum += ri[rr];
      }
      const double g = block_sum<NW>(rsum, s_red) / m;
      __syncthreads();
      double f2 = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m)
          for (int j = 0; j < m; ++j) {
            const double x = -0.5 * ((at(i, j) - (ri[rr] + s_v[j])) + g);
            at(i, j) = x;
            f2 = fma(x, x, f2);
          }
      }
      zero_tol = 64.0 * m * DBL_EPSILON * sqrt(block_sum<NW>(f2, s_red));
    }

    /* ---- Householder tridiagonalisation (dsytd2, lower), the k_css_mds step on the slab;
     * after step k column k holds the reflector v_k */
    for (int k = 0; k < m; ++k) {
      __syncthreads();
      /* row k right of the diagonal (zeros at j <= k) and d_k; A(k, j) as lane k holds it */
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m) s_row[i] = i > k ? at(k, i) : 0.0;
        if (i == k) s_d[k] = at(k, k);
      }
      __syncthreads();
      if (k >= m - 2) {
        if (tid == 0 && k == m - 2) s_e[k] = s_row[k + 1];
        continue;
      }
      const double alpha = s_row[k + 1];
      double xi[R], praw[R], ak1[R];
      double sigma = 0.0, q = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        const bool row = i < m;
        xi[rr] = (i > k + 1 && row) ? s_row[i] : 0.0;
        praw[rr] = 0.0;
        ak1[rr] = 0.0;
        if (i > k && row) {
          double p0 = 0.0, p1 = 0.0;
          int j = k + 1;
          for (; j + 1 < m; j += 2) {
            p0 = fma(at(i, j), s_row[j], p0);
            p1 = fma(at(i, j + 1), s_row[j + 1], p1);
          }
          if (j < m) p0 = fma(at(i, j), s_row[j], p0);
          praw[rr] = p0 + p1;
          ak1[rr] = at(i, k + 1);
        }
        sigma = fma(xi[rr], xi[rr], sigma);
        if (i > k && row) q = fma(s_row[i], praw[rr], q);
        if (i == k + 1) {
          s_red[2 * NW] = praw[rr];
          s_red[2 * NW + 1] = ak1[rr];
        }
      }
      block_sum2<NW>(sigma, q, s_red);
      const double pr1 = s_red[2 * NW], a11 = s_red[2 * NW + 1];
      double tau = 0.0, beta = alpha, scale = 0.0;
      if (sigma != 0.0) {
        beta = -copysign(sqrt_pos(alpha * alpha + sigma), alpha);
        const double r = fast_rcp(beta * (alpha - beta));
        tau = -(alpha - beta) * (alpha - beta) * r;
        scale = beta * r;
      }
      /* v = scale (x - beta e_{k+1}), v_{k+1} = 1;  p = tau A v;  w = p + K v */
      const double K = -0.5 * tau * (tau * scale * scale) * fma(beta, fma(beta, a11, -2.0 * pr1), q);
      double vi[R], wi[R];
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        const bool row = i < m;
        vi[rr] = (i == k + 1) ? 1.0 : xi[rr] * scale;
        const double pi = (i > k && row) ? (tau * scale) * fma(-beta, ak1[rr], praw[rr]) : 0.0;
        wi[rr] = fma(K, vi[rr], pi);
        if (i < MP) {
          s_v[i] = vi[rr];
          s_w[i] = wi[rr];
        }
      }
      if (tid == 0) {
        s_e[k] = beta;
        s_tau[k] = tau;
      }
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i > k && i < m)
          for (int j = k + 1; j < m; ++j) at(i, j) = fma(-vi[rr], s_w[j], fma(-wi[rr], s_v[j], at(i, j)));
        if (i < m) at(i, k) = vi[rr]; /* stash v_k in the dead column k */
      }
    }
    __syncthreads();

    /* ---- the two largest eigenvalues of T (as k_css_mds) */
    double glo, ghi;
    {
      double lo = DBL_MAX, hi = -DBL_MAX;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m) {
          const double r = (i > 0 ? fabs(s_e[i - 1]) : 0.0) + (i < m - 1 ? fabs(s_e[i]) : 0.0);
          lo = fmin(lo, s_d[i] - r);
          hi = fmax(hi, s_d[i] + r);
        }
      }
      for (int t = tid; t < MP + 4; t += NT) s_e2[t] = (t >= 1 && t < m) ? s_e[t - 1] * s_e[t - 1] : 0.0;
      glo = block_reduce<NW, OpMin>(lo, s_red);
      ghi = block_reduce<NW, OpMax>(hi, s_red);
      const double pad = 2.0 * DBL_EPSILON * fmax(fabs(glo), fabs(ghi)) * m + DBL_MIN;
      glo -= pad;
      ghi += pad;
      for (int t = tid; t < MP + 4; t += NT)
        if (t >= m) s_d[t] = 2.0 * fabs(ghi) + 2.0 * fabs(glo) + 1.0;
    }
    const double bis_tol = CSS_BISECT_TOL * fmax(fabs(glo), fabs(ghi)) + DBL_MIN;
    __syncthreads();
    if (tid < 64) bisect_top2(m, glo, ghi, bis_tol, s_d, s_e2, s_lam, tid);
    __syncthreads();

    /* ---- eigenvectors of T: two inverse-iteration solves, orthogonalised */
    if (tid < 2) invit_factor<MP>(m, tid, s_d, s_e, s_lam, s_lu, s_x, s_piv, s_y);
    __syncthreads();
    {
      const double tiny = DBL_EPSILON * fmax(fmax(fabs(glo), fabs(ghi)), DBL_MIN);
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const double u0 = s_lu[e][0][i];
            s_lu[e][0][i] = fast_rcp(u0 == 0.0 ? tiny : u0);
          }
      }
    }
    double y1[R], y2[R];
#pragma unroll
    for (int rr = 0; rr < R; ++rr) y1[rr] = y2[rr] = 0.0;
    for (int itn = 0; itn < 2; ++itn) {
      __threadfence_block();
      __syncthreads();
      if (tid < 2) invit_solve<MP>(m, tid, s_lu, s_x, s_piv, s_y);
      __syncthreads();
      double n1 = 0.0, n2 = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        y1[rr] = i < m ? s_y[0][i] : 0.0;
        y2[rr] = i < m ? s_y[1][i] : 0.0;
        n1 = fma(y1[rr], y1[rr], n1);
        n2 = fma(y2[rr], y2[rr], n2);
      }
      block_sum2<NW>(n1, n2, s_red);
      const double s1 = 1.0 / sqrt(n1), s2 = 1.0 / sqrt(n2);
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        y1[rr] *= s1;
        y2[rr] *= s2;
        if (itn == 0 && i < m) {
          s_y[0][i] = y1[rr];
          s_y[1][i] = y2[rr];
        }
      }
    }
    {
      double dt = 0.0, zero = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) dt = fma(y1[rr], y2[rr], dt);
      block_sum2<NW>(dt, zero, s_red);
      double n2 = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        y2[rr] = fma(-dt, y1[rr], y2[rr]);
        n2 = fma(y2[rr], y2[rr], n2);
      }
      zero = 0.0;
      block_sum2<NW>(n2, zero, s_red);
      const double s2 = 1.0 / sqrt(n2);
#pragma unroll
      for (int rr = 0; rr < R; ++rr) y2[rr] *= s2;
    }
    {
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m) {
          s_y[0][i] = y1[rr];
          s_y[1][i] = y2[rr];
        }
      }
      __syncthreads();
      double t1 = 0.0, t2 = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m) {
          const double el = i > 0 ? s_e[i - 1] : 0.0, er = i + 1 < m ? s_e[i] : 0.0;
          const int il = i > 0 ? i - 1 : 0, ir = i + 1 < m ? i + 1 : i;
          t1 += y1[rr] * (s_d[i] * y1[rr] + el * s_y[0][il] + er * s_y[0][ir]);
          t2 += y2[rr] * (s_d[i] * y2[rr] + el * s_y[1][il] + er * s_y[1][ir]);
        }
      }
      block_sum2<NW>(t1, t2, s_red);
      if (tid == 0) {
        s_lam[0] = fabs(t1) <= zero_tol ? 0.0 : t1;
        s_lam[1] = fabs(t2) <= zero_tol ? 0.0 : t2;
      }
      __syncthreads();
    }

    /* ---- back-transformation y <- H_0 H_1 ... H_{m-3} y (v_k in column k) */
    for (int k = m - 3; k >= 0; --k) {
      double vk[R], d1 = 0.0, d2 = 0.0;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        vk[rr] = i < m ? at(i, k) : 0.0;
        d1 = fma(vk[rr], y1[rr], d1);
        d2 = fma(vk[rr], y2[rr], d2);
      }
      const double t = s_tau[k];
      block_sum2<NW>(d1, d2, s_red);
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        y1[rr] = fma(-(t * d1), vk[rr], y1[rr]);
        y2[rr] = fma(-(t * d2), vk[rr], y2[rr]);
      }
    }

    /* ---- X = Q sqrt(L) (css.c:545-556), then calc_dist + css on identity groups */
    {
      const double L1 = sqrt(s_lam[0]), L2 = sqrt(s_lam[1]);
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        const int i = tid + rr * NT;
        if (i < m) {
          s_x[2 * i] = y1[rr] * L1 + y2[rr] * 0.0;
          s_x[2 * i + 1] = y1[rr] * 0.0 + y2[rr] * L2;
        }
      }
      __syncthreads();
    }
    const double score = css_score<NW>(s_tr, a, b, [&](int p, int q) { return xdist(s_x, p, q); }, s_red);
    if (score == -1.0) continue; /* the reference's "discarded" marker (css.c:127) */
    if (tid == 0) {
      scores[d.w_out + wl] = score;
      if (!want_x) pvals[d.w_out + wl] = 1.0; /* runs == 0: p = (0 + 1) / (0 + 1) */
    }
    if (want_x) {
      for (int e = tid; e < xstride; e += NT) xbuf[w * xstride + e] = (e < 2 * m) ? s_x[e] : 0.0;
      if (tid == 0) status[w] = 1;
    }
  }
}


int gd_css_launch_big(int mp, const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, double *slab, hipStream_t s) {
  const int ld = gd_css_big_ld(mp);
  const int64_t per = gd_css_big_slab_per_wg(mp), grid = gd_css_big_grid(wtotal, mp);
  CSS_PROF_LAUNCH(s);
#define CSS_BIG(T, RR)                                                                                             \
  hipLaunchKernelGGL((k_css_mds_big<T, RR>), dim3((unsigned)grid), dim3(T / RR), 0, s, d_ch, nchrom, d_pl, planes, \
                     lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x, force_literal, 2 * mp, scores, p, xbuf, status,  \
                     flags, slab, per, ld)
  if (mp <= 256)
    CSS_BIG(256, 1);
  else if (mp <= 512)
    CSS_BIG(512, 1);
  else if (mp <= 1024)
    CSS_BIG(1024, 2);
  else
    CSS_BIG(2048, 4);
#undef CSS_BIG
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}
