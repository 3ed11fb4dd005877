/*
 * gd_css_h40.hip -- the 25..40-individual CSS MDS tier, two windows per wave (k_css_mds_h40 / k_css_mds_p40; css.c:181-223, 277-366, 505-647)
 */
#include "gd_css_common.h"

/* ------------------------------------------------------------------------ */
/* The 25..40-individual tier with TWO windows per wave (k_css_mds_p40).  Window */
/* A's rows sit in lanes 0..39 (40 columns each), window B's rows 0..23 in lanes */
/* 40..63 and its rows 24..39 in LDS, each worked by a lane quad over interleaved */
/* columns (as k_css_mds_t80).  Both windows run the same Householder            */
/* instructions; reductions, scalar recurrences and the eigen phases are kept per */
/* window.  The one-window layout left 24 lanes idle and paid every per-step      */
/* instruction for 40 rows; here one instruction serves 80.                       */
/* ------------------------------------------------------------------------ */
namespace {
constexpr int P40 = 40, P40_BMAIN = 24, P40_TS = 10; /* order, B rows in VGPRs, tail columns per lane */
/* tail row stride in doubles: 2 * 44 = 24 (mod 64) dwords, so the 8 tail rows of a 32-lane
 * group start 8 banks apart (k_css_mds_t80) */
constexpr int P40_TSTRIDE = 44;
#ifndef H40_BPERM
#define H40_BPERM 1
#endif

/* the Householder scalars of one window from its reduced |x|^2 (sigma), r^T A r (q),
 * (A r)_{K+1} (pr1) and A_{K+1,K+1} (a11) -- hh_step_static's recurrences */
__device__ __forceinline__ void hh_scalars(double alpha, double sigma, double q, double pr1, double a11, double *tau,
                                           double *beta, double *scale, double *Kc) {
  double t = 0.0, be = alpha, sc = 0.0;
  if (sigma != 0.0) {
    be = -copysign(sqrt_pos(alpha * alpha + sigma), alpha);
    const double r = fast_rcp(be * (alpha - be));
    t = -(alpha - be) * (alpha - be) * r;
    sc = be * r;
  }
  *tau = t;
  *beta = be;
  *scale = sc;
  *Kc = -0.5 * t * (t * sc * sc) * fma(be, fma(be, a11, -2.0 * pr1), q);
}

template <int K>
__device__ __forceinline__ void p40_step(double (&A)[P40], int mA, int mB, double (*s_row)[P40 + 2],
                                         double (*s_v)[P40], double (*s_w)[P40], double (*s_d)[P40 + 4],
                                         double (*s_e)[P40], double (*s_tau)[P40], double (*s_tail)[P40_TSTRIDE]) {
  constexpr int MP = P40;
  const int lane = css_lane_now();
  const int win = lane < MP ? 0 : 1, r = win ? lane - MP : lane;
  const int tr = lane >> 2, tq = lane & 3, R = P40_BMAIN + tr;
  const bool row = r < (win ? mB : mA), trow = R < mB;
  __syncthreads();
  /* publish row K of each window (zeros at j <= K) and its diagonal */
  {
    const bool pubA = lane == K, pubB = K < P40_BMAIN && lane == MP + K;
    if (pubA || pubB) {
      double *dst = s_row[pubA ? 0 : 1];
#pragma unroll
      for (int jb = 0; jb < MP / 8; ++jb)
        if (8 * jb + 7 >= K) {
#pragma unroll
          for (int u = 0; u < 8; u += 2) {
            const int j = 8 * jb + u;
            *reinterpret_cast<double2 *>(dst + j) = make_double2(j > K ? A[j] : 0.0, j + 1 > K ? A[j + 1] : 0.0);
          }
        }
      s_d[pubA ? 0 : 1][K] = A[K];
    }
  }
  if constexpr (K >= P40_BMAIN) {
    const double *src = s_tail[K - P40_BMAIN];
    if (lane < MP) s_row[1][lane] = lane > K ? src[lane] : 0.0;
    if (lane == 0) s_d[1][K] = src[K];
  }
  __syncthreads();
  if constexpr (K >= MP - 2) {
    if (lane == 0) {
      if (K == mA - 2) s_e[0][K] = s_row[0][K + 1];
      if (K == mB - 2) s_e[1][K] = s_row[1][K + 1];
    }
    return;
  } else {
    const double *srw = s_row[win];
    const double xi = (r > K + 1 && row) ? srw[r] : 0.0;
    double p0 = 0, p1 = 0;
#pragma unroll
    for (int jb = 0; jb < MP / 8; ++jb) {
      if (8 * jb + 7 > K) {
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
          if (8 * jb + u > K) p0 = fma(A[8 * jb + u], srw[8 * jb + u], p0);
          if (8 * jb + u + 1 > K) p1 = fma(A[8 * jb + u + 1], srw[8 * jb + u + 1], p1);
        }
        CSS_PIN(p0);
        CSS_PIN(p1);
      }
    }
    const double ak1 = A[K + 1];
    const double praw = p0 + p1;
    /* window B's tail row over the live column groups (s_row is 0 at j <= K) */
    const double *trw = s_tail[tr];
    const double *srb = s_row[1];
    double t0 = 0, t1 = 0;
#pragma unroll
    for (int s = 0; s < P40_TS; ++s) {
      if (4 * s + 3 > K) {
        const int j = 4 * s + tq;
        if (s & 1)
          t1 = fma(trw[j], srb[j], t1);
        else
          t0 = fma(trw[j], srb[j], t0);
      }
    }
    const double pt = quad_sum(t0 + t1);
    const double akt = trw[K + 1];
    const double xr = (R > K + 1 && trow) ? srb[R] : 0.0;
    /* |x|^2 and r^T A r per window in two reductions */
    const double sq = xi * xi, qm = ((r > K && row) ? srw[r] : 0.0) * praw;
    double sigA = win ? 0.0 : sq, qA = win ? 0.0 : qm;
    double sigB = (win ? sq : 0.0) + (tq == 0 ? xr * xr : 0.0);
    double qB = (win ? qm : 0.0) + ((tq == 0 && R > K && trow) ? srb[R] * pt : 0.0);
    wave_sum2(sigA, qA);
    wave_sum2(sigB, qB);
    const double pr1A = readlane_f64(praw, K + 1), a11A = readlane_f64(ak1, K + 1);
    double pr1B, a11B;
    if constexpr (K + 1 < P40_BMAIN) {
      pr1B = readlane_f64(praw, MP + K + 1);
      a11B = readlane_f64(ak1, MP + K + 1);
    } else {
      pr1B = readlane_f64(pt, 4 * (K + 1 - P40_BMAIN));
      a11B = readlane_f64(akt, 4 * (K + 1 - P40_BMAIN));
    }
    double tauA, betaA, scaleA, KcA, tauB, betaB, scaleB, KcB;
    hh_scalars(s_row[0][K + 1], sigA, qA, pr1A, a11A, &tauA, &betaA, &scaleA, &KcA);
    hh_scalars(srb[K + 1], sigB, qB, pr1B, a11B, &tauB, &betaB, &scaleB, &KcB);
    const double tau = win ? tauB : tauA, beta = win ? betaB : betaA, scale = win ? scaleB : scaleA,
                 Kc = win ? KcB : KcA;
    const double vi = (r == K + 1) ? 1.0 : xi * scale;
    const double pi = (r > K && row) ? (tau * scale) * fma(-beta, ak1, praw) : 0.0;
    const double wi = fma(Kc, vi, pi);
    const double vt = (R == K + 1) ? 1.0 : xr * scaleB;
    const double ptl = (R > K && trow) ? (tauB * scaleB) * fma(-betaB, akt, pt) : 0.0;
    const double wt = fma(KcB, vt, ptl);
    if (lane == 0) {
      s_e[0][K] = betaA;
      s_tau[0][K] = tauA;
      s_e[1][K] = betaB;
      s_tau[1][K] = tauB;
    }
    s_v[win][r] = vi;
    s_w[win][r] = wi;
    if (tq == 0) {
      s_v[1][R] = vt;
      s_w[1][R] = wt;
    }
    __syncthreads();
    const double *sv = s_v[win], *sw = s_w[win];
#pragma unroll
    for (int jb = 0; jb < MP / 8; ++jb) {
      if (8 * jb + 7 > K) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = 8 * jb + u;
          if (j > K) A[j] = fma(-vi, sw[j], fma(-wi, sv[j], A[j]));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) CSS_PIN(A[8 * jb + u]);
      }
    }
    A[K] = vi; /* stash v_K in the dead column K */
    double *tw = s_tail[tr];
    const double *svb = s_v[1], *swb = s_w[1];
#pragma unroll
    for (int s = 0; s < P40_TS; ++s) {
      if (4 * s + 3 > K) {
        const int j = 4 * s + tq;
        tw[j] = fma(-vt, swb[j], fma(-wt, svb[j], tw[j]));
      }
    }
    if (tq == (K & 3)) tw[K] = vt;
  }
}

template <int K>
struct P40Steps {
  static __device__ __forceinline__ void run(double (&A)[P40], int mA, int mB, double (*s_row)[P40 + 2],
                                             double (*s_v)[P40], double (*s_w)[P40], double (*s_d)[P40 + 4],
                                             double (*s_e)[P40], double (*s_tau)[P40],
                                             double (*s_tail)[P40_TSTRIDE]) {
    if ((K & 7) == 0 && K >= mA && K >= mB) return; /* exits only at block boundaries (hh_step_static) */
    p40_step<K>(A, mA, mB, s_row, s_v, s_w, s_d, s_e, s_tau, s_tail);
    P40Steps<K + 1>::run(A, mA, mB, s_row, s_v, s_w, s_d, s_e, s_tau, s_tail);
  }
};
template <>
struct P40Steps<P40> {
  static __device__ __forceinline__ void run(double (&)[P40], int, int, double (*)[P40 + 2], double (*)[P40],
                                             double (*)[P40], double (*)[P40 + 4], double (*)[P40], double (*)[P40],
                                             double (*)[P40_TSTRIDE]) {}
};

/* 17-section bisection for the two largest eigenvalues of both windows' T, a quarter
 * wave per eigenvalue (bisect_top2 with 16 lanes instead of 32) */
template <bool ZFIX = true> /* false: FMA-only chain over floored e^2 (bisect_top2) */
__device__ __forceinline__ void p40_bisect(int mA, int mB, const double *glo, const double *ghi, const double *tol,
                                           const double (*s_d)[P40 + 4], const double (*s_e2)[P40 + 4],
                                           double (*s_lam)[2], int lane) {
  const int w = lane >> 5, hh = (lane >> 4) & 1, j = lane & 15;
  const int m = w ? mB : mA;
  const int m4 = (m + 3) & ~3;
  const int target = m - 1 - hh;
  const double *dd = s_d[w], *ee = s_e2[w];
  double l = m > 0 ? glo[w] : 0.0, u = m > 0 ? ghi[w] : 0.0;
  const double bt = tol[w];
  bool conv = m <= 0;
#ifdef GD_CSS_SKIP_BISECT
  conv = true;
#endif
  for (int it = 0; it < 120; ++it) {
    if (__all(conv)) break;
    const double x = l + (u - l) * ((double)(j + 1) * (1.0 / 17.0));
    double pm = 1.0, pc = 1.0;
    int cnt = 0;
    for (int k = 0; k < m4; k += 4) {
      const double2 d01 = *reinterpret_cast<const double2 *>(dd + k);
      const double2 d23 = *reinterpret_cast<const double2 *>(dd + k + 2);
      const double2 e01 = *reinterpret_cast<const double2 *>(ee + k);
      const double2 e23 = *reinterpret_cast<const double2 *>(ee + k + 2);
      const double dk[4] = {d01.x, d01.y, d23.x, d23.y};
      const double ek[4] = {e01.x, e01.y, e23.x, e23.y};
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        double pn = fma(dk[uu] - x, pc, -(ek[uu] * pm));
        if constexpr (ZFIX) pn = (pn == 0.0) ? -pc * DBL_MIN : pn;
        cnt += (int)((__double2hiint(pn) ^ __double2hiint(pc)) < 0);
        pm = pc;
        pc = pn;
      }
      const int ex = __builtin_amdgcn_frexp_exp(fmax(fabs(pm), fabs(pc)));
      pm = __builtin_amdgcn_ldexp(pm, -ex);
      pc = __builtin_amdgcn_ldexp(pc, -ex);
    }
    double nl = cnt <= target ? x : l;
    double nu = cnt <= target ? u : x;
    nl = row_allreduce<OpMax>(nl); /* the quarter wave is one DPP row */
    nu = row_allreduce<OpMin>(nu);
    if (!conv) {
      const bool same = (nl == l && nu == u);
      l = nl;
      u = nu;
      conv = same || (u - l) <= bt;
    }
  }
  if (j == 0 && m > 0) s_lam[w][hh] = 0.5 * (l + u);
}
}  // namespace

#ifndef CSS_P40_WAVES
#define CSS_P40_WAVES 3 /* waves per SIMD the register allocator must reach */
#endif
__global__ void __launch_bounds__(64, CSS_P40_WAVES)
    k_css_mds_p40(const gd_chrom_dev *ch, int nchrom, const gd_css_planes *pl, const uint32_t *planes,
                  const int32_t *lo_a_, const int32_t *hi_a_, const int32_t *lo_b_, const double *avals,
                  const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *pvals,
                  double *xbuf, uint8_t *status, unsigned *flags) {
  constexpr int MP = P40;
  __shared__ __attribute__((aligned(16))) double s_tail[MP - P40_BMAIN][P40_TSTRIDE];
  __shared__ __attribute__((aligned(16))) union {
    struct {
      double e2[2][MP + 4]; /* bisection only (after the Householder steps) */
      double row[2][MP + 2];
      double v[2][MP], w[2][MP];
      uint64_t mask[2][2 * MP];
      double vals[2][MP];
    } a;
    struct {
      double lu[2][2][3][MP];
      double y[2][2][MP];
      uint8_t piv[2][2][MP];
    } b;
  } s_u;
  __shared__ __attribute__((aligned(16))) double s_d[2][MP + 4];
  __shared__ double s_e[2][MP], s_tau[2][MP];
  __shared__ double s_x[2][2 * MP];
  __shared__ int s_tr[MP];
  __shared__ double s_lam[2][2];
  __shared__ double s_red[4];

  const int lane = threadIdx.x;
  const int win = lane < MP ? 0 : 1, r = win ? lane - MP : lane;
  const int tr = lane >> 2, tq = lane & 3, R = P40_BMAIN + tr;
  if (lane < MP) s_tr[lane] = lane;

  /* the two windows' bookkeeping (uniform) */
  int64_t W[2];
  int C[2], Aa[2], Bb[2], M[2], npos[2];
  int32_t LA[2], LB[2];
  bool lit[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    W[x] = 2 * (int64_t)blockIdx.x + x;
    M[x] = 0;
    C[x] = 0;
    Aa[x] = Bb[x] = 1;
    npos[x] = 0;
    LA[x] = LB[x] = 0;
    lit[x] = false;
    if (W[x] >= wtotal) continue;
    const int c = chrom_of(ch, nchrom, W[x]);
    const gd_chrom_dev &d = ch[c];
    const int a = d.asize, b = d.bsize, m = a + b;
    const int32_t la = lo_a_[W[x]], ha = hi_a_[W[x]], lb = lo_b_[W[x]];
    const int np = (ha - la) / a;
    if (np <= 0) continue;
    if ((int64_t)lb + (int64_t)np * b > d.blen) {
      if (lane == 0) atomicOr(flags, GD_FLAG_B_BOUNDS);
      continue;
    }
    if (m > MP) {
      if (lane == 0) atomicOr(flags, GD_FLAG_BAD_SIZE);
      continue;
    }
    C[x] = c;
    Aa[x] = a;
    Bb[x] = b;
    M[x] = m;
    npos[x] = np;
    LA[x] = la;
    LB[x] = lb;
    lit[x] = force_literal || (la % a) != 0 || (lb % b) != 0;
  }
  if (M[0] == 0 && M[1] == 0) return;
  CSS_PROF_INIT;

  /* ---- regular windows?  (k_css_mds) */
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    if (M[x] == 0 || lit[x]) continue;
    const gd_css_planes P = pl[C[x]];
    const int a = Aa[x], b = Bb[x];
    const int64_t ra = LA[x] / a, rb = LB[x] / b;
    int irr = 0;
    for (int k = lane; k * 64 < npos[x]; k += 64) {
      const int nb = min(64, npos[x] - 64 * k);
      const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
      const uint64_t xa = plane_bits64(planes + P.pa + (int64_t)(2 * a) * P.wa, ra + 64 * k) & tail;
      const uint64_t xb = plane_bits64(planes + P.pb + (int64_t)(2 * b) * P.wb, rb + 64 * k) & tail;
      irr |= (xa | xb) != 0;
    }
    lit[x] = __syncthreads_or(irr);
  }

  /* ---- compare_all: main row r of window `win` in A, tail row R of B into s_tail */
  const int mm = M[win];
  const bool row = r < mm, trow = R < M[1];
  double A[MP];
  {
    int acc[MP], acct[P40_TS];
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) acc[jj] = 0;
#pragma unroll
    for (int s = 0; s < P40_TS; ++s) acct[s] = 0;
    const bool popA = M[0] > 0 && !lit[0], popB = M[1] > 0 && !lit[1];
    const int nk = max(popA ? (npos[0] + 63) >> 6 : 0, popB ? (npos[1] + 63) >> 6 : 0);
    for (int k = 0; k < nk; ++k) {
      __syncthreads();
      for (int idx = lane; idx < 2 * MP; idx += 64) {
        const int x = idx >= MP, rr = x ? idx - MP : idx;
        uint64_t Pm = 0, Nm = 0;
        if ((x ? popB : popA) && rr < M[x] && 64 * k < npos[x]) {
          const gd_css_planes P = pl[C[x]];
          const int a = Aa[x], b = Bb[x];
          const int nb = min(64, npos[x] - 64 * k);
          const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
          const uint32_t *base = rr < a ? planes + P.pa + (int64_t)(2 * rr) * P.wa
                                        : planes + P.pb + (int64_t)(2 * (rr - a)) * P.wb;
          const int64_t nw = rr < a ? P.wa : P.wb;
          const int64_t r0 = (rr < a ? LA[x] / a : LB[x] / b) + 64 * k;
          Pm = plane_bits64(base, r0) & tail;
          Nm = plane_bits64(base + nw, r0) & tail;
        }
        s_u.a.mask[x][2 * rr] = Pm;
        s_u.a.mask[x][2 * rr + 1] = Nm;
      }
      __syncthreads();
      const uint64_t *mk = s_u.a.mask[win];
      const uint64_t Pi = mk[2 * r], Ni = mk[2 * r + 1];
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) {
        acc[jj] += __popcll(Pi & mk[2 * jj + 1]) + __popcll(Ni & mk[2 * jj]);
        if ((jj & 7) == 7) {
#pragma unroll
          for (int u = jj - 7; u <= jj; ++u) CSS_PIN(acc[u]);
        }
      }
      const uint64_t *mb = s_u.a.mask[1];
      const uint64_t Pt = mb[2 * R], Nt = mb[2 * R + 1];
#pragma unroll
      for (int s = 0; s < P40_TS; ++s) {
        const int j = 4 * s + tq;
        acct[s] += __popcll(Pt & mb[2 * j + 1]) + __popcll(Nt & mb[2 * j]);
      }
    }
    /* literal windows: the reference predicate per SNP (k_css_mds) */
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      if (M[x] == 0 || !lit[x]) continue;
      const gd_chrom_dev &d = ch[C[x]];
      const int a = Aa[x], b = Bb[x], m = M[x];
      const double *av = avals + d.a_off + LA[x], *bv = bvals + d.b_off + LB[x];
      for (int k = 0; k < npos[x]; ++k) {
        __syncthreads();
        for (int rr = lane; rr < m; rr += 64)
          s_u.a.vals[x][rr] = rr < a ? av[(int64_t)k * a + rr] : bv[(int64_t)k * b + (rr - a)];
        __syncthreads();
        const double *sv = s_u.a.vals[x];
        int io = r, ro = R, mo = m, ao = a;
        CSS_OPAQUE_V(io);
        CSS_OPAQUE_V(ro);
        CSS_OPAQUE_S(mo);
        CSS_OPAQUE_S(ao);
        if (win == x) {
          const double vi = sv[io];
#pragma unroll
          for (int jj = 0; jj < MP; ++jj) {
            if (jj < mo) {
              const double vj = sv[jj];
              const bool cast_i = ((io < ao) == (jj < ao)) ? (io > jj) : (io < ao);
              const double prod = cast_i ? x86_int(vi) * vj : x86_int(vj) * vi;
              acc[jj] += prod == -9.0;
            }
          }
        }
        if (x == 1) {
          const double vr = sv[ro];
#pragma unroll
          for (int s = 0; s < P40_TS; ++s) {
            const int j = 4 * s + tq;
            if (j < mo) {
              const double vj = sv[j];
              const bool cast_r = ((ro < ao) == (j < ao)) ? (ro > j) : (ro < ao);
              const double prod = cast_r ? x86_int(vr) * vj : x86_int(vj) * vr;
              acct[s] += prod == -9.0;
            }
          }
        }
      }
    }
    int mo = mm, mb = M[1];
    CSS_OPAQUE_V(mo);
    CSS_OPAQUE_S(mb);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) A[jj] = (row && jj < mo) ? (double)acc[jj] : 0.0;
#pragma unroll
    for (int s = 0; s < P40_TS; ++s) {
      const int j = 4 * s + tq;
      s_tail[tr][j] = (trow && j < mb) ? (double)acct[s] : 0.0;
    }
  }

  CSS_PROF(0);
  /* ---- fill_averages per window (k_css_mds) */
  double avgw[2];
  {
    int un = 0, unt = 0;
    double sm = 0, smt = 0;
    int mo = mm, mb = M[1];
    CSS_OPAQUE_V(mo);
    CSS_OPAQUE_S(mb);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) {
      if (row && jj < mo) {
        if (A[jj] < 0.00001)
          ++un;
        else
          sm += A[jj];
      }
    }
#pragma unroll
    for (int s = 0; s < P40_TS; ++s) {
      const int j = 4 * s + tq;
      const double t = s_tail[tr][j];
      if (trow && j < mb) {
        if (t < 0.00001)
          ++unt;
        else
          smt += t;
      }
    }
    double uA = win ? 0.0 : (double)un, sA = win ? 0.0 : sm;
    double uB = (win ? (double)un : 0.0) + (double)unt, sB = (win ? sm : 0.0) + smt;
    wave_sum2(uA, sA); /* sums of integers: exact in any order */
    wave_sum2(uB, sB);
    const double us[2] = {uA, uB}, ss[2] = {sA, sB};
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int tot = M[x] * M[x];
      avgw[x] = 0.0;
      if (M[x] == 0) continue;
      if ((int)us[x] > tot / 2) {
        M[x] = 0; /* discarded window: outputs untouched, its rows drop out below */
        continue;
      }
      avgw[x] = ss[x] / tot;
    }
  }
  if (M[0] == 0 && M[1] == 0) return;
  const int mA = M[0], mB = M[1];
  const int m_me = win ? mB : mA;
  const bool rowk = r < m_me, trowk = R < mB; /* rows of windows still alive */
  {
    const double av = win ? avgw[1] : avgw[0];
    CSS_OPAQUE_ROW(A);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) A[jj] = fma(av, 1.0 - fmin(A[jj], 1.0), A[jj]);
#pragma unroll
    for (int s = 0; s < P40_TS; ++s) {
      double *t = &s_tail[tr][4 * s + tq];
      *t = fma(avgw[1], 1.0 - fmin(*t, 1.0), *t);
    }
  }

  /* ---- B = -1/2 Z (D o D) Z per window by double centering */
  double ztol[2];
  {
    double rs = 0, rst = 0;
    int mo = m_me, mb = mB;
    CSS_OPAQUE_V(mo);
    CSS_OPAQUE_S(mb);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) {
      A[jj] = (rowk && jj < mo) ? A[jj] * A[jj] : 0.0;
      rs += A[jj];
    }
#pragma unroll
    for (int s = 0; s < P40_TS; ++s) {
      const int j = 4 * s + tq;
      double *t = &s_tail[tr][j];
      const double sq = (trowk && j < mb) ? *t * *t : 0.0;
      *t = sq;
      rst += sq;
    }
    rst = quad_sum(rst);
    const double ri = rowk ? rs / m_me : 0.0, rt = trowk ? rst / mB : 0.0;
    __syncthreads();
    s_u.a.v[win][r] = ri;
    if (tq == 0) s_u.a.v[1][R] = rt;
    double gA = win ? 0.0 : ri, gB = (win ? ri : 0.0) + (tq == 0 ? rt : 0.0);
    wave_sum2(gA, gB);
    gA = mA > 0 ? gA / mA : 0.0;
    gB = mB > 0 ? gB / mB : 0.0;
    const double g = win ? gB : gA;
    __syncthreads();
    const double *sv = s_u.a.v[win], *svb = s_u.a.v[1];
    CSS_OPAQUE_V(mo);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) {
      A[jj] = (rowk && jj < mo) ? -0.5 * ((A[jj] - (ri + sv[jj])) + g) : 0.0;
      if ((jj & 7) == 7) {
#pragma unroll
        for (int u = jj - 7; u <= jj; ++u) CSS_PIN(A[u]);
      }
    }
    double f2 = 0, f2t = 0;
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) f2 = fma(A[jj], A[jj], f2);
#pragma unroll
    for (int s = 0; s < P40_TS; ++s) {
      const int j = 4 * s + tq;
      double *t = &s_tail[tr][j];
      const double cv = (trowk && j < mb) ? -0.5 * ((*t - (rt + svb[j])) + gB) : 0.0;
      *t = cv;
      f2t = fma(cv, cv, f2t);
    }
    double fA = win ? 0.0 : f2, fB = (win ? f2 : 0.0) + f2t;
    wave_sum2(fA, fB);
    /* eigenvalues within rounding of 0 count as 0 (oracle/css_oracle.c, cmds) */
    ztol[0] = 64.0 * mA * DBL_EPSILON * sqrt(fA);
    ztol[1] = 64.0 * mB * DBL_EPSILON * sqrt(fB);
  }

  CSS_PROF(1);
  /* ---- Householder tridiagonalisation of both windows (LAPACK dsytd2, lower) */
#ifndef GD_CSS_SKIP_TRIDIAG
  P40Steps<0>::run(A, mA, mB, s_u.a.row, s_u.a.v, s_u.a.w, s_d, s_e, s_tau, s_tail);
#endif
  __syncthreads();

  CSS_PROF(2);
  /* ---- the two largest eigenvalues of each T */
  double glo[2], ghi[2], btol[2];
  {
    double lo = DBL_MAX, hi = -DBL_MAX, lot = DBL_MAX, hit = -DBL_MAX;
    if (rowk) {
      const double *e = s_e[win];
      const double rr = (r > 0 ? fabs(e[r - 1]) : 0.0) + (r < m_me - 1 ? fabs(e[r]) : 0.0);
      lo = s_d[win][r] - rr;
      hi = s_d[win][r] + rr;
    }
    if (tq == 0 && trowk) {
      const double rr = fabs(s_e[1][R - 1]) + (R < mB - 1 ? fabs(s_e[1][R]) : 0.0);
      lot = s_d[1][R] - rr;
      hit = s_d[1][R] + rr;
    }
    for (int k = lane; k < 2 * (MP + 4); k += 64) {
      const int x = k >= MP + 4, kk = x ? k - (MP + 4) : k;
      s_u.a.e2[x][kk] = (kk >= 1 && kk < M[x]) ? s_e[x][kk - 1] * s_e[x][kk - 1] : 0.0;
    }
    const double loA = block_reduce<1, OpMin>(win ? DBL_MAX : lo, s_red);
    const double hiA = block_reduce<1, OpMax>(win ? -DBL_MAX : hi, s_red);
    const double loB = block_reduce<1, OpMin>(fmin(win ? lo : DBL_MAX, lot), s_red);
    const double hiB = block_reduce<1, OpMax>(fmax(win ? hi : -DBL_MAX, hit), s_red);
    const double l2[2] = {loA, loB}, h2[2] = {hiA, hiB};
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      glo[x] = ghi[x] = btol[x] = 0.0;
      if (M[x] == 0) continue;
      const double pad = 2.0 * DBL_EPSILON * fmax(fabs(l2[x]), fabs(h2[x])) * M[x] + DBL_MIN;
      glo[x] = l2[x] - pad;
      ghi[x] = h2[x] + pad;
      btol[x] = CSS_BISECT_TOL * fmax(fabs(glo[x]), fabs(ghi[x])) + DBL_MIN;
    }
    for (int k = lane; k < 2 * (MP + 4); k += 64) {
      const int x = k >= MP + 4, kk = x ? k - (MP + 4) : k;
      if (kk >= M[x]) s_d[x][kk] = 2.0 * fabs(ghi[x]) + 2.0 * fabs(glo[x]) + 1.0;
    }
  }
  __syncthreads();
  p40_bisect(mA, mB, glo, ghi, btol, s_d, s_u.a.e2, s_lam, lane);
  __syncthreads();

  CSS_PROF(3);
  /* ---- eigenvectors of each T: two steps of inverse iteration (lanes 0..3) */
  if (lane < 4 && M[lane >> 1] > 0) {
    const int x = lane >> 1, e = lane & 1;
    invit_factor<MP>(M[x], e, s_d[x], s_e[x], s_lam[x], s_u.b.lu[x], s_x[x], s_u.b.piv[x], s_u.b.y[x]);
  }
  __syncthreads();
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const double tiny = DBL_EPSILON * fmax(fmax(fabs(glo[x]), fabs(ghi[x])), DBL_MIN);
    for (int k = lane; k < M[x]; k += 64) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double u0 = s_u.b.lu[x][e][0][k];
        s_u.b.lu[x][e][0][k] = fast_rcp(u0 == 0.0 ? tiny : u0);
      }
    }
  }
  double y1 = 0.0, y2 = 0.0, y1t = 0.0, y2t = 0.0;
#ifdef GD_CSS_SKIP_INVIT
  for (int itn = 0; itn < 0; ++itn) {
#else
  for (int itn = 0; itn < 2; ++itn) {
#endif
    __syncthreads();
    if (lane < 4 && M[lane >> 1] > 0) {
      const int x = lane >> 1;
      invit_solve<MP>(M[x], lane & 1, s_u.b.lu[x], s_x[x], s_u.b.piv[x], s_u.b.y[x]);
    }
    __syncthreads();
    y1 = rowk ? s_u.b.y[win][0][r] : 0.0;
    y2 = rowk ? s_u.b.y[win][1][r] : 0.0;
    y1t = trowk ? s_u.b.y[1][0][R] : 0.0;
    y2t = trowk ? s_u.b.y[1][1][R] : 0.0;
    double n1A = win ? 0.0 : y1 * y1, n2A = win ? 0.0 : y2 * y2;
    double n1B = (win ? y1 * y1 : 0.0) + (tq == 0 ? y1t * y1t : 0.0);
    double n2B = (win ? y2 * y2 : 0.0) + (tq == 0 ? y2t * y2t : 0.0);
    wave_sum2(n1A, n2A);
    wave_sum2(n1B, n2B);
    const double r1A = 1.0 / sqrt(n1A), r2A = 1.0 / sqrt(n2A), r1B = 1.0 / sqrt(n1B), r2B = 1.0 / sqrt(n2B);
    y1 *= win ? r1B : r1A;
    y2 *= win ? r2B : r2A;
    y1t *= r1B;
    y2t *= r2B;
    __syncthreads();
    if (itn == 0) {
      if (rowk) {
        s_u.b.y[win][0][r] = y1;
        s_u.b.y[win][1][r] = y2;
      }
      if (tq == 0 && trowk) {
        s_u.b.y[1][0][R] = y1t;
        s_u.b.y[1][1][R] = y2t;
      }
    }
  }
  /* orthogonalise the second vector against the first (close eigenvalues) */
  {
    double dA = win ? 0.0 : y1 * y2, dB = (win ? y1 * y2 : 0.0) + (tq == 0 ? y1t * y2t : 0.0);
    wave_sum2(dA, dB);
    const double dt = win ? dB : dA;
    y2 = fma(-dt, y1, y2);
    y2t = fma(-dB, y1t, y2t);
    double nA = win ? 0.0 : y2 * y2, nB = (win ? y2 * y2 : 0.0) + (tq == 0 ? y2t * y2t : 0.0);
    wave_sum2(nA, nB);
    const double rA = 1.0 / sqrt(nA), rB = 1.0 / sqrt(nB);
    y2 *= win ? rB : rA;
    y2t *= rB;
  }
  /* eigenvalues = Rayleigh quotients y^T T y of the unit vectors (k_css_mds) */
  {
    __syncthreads();
    if (rowk) {
      s_u.b.y[win][0][r] = y1;
      s_u.b.y[win][1][r] = y2;
    }
    if (tq == 0 && trowk) {
      s_u.b.y[1][0][R] = y1t;
      s_u.b.y[1][1][R] = y2t;
    }
    __syncthreads();
    double t1 = 0.0, t2 = 0.0, t1t = 0.0, t2t = 0.0;
    if (rowk) {
      const double *e = s_e[win], *dd = s_d[win];
      const double(*sy)[MP] = s_u.b.y[win];
      const double el = r > 0 ? e[r - 1] : 0.0, er = r + 1 < m_me ? e[r] : 0.0;
      const int il = r > 0 ? r - 1 : 0, ir = r + 1 < m_me ? r + 1 : r;
      t1 = y1 * (dd[r] * y1 + el * sy[0][il] + er * sy[0][ir]);
      t2 = y2 * (dd[r] * y2 + el * sy[1][il] + er * sy[1][ir]);
    }
    if (tq == 0 && trowk) {
      const double(*sy)[MP] = s_u.b.y[1];
      const double el = s_e[1][R - 1], er = R + 1 < mB ? s_e[1][R] : 0.0;
      const int il = R - 1, ir = R + 1 < mB ? R + 1 : R;
      t1t = y1t * (s_d[1][R] * y1t + el * sy[0][il] + er * sy[0][ir]);
      t2t = y2t * (s_d[1][R] * y2t + el * sy[1][il] + er * sy[1][ir]);
    }
    double a1 = win ? 0.0 : t1, a2 = win ? 0.0 : t2;
    double b1 = (win ? t1 : 0.0) + t1t, b2 = (win ? t2 : 0.0) + t2t;
    wave_sum2(a1, a2);
    wave_sum2(b1, b2);
    if (lane == 0) {
      s_lam[0][0] = fabs(a1) <= ztol[0] ? 0.0 : a1;
      s_lam[0][1] = fabs(a2) <= ztol[0] ? 0.0 : a2;
      s_lam[1][0] = fabs(b1) <= ztol[1] ? 0.0 : b1;
      s_lam[1][1] = fabs(b2) <= ztol[1] ? 0.0 : b2;
    }
    __syncthreads();
  }

  CSS_PROF(4);
  /* ---- back-transformation y <- H_0 H_1 ... H_{m-3} y per window */
#ifndef GD_CSS_SKIP_BACK
#pragma unroll
  for (int k = MP - 3; k >= 0; --k) {
    const bool liveA = k <= mA - 3, liveB = k <= mB - 3;
    if (liveA || liveB) {
      const bool mine = win ? liveB : liveA;
      const double vk = (rowk && mine) ? A[k] : 0.0;
      const double vkt = (trowk && liveB) ? s_tail[tr][k] : 0.0;
      const double tA = liveA ? s_tau[0][k] : 0.0, tB = liveB ? s_tau[1][k] : 0.0;
      double d1A = win ? 0.0 : vk * y1, d2A = win ? 0.0 : vk * y2;
      double d1B = (win ? vk * y1 : 0.0) + (tq == 0 ? vkt * y1t : 0.0);
      double d2B = (win ? vk * y2 : 0.0) + (tq == 0 ? vkt * y2t : 0.0);
      wave_sum2(d1A, d2A);
      wave_sum2(d1B, d2B);
      const double t = win ? tB : tA, d1 = win ? d1B : d1A, d2 = win ? d2B : d2A;
      y1 = fma(-(t * d1), vk, y1);
      y2 = fma(-(t * d2), vk, y2);
      y1t = fma(-(tB * d1B), vkt, y1t);
      y2t = fma(-(tB * d2B), vkt, y2t);
      asm volatile("" ::: "memory"); /* one s_tau load in flight, not MP */
    }
  }
#endif

  CSS_PROF(5);
  /* ---- X = Q sqrt(L) (css.c:545-556), then calc_dist + css on identity groups */
  {
    const double L1A = sqrt(s_lam[0][0]), L2A = sqrt(s_lam[0][1]);
    const double L1B = sqrt(s_lam[1][0]), L2B = sqrt(s_lam[1][1]);
    __syncthreads();
    if (rowk) {
      const double L1 = win ? L1B : L1A, L2 = win ? L2B : L2A;
      s_x[win][2 * r] = y1 * L1 + y2 * 0.0;
      s_x[win][2 * r + 1] = y1 * 0.0 + y2 * L2;
    }
    if (tq == 0 && trowk) {
      s_x[1][2 * R] = y1t * L1B + y2t * 0.0;
      s_x[1][2 * R + 1] = y1t * 0.0 + y2t * L2B;
    }
    __syncthreads();
  }
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    if (M[x] == 0) continue;
    const double *X = s_x[x];
    const double score = css_score<1>(s_tr, Aa[x], Bb[x], [&](int p, int q) { return xdist(X, p, q); }, s_red);
    if (score == -1.0) continue; /* the reference's "discarded" marker (css.c:127) */
    const gd_chrom_dev &d = ch[C[x]];
    const int64_t wl = W[x] - d.w_base;
    if (lane == 0) {
      scores[d.w_out + wl] = score;
      if (!want_x) pvals[d.w_out + wl] = 1.0; /* runs == 0: p = (0 + 1) / (0 + 1) */
    }
    if (want_x) {
      for (int e = lane; e < 2 * MP; e += 64) xbuf[W[x] * 2 * MP + e] = (e < 2 * M[x]) ? X[e] : 0.0;
      if (lane == 0) status[W[x]] = 1;
    }
  }
  CSS_PROF(6);
}

/* ------------------------------------------------------------------------ */
/* The 25..40-individual tier with one window per HALF wave (k_css_mds_h40).  */
/* Window h = lane / 32 keeps its rows 0..31 in the half's lanes (40 columns     */
/* each) and its rows 32..39 in LDS, each worked by a lane quad over interleaved */
/* columns.  The two windows are symmetric, so every per-window quantity is a    */
/* per-lane value: one set of Householder scalars serves both windows, and the   */
/* step's two sums (|x|^2 and r^T A r) are all-reduced within each half by four  */
/* DPP stages and one v_permlane16_swap -- k_css_mds_p40 (window B split over    */
/* lanes and LDS) paid two full-wave reductions, two scalar recurrences and a    */
/* select per quantity for the same two windows.                                */
/* ------------------------------------------------------------------------ */
namespace {
constexpr int H40_MAIN = 32, H40_TS = 10, H40_TSTRIDE = 44; /* rows in VGPRs, tail columns per lane, tail row stride */

/* sums over each 32-lane half, every lane of a half holding the same bits (every stage
 * adds a lane to its mirror image, and IEEE addition commutes) */
/* a half-uniform value of lane L of each half (L wave-uniform) */
__device__ __forceinline__ double half_lane(double v, int L, bool h) {
  const double v0 = readlane_f64(v, L), v1 = readlane_f64(v, 32 + L);
  return h ? v1 : v0;
}
/* the same through the LDS crossbar: two ds_bpermute from lane (lane & 32) + L, no VALU but the
 * address (k_css_mds_h40 is VALU-bound: four readlanes, two moves and two selects per value
 * cost more than the LDS latency, which the half-wave sums beside these reads cover) */
__device__ __forceinline__ double half_bperm(double v, int L, int lane) {
  const int addr = ((lane & 32) + L) << 2;
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(u >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

template <int K>
__device__ __forceinline__ void h40_step(double (&A)[P40], const int (&M)[2], double (*s_row)[P40 + 2],
                                         double (*s_v)[P40], double (*s_w)[P40], double (*s_d)[P40 + 4],
                                         double (*s_e)[P40], double (*s_tau)[P40],
                                         double (*s_tail)[8][H40_TSTRIDE]) {
  constexpr int MP = P40;
  const int lane = css_lane_now();
  const bool h = lane >= 32;
  const int hi = h ? 1 : 0, r = lane & 31;
  const int tr = r >> 2, tq = lane & 3, R = H40_MAIN + tr;
  const int mine = h ? M[1] : M[0];
  const bool row = r < mine, trow = R < mine;
  __syncthreads();
  /* publish row K of each window (zeros at j <= K) and its diagonal */
  if constexpr (K < H40_MAIN) {
    if (r == K) {
      double *dst = s_row[hi];
#pragma unroll
      for (int jb = 0; jb < MP / 8; ++jb)
        if (8 * jb + 7 >= K) {
#pragma unroll
          for (int u = 0; u < 8; u += 2) {
            const int j = 8 * jb + u;
            *reinterpret_cast<double2 *>(dst + j) = make_double2(j > K ? A[j] : 0.0, j + 1 > K ? A[j + 1] : 0.0);
          }
        }
      s_d[hi][K] = A[K];
    }
  } else {
    const double *src = s_tail[hi][K - H40_MAIN];
    s_row[hi][r] = r > K ? src[r] : 0.0;
    if (r < MP - H40_MAIN) s_row[hi][H40_MAIN + r] = H40_MAIN + r > K ? src[H40_MAIN + r] : 0.0;
    if (r == 0) s_d[hi][K] = src[K];
  }
  __syncthreads();
  if constexpr (K >= MP - 2) {
    if (r == 0 && K == mine - 2) s_e[hi][K] = s_row[hi][K + 1];
    return;
  } else {
    const double *srw = s_row[hi];
    const double xi = (r > K + 1 && row) ? srw[r] : 0.0;
    double p0 = 0, p1 = 0;
#pragma unroll
    for (int jb = 0; jb < MP / 8; ++jb) {
      if (8 * jb + 7 > K) {
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
          if (8 * jb + u > K) p0 = fma(A[8 * jb + u], srw[8 * jb + u], p0);
          if (8 * jb + u + 1 > K) p1 = fma(A[8 * jb + u + 1], srw[8 * jb + u + 1], p1);
        }
        CSS_PIN(p0);
        CSS_PIN(p1);
      }
    }
    const double ak1 = A[K + 1];
    const double praw = p0 + p1;
    /* the tail row over the live column groups (s_row is 0 at j <= K) */
    const double *trw = s_tail[hi][tr];
    double t0 = 0, t1 = 0;
#pragma unroll
    for (int s = 0; s < H40_TS; ++s) {
      if (4 * s + 3 > K) {
        const int j = 4 * s + tq;
        if (s & 1)
          t1 = fma(trw[j], srw[j], t1);
        else
          t0 = fma(trw[j], srw[j], t0);
      }
    }
    const double pt = quad_sum(t0 + t1);
    const double akt = trw[K + 1];
    const double xr = (R > K + 1 && trow) ? srw[R] : 0.0;
    /* |x|^2 and r^T A r of each window, all-reduced within its half */
    double sig = xi * xi + (tq == 0 ? xr * xr : 0.0);
    double q = ((r > K && row) ? srw[r] : 0.0) * praw + ((tq == 0 && R > K && trow) ? srw[R] * pt : 0.0);
    half_sum2(sig, q);
    double pr1, a11;
    if constexpr (K + 1 < H40_MAIN) {
      pr1 = half_lane(praw, K + 1, h);
      a11 = half_lane(ak1, K + 1, h);
    } else {
      pr1 = half_lane(pt, 4 * (K + 1 - H40_MAIN), h);
      a11 = half_lane(akt, 4 * (K + 1 - H40_MAIN), h);
    }
    double tau, beta, scale, Kc;
    hh_scalars(srw[K + 1], sig, q, pr1, a11, &tau, &beta, &scale, &Kc);
    const double vi = (r == K + 1) ? 1.0 : xi * scale;
    const double pi = (r > K && row) ? (tau * scale) * fma(-beta, ak1, praw) : 0.0;
    const double wi = fma(Kc, vi, pi);
    const double vt = (R == K + 1) ? 1.0 : xr * scale;
    const double ptl = (R > K && trow) ? (tau * scale) * fma(-beta, akt, pt) : 0.0;
    const double wt = fma(Kc, vt, ptl);
    if (r == 0) {
      s_e[hi][K] = beta;
      s_tau[hi][K] = tau;
    }
    s_v[hi][r] = vi;
    s_w[hi][r] = wi;
    if (tq == 0) {
      s_v[hi][R] = vt;
      s_w[hi][R] = wt;
    }
    __syncthreads();
    const double *sv = s_v[hi], *sw = s_w[hi];
#pragma unroll
    for (int jb = 0; jb < MP / 8; ++jb) {
      if (8 * jb + 7 > K) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = 8 * jb + u;
          if (j > K) A[j] = fma(-vi, sw[j], fma(-wi, sv[j], A[j]));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) CSS_PIN(A[8 * jb + u]);
      }
    }
    A[K] = vi; /* stash v_K in the dead column K */
    double *tw = s_tail[hi][tr];
#pragma unroll
    for (int s = 0; s < H40_TS; ++s) {
      if (4 * s + 3 > K) {
        const int j = 4 * s + tq;
        tw[j] = fma(-vt, sw[j], fma(-wt, sv[j], tw[j]));
      }
    }
    if (tq == (K & 3)) tw[K] = vt;
  }
}

template <int K>
struct H40Steps {
  static __device__ __forceinline__ void run(double (&A)[P40], const int (&M)[2], double (*s_row)[P40 + 2],
                                             double (*s_v)[P40], double (*s_w)[P40], double (*s_d)[P40 + 4],
                                             double (*s_e)[P40], double (*s_tau)[P40],
                                             double (*s_tail)[8][H40_TSTRIDE]) {
    if ((K & 7) == 0 && K >= M[0] && K >= M[1]) return; /* exits only at block boundaries (hh_step_static) */
    h40_step<K>(A, M, s_row, s_v, s_w, s_d, s_e, s_tau, s_tail);
    H40Steps<K + 1>::run(A, M, s_row, s_v, s_w, s_d, s_e, s_tau, s_tail);
  }
};
template <>
struct H40Steps<P40> {
  static __device__ __forceinline__ void run(double (&)[P40], const int (&)[2], double (*)[P40 + 2], double (*)[P40],
                                             double (*)[P40], double (*)[P40 + 4], double (*)[P40], double (*)[P40],
                                             double (*)[8][H40_TSTRIDE]) {}
};

/* The fused Householder step of k_css_mds_t80 on each half wave (CSS_H40_FUSED): row K of
 * each window is read as column K -- every lane carries its own entry of it and p = A r from
 * the previous pass (H40Carry) --, so a step is one half-wave sum, the scalars, one LDS round
 * trip of (v_i, w_i) and the next column, and one pass over the row that applies the rank-2
 * update and accumulates the next step's p.  The unfused h40_step publishes row K from one
 * lane first and takes two LDS round trips and two passes. */
struct H40Carry {
  double r, p, rt, pt; /* column K entry and p_i of this lane's main row and tail row */
};

template <int K>
__device__ __forceinline__ void h40_fused_pass(double (&A)[P40], double vi, double wi, double vt, double wt,
                                               const double2 *s_vw, const double *s_r,
                                               double (*s_tail)[H40_TSTRIDE], H40Carry &c) {
  constexpr int MP = P40;
  const int lane = css_lane_now(), tr = (lane & 31) >> 2, tq = lane & 3;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#ifndef H40_FB
#define H40_FB 4
#endif
  constexpr int FB = H40_FB; /* columns per pinned group */
  constexpr int NB = MP / FB, JB0 = (K + 1) / FB;
  double2 cvw[FB];
  double cr[FB];
#pragma unroll
  for (int u = 0; u < FB; ++u) {
    cvw[u] = s_vw[FB * JB0 + u];
    cr[u] = s_r[FB * JB0 + u];
  }
#pragma unroll
  for (int jb = JB0; jb < NB; ++jb) {
    double2 nvw[FB];
    double nr[FB];
    if (jb + 1 < NB) {
#pragma unroll
      for (int u = 0; u < FB; ++u) {
        nvw[u] = s_vw[FB * (jb + 1) + u];
        nr[u] = s_r[FB * (jb + 1) + u];
      }
    }
#pragma unroll
    for (int u = 0; u < FB; ++u) {
      const int j = FB * jb + u;
      if (j > K) A[j] = fma(-vi, cvw[u].y, fma(-wi, cvw[u].x, A[j]));
    }
#pragma unroll
    for (int u = 0; u < FB; ++u) CSS_PIN(A[FB * jb + u]);
#pragma unroll
    for (int u = 0; u < FB; ++u) {
      const int j = FB * jb + u;
      if (j > K + 1) p[u & 3] = fma(A[j], cr[u], p[u & 3]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) CSS_PIN(p[u]);
    if (jb + 1 < NB) {
#pragma unroll
      for (int u = 0; u < FB; ++u) {
        cvw[u] = nvw[u];
        cr[u] = nr[u];
      }
    }
  }
  A[K] = vi; /* stash v_K in the dead column K */
  double *tw = s_tail[tr];
  double t0 = 0.0, t1 = 0.0;
#pragma unroll
  for (int s = 0; s < H40_TS; ++s) {
    if (4 * s + 3 > K) { /* v_j = w_j = 0 at j <= K: the dead columns stay */
      const int j = 4 * s + tq;
      const double2 vw = s_vw[j];
      const double t = fma(-vt, vw.y, fma(-wt, vw.x, tw[j]));
      tw[j] = t;
      if (s & 1)
        t1 = fma(t, s_r[j], t1);
      else
        t0 = fma(t, s_r[j], t0);
    }
  }
  if (tq == (K & 3)) tw[K] = vt;
  c.p = (p[0] + p[1]) + (p[2] + p[3]);
  c.pt = quad_sum(t0 + t1);
}

/* column 0 and p = A r before step 0 */
__device__ __forceinline__ void h40_fused_start(const double (&A)[P40], double (*s_r)[P40 + 2], double (*s_d)[P40 + 4],
                                                double (*s_tail)[8][H40_TSTRIDE], H40Carry &c) {
  constexpr int MP = P40;
  const int lane = css_lane_now(), hi = lane >> 5, r = lane & 31, tr = r >> 2, tq = lane & 3, R = H40_MAIN + tr;
  c.r = A[0];
  c.rt = s_tail[hi][tr][0];
  __syncthreads();
  s_r[hi][r] = r > 0 ? c.r : 0.0;
  if (tq == 0) s_r[hi][R] = c.rt;
  if (r == 0) s_d[hi][0] = c.r;
  __syncthreads();
  const double *sr = s_r[hi];
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 1; j < MP; ++j) {
    p[j & 3] = fma(A[j], sr[j], p[j & 3]);
    if ((j & 7) == 7) {
#pragma unroll
      for (int u = 0; u < 4; ++u) CSS_PIN(p[u]);
    }
  }
  const double *trw = s_tail[hi][tr];
  double t0 = 0.0, t1 = 0.0;
#pragma unroll
  for (int s = 0; s < H40_TS; ++s) {
    const int j = 4 * s + tq;
    if (s & 1)
      t1 = fma(trw[j], sr[j], t1);
    else
      t0 = fma(trw[j], sr[j], t0);
  }
  c.p = (p[0] + p[1]) + (p[2] + p[3]);
  c.pt = quad_sum(t0 + t1);
}

/* One fused step K <= MP - 3 of both windows (hh_step_static's arithmetic, per half) */
template <int K>
__device__ __forceinline__ void h40_fstep(double (&A)[P40], const int (&M)[2], H40Carry &c, double2 (*s_vw)[P40],
                                          double (*s_r)[P40 + 2], double (*s_d)[P40 + 4], double (*s_e)[P40],
                                          double (*s_tau)[P40], double (*s_tail)[8][H40_TSTRIDE]) {
  const int lane = css_lane_now();
  const bool h = lane >= 32;
  const int hi = h ? 1 : 0, r = lane & 31, tr = r >> 2, tq = lane & 3, R = H40_MAIN + tr;
  /* rows >= m of a window are zero and stay zero (their v, w, r and p are zero, k_css_mds_t80):
   * only the rows the earlier steps finished (<= K) need masking */
  const double xi = (r > K + 1) ? c.r : 0.0;
  const double xr = (R > K + 1) ? c.rt : 0.0;
  /* |x|^2 and r^T A r of each window in one half-wave sum; a tail row counts once */
  double sigma = xi * xi + (tq == 0 ? xr * xr : 0.0);
  double q = ((r > K) ? c.r * c.p : 0.0) + ((tq == 0 && R > K) ? c.rt * c.pt : 0.0);
  half_sum2(sigma, q);
  double alpha, pr1, a11;
#if H40_BPERM
  if constexpr (K + 1 < H40_MAIN) {
    alpha = half_bperm(c.r, K + 1, lane);
    pr1 = half_bperm(c.p, K + 1, lane);
    a11 = half_bperm(A[K + 1], K + 1, lane);
  } else {
    alpha = half_bperm(c.rt, 4 * (K + 1 - H40_MAIN), lane);
    pr1 = half_bperm(c.pt, 4 * (K + 1 - H40_MAIN), lane);
    a11 = s_tail[hi][K + 1 - H40_MAIN][K + 1];
  }
#else
  if constexpr (K + 1 < H40_MAIN) {
    alpha = half_lane(c.r, K + 1, h);
    pr1 = half_lane(c.p, K + 1, h);
    a11 = half_lane(A[K + 1], K + 1, h);
  } else {
    alpha = half_lane(c.rt, 4 * (K + 1 - H40_MAIN), h);
    pr1 = half_lane(c.pt, 4 * (K + 1 - H40_MAIN), h);
    a11 = s_tail[hi][K + 1 - H40_MAIN][K + 1];
  }
#endif
  double tau, beta, scale, Kc;
  hh_scalars(alpha, sigma, q, pr1, a11, &tau, &beta, &scale, &Kc);
  const double ak1 = A[K + 1];
  const double vi = (r == K + 1) ? 1.0 : xi * scale;
  const double pi = (r > K) ? (tau * scale) * fma(-beta, ak1, c.p) : 0.0;
  const double wi = fma(Kc, vi, pi);
  const double akt = s_tail[hi][tr][K + 1];
  const double vt = (R == K + 1) ? 1.0 : xr * scale;
  const double ptl = (R > K) ? (tau * scale) * fma(-beta, akt, c.pt) : 0.0;
  const double wt = fma(Kc, vt, ptl);
#if H40_BPERM
  /* w at row K + 1 as that lane forms it (v = 1 there, p from the scalars): the same bits */
  const double wk1 = fma(Kc, 1.0, (tau * scale) * fma(-beta, a11, pr1));
#else
  double wk1;
  if constexpr (K + 1 < H40_MAIN)
    wk1 = half_lane(wi, K + 1, h);
  else
    wk1 = half_lane(wt, 4 * (K + 1 - H40_MAIN), h);
#endif
  /* column K + 1 after this step (the update's formula at v_{K+1} = 1) */
  const double rn = fma(-vi, wk1, fma(-wi, 1.0, ak1));
  const double rnt = fma(-vt, wk1, fma(-wt, 1.0, akt));
  __syncthreads();
  if (r == 0) {
    s_e[hi][K] = beta;
    s_tau[hi][K] = tau;
  }
  s_vw[hi][r] = make_double2(vi, wi);
  s_r[hi][r] = r > K + 1 ? rn : 0.0;
  if (tq == 0) {
    s_vw[hi][R] = make_double2(vt, wt);
    s_r[hi][R] = R > K + 1 ? rnt : 0.0;
  }
  if constexpr (K + 1 < H40_MAIN) {
    if (r == K + 1) s_d[hi][K + 1] = rn;
  } else {
    if (r == 4 * (K + 1 - H40_MAIN)) s_d[hi][K + 1] = rnt;
  }
  __syncthreads();
  h40_fused_pass<K>(A, vi, wi, vt, wt, s_vw[hi], s_r[hi], s_tail[hi], c);
  c.r = rn;
  c.rt = rnt;
}

template <int K>
struct H40FSteps {
  static __device__ __forceinline__ void run(double (&A)[P40], const int (&M)[2], H40Carry &c, double2 (*s_vw)[P40],
                                             double (*s_r)[P40 + 2], double (*s_d)[P40 + 4], double (*s_e)[P40],
                                             double (*s_tau)[P40], double (*s_tail)[8][H40_TSTRIDE]) {
    if ((K & 7) == 0 && K >= M[0] && K >= M[1]) return; /* exits only at block boundaries (hh_step_static) */
    if constexpr (K <= P40 - 3) {
      h40_fstep<K>(A, M, c, s_vw, s_r, s_d, s_e, s_tau, s_tail);
      H40FSteps<K + 1>::run(A, M, c, s_vw, s_r, s_d, s_e, s_tau, s_tail);
    } else {
      /* K = MP - 2: no reflector; e_{MP-2} = column MP - 2 at row MP - 1, d_{MP-1} */
      const int lane = css_lane_now();
      const bool h = lane >= 32;
      const int hi = h ? 1 : 0, r = lane & 31, mine = h ? M[1] : M[0];
      const double e = half_lane(c.rt, 4 * (P40 - 1 - H40_MAIN), h);
      __syncthreads();
      if (r == 0) {
        if (K == mine - 2) s_e[hi][K] = e;
        s_d[hi][K + 1] = s_tail[hi][P40 - 1 - H40_MAIN][P40 - 1];
      }
    }
  }
};
}  // namespace

__global__ void __launch_bounds__(64, CSS_P40_WAVES)
    k_css_mds_h40(const gd_chrom_dev *ch, int nchrom, const gd_css_planes *pl, const uint32_t *planes,
                  const int32_t *lo_a_, const int32_t *hi_a_, const int32_t *lo_b_, const double *avals,
                  const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *pvals,
                  double *xbuf, uint8_t *status, unsigned *flags) {
  constexpr int MP = P40;
  __shared__ __attribute__((aligned(16))) double s_tail[2][8][H40_TSTRIDE];
  /* the phase buffers share one region (12 workgroups per CU: <= 13.6 KB in all): the
   * distance build's masks / values and the Householder steps' row, v, w never live at once;
   * the pivoted-LU fallback holds one eigenvector's factors at a time */
  __shared__ __attribute__((aligned(16))) union {
    struct {
      double e2[2][MP + 4]; /* bisection only (after the Householder steps) */
      union {
        struct {
          uint64_t mask[2][2 * MP];
          double vals[2][MP];
        };
        struct {
          double row[2][MP + 2];
          double v[2][MP], w[2][MP];
        };
      };
    } a;
    struct {
      double lu[2][1][3][MP];
      double y[2][2][MP]; /* [window][slot 0: the solve, slot 1: the first eigenvector] */
      uint8_t piv[2][1][MP];
    } b;
    struct {
      double e2[2][MP + 4]; /* = a.e2: the twisted factorisations read it */
      double Q[2][2][2][MP];
    } c;
  } s_u;
  __shared__ __attribute__((aligned(16))) double s_d[2][MP + 4];
  __shared__ double s_e[2][MP], s_tau[2][MP];
  __shared__ double s_x[2][2 * MP];
  __shared__ double s_lam[2][2];

  const int lane = threadIdx.x;
  const bool h = lane >= 32;
  const int hi = h ? 1 : 0, r = lane & 31;
  const int tr = r >> 2, tq = lane & 3, R = H40_MAIN + tr;

  /* the two windows' bookkeeping (uniform) */
  int64_t W[2];
  int C[2], Aa[2], Bb[2], M[2], npos[2];
  int32_t LA[2], LB[2];
  bool lit[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    W[x] = 2 * (int64_t)blockIdx.x + x;
    M[x] = 0;
    C[x] = 0;
    Aa[x] = Bb[x] = 1;
    npos[x] = 0;
    LA[x] = LB[x] = 0;
    lit[x] = false;
    if (W[x] >= wtotal) continue;
    const int c = chrom_of(ch, nchrom, W[x]);
    const gd_chrom_dev &d = ch[c];
    const int a = d.asize, b = d.bsize, m = a + b;
    const int32_t la = lo_a_[W[x]], ha = hi_a_[W[x]], lb = lo_b_[W[x]];
    const int np = (ha - la) / a;
    if (np <= 0) continue;
    if ((int64_t)lb + (int64_t)np * b > d.blen) {
      if (lane == 0) atomicOr(flags, GD_FLAG_B_BOUNDS);
      continue;
    }
    if (m > MP) {
      if (lane == 0) atomicOr(flags, GD_FLAG_BAD_SIZE);
      continue;
    }
    C[x] = c;
    Aa[x] = a;
    Bb[x] = b;
    M[x] = m;
    npos[x] = np;
    LA[x] = la;
    LB[x] = lb;
    lit[x] = force_literal || (la % a) != 0 || (lb % b) != 0;
  }
  if (M[0] == 0 && M[1] == 0) return;
  CSS_PROF_INIT;

  /* ---- regular windows?  (k_css_mds) */
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    if (M[x] == 0 || lit[x]) continue;
    const gd_css_planes P = pl[C[x]];
    const int a = Aa[x], b = Bb[x];
    const int64_t ra = LA[x] / a, rb = LB[x] / b;
    int irr = 0;
    for (int k = lane; k * 64 < npos[x]; k += 64) {
      const int nb = min(64, npos[x] - 64 * k);
      const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
      const uint64_t xa = plane_bits64(planes + P.pa + (int64_t)(2 * a) * P.wa, ra + 64 * k) & tail;
      const uint64_t xb = plane_bits64(planes + P.pb + (int64_t)(2 * b) * P.wb, rb + 64 * k) & tail;
      irr |= (xa | xb) != 0;
    }
    lit[x] = __syncthreads_or(irr);
  }

  /* ---- compare_all: main row r of window h in A, its tail row R into s_tail[h] */
  const int mm = (h ? M[1] : M[0]);
  const bool row = r < mm, trow = R < mm;
  double A[MP];
  {
    int acc[MP], acct[H40_TS];
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) acc[jj] = 0;
#pragma unroll
    for (int s = 0; s < H40_TS; ++s) acct[s] = 0;
    const bool popA = M[0] > 0 && !lit[0], popB = M[1] > 0 && !lit[1];
    const int nk = max(popA ? (npos[0] + 63) >> 6 : 0, popB ? (npos[1] + 63) >> 6 : 0);
    for (int k = 0; k < nk; ++k) {
      __syncthreads();
      for (int idx = lane; idx < 2 * MP; idx += 64) {
        const int x = idx >= MP, rr = x ? idx - MP : idx;
        uint64_t Pm = 0, Nm = 0;
        if ((x ? popB : popA) && rr < M[x] && 64 * k < npos[x]) {
          const gd_css_planes P = pl[C[x]];
          const int a = Aa[x], b = Bb[x];
          const int nb = min(64, npos[x] - 64 * k);
          const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
          const uint32_t *base = rr < a ? planes + P.pa + (int64_t)(2 * rr) * P.wa
                                        : planes + P.pb + (int64_t)(2 * (rr - a)) * P.wb;
          const int64_t nw = rr < a ? P.wa : P.wb;
          const int64_t r0 = (rr < a ? LA[x] / a : LB[x] / b) + 64 * k;
          Pm = plane_bits64(base, r0) & tail;
          Nm = plane_bits64(base + nw, r0) & tail;
        }
        s_u.a.mask[x][2 * rr] = Pm;
        s_u.a.mask[x][2 * rr + 1] = Nm;
      }
      __syncthreads();
      const uint64_t *mk = s_u.a.mask[hi];
      const uint64_t Pi = mk[2 * r], Ni = mk[2 * r + 1];
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) {
        acc[jj] += __popcll(Pi & mk[2 * jj + 1]) + __popcll(Ni & mk[2 * jj]);
        if ((jj & 7) == 7) {
#pragma unroll
          for (int u = jj - 7; u <= jj; ++u) CSS_PIN(acc[u]);
        }
      }
      const uint64_t Pt = mk[2 * R], Nt = mk[2 * R + 1];
#pragma unroll
      for (int s = 0; s < H40_TS; ++s) {
        const int j = 4 * s + tq;
        acct[s] += __popcll(Pt & mk[2 * j + 1]) + __popcll(Nt & mk[2 * j]);
      }
    }
    /* literal windows: the reference predicate per SNP (k_css_mds) */
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      if (M[x] == 0 || !lit[x]) continue;
      const gd_chrom_dev &d = ch[C[x]];
      const int a = Aa[x], b = Bb[x], m = M[x];
      const double *av = avals + d.a_off + LA[x], *bv = bvals + d.b_off + LB[x];
      for (int k = 0; k < npos[x]; ++k) {
        __syncthreads();
        for (int rr = lane; rr < m; rr += 64)
          s_u.a.vals[x][rr] = rr < a ? av[(int64_t)k * a + rr] : bv[(int64_t)k * b + (rr - a)];
        __syncthreads();
        const double *sv = s_u.a.vals[x];
        int io = r, ro = R, mo = m, ao = a;
        CSS_OPAQUE_V(io);
        CSS_OPAQUE_V(ro);
        CSS_OPAQUE_S(mo);
        CSS_OPAQUE_S(ao);
        if (hi == x) {
          const double vi = sv[io];
#pragma unroll
          for (int jj = 0; jj < MP; ++jj) {
            if (jj < mo) {
              const double vj = sv[jj];
              const bool cast_i = ((io < ao) == (jj < ao)) ? (io > jj) : (io < ao);
              const double prod = cast_i ? x86_int(vi) * vj : x86_int(vj) * vi;
              acc[jj] += prod == -9.0;
            }
          }
          const double vr = sv[ro];
#pragma unroll
          for (int s = 0; s < H40_TS; ++s) {
            const int j = 4 * s + tq;
            if (j < mo) {
              const double vj = sv[j];
              const bool cast_r = ((ro < ao) == (j < ao)) ? (ro > j) : (ro < ao);
              const double prod = cast_r ? x86_int(vr) * vj : x86_int(vj) * vr;
              acct[s] += prod == -9.0;
            }
          }
        }
      }
    }
    int mo = mm;
    CSS_OPAQUE_V(mo);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) A[jj] = (row && jj < mo) ? (double)acc[jj] : 0.0;
#pragma unroll
    for (int s = 0; s < H40_TS; ++s) {
      const int j = 4 * s + tq;
      s_tail[hi][tr][j] = (trow && j < mo) ? (double)acct[s] : 0.0;
    }
  }

  CSS_PROF(0);
  /* ---- fill_averages per window (k_css_mds) */
  double avg;
  {
    /* the entries are exact integer counts, zero outside the window's m x m (masked above):
     * "< 1e-5" is "== 0", so the valid sum is the plain sum and the count of nonzero
     * entries the sum of min(v, 1) -- no per-entry branch (k_css_mds_t80) */
    double s4[2] = {0.0, 0.0}, n4[2] = {0.0, 0.0};
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) {
      s4[jj & 1] += A[jj];
      n4[jj & 1] += fmin(A[jj], 1.0);
    }
#pragma unroll
    for (int s = 0; s < H40_TS; ++s) {
      const double t = s_tail[hi][tr][4 * s + tq];
      s4[s & 1] += t;
      n4[s & 1] += fmin(t, 1.0);
    }
    double nz = n4[0] + n4[1], ss = s4[0] + s4[1];
    half_sum2(nz, ss); /* sums of integers: exact in any order */
    const double n2[2] = {readlane_f64(nz, 0), readlane_f64(nz, 32)};
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int tot = M[x] * M[x];
      if (M[x] != 0 && tot - (int)n2[x] > tot / 2) M[x] = 0; /* discarded window: outputs untouched */
    }
    avg = mm > 0 ? ss / (mm * mm) : 0.0;
  }
  if (M[0] == 0 && M[1] == 0) return;
  const int m_me = (h ? M[1] : M[0]);
  const bool rowk = r < m_me, trowk = R < m_me; /* rows of windows still alive */
  {
    CSS_OPAQUE_ROW(A);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) A[jj] = fma(avg, 1.0 - fmin(A[jj], 1.0), A[jj]);
#pragma unroll
    for (int s = 0; s < H40_TS; ++s) {
      double *t = &s_tail[hi][tr][4 * s + tq];
      *t = fma(avg, 1.0 - fmin(*t, 1.0), *t);
    }
  }

  /* ---- B = -1/2 Z (D o D) Z per window by double centering */
  double ztol[2];
  {
    double rs = 0, rst = 0;
    int mo = m_me;
    CSS_OPAQUE_V(mo);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) {
      A[jj] = (rowk && jj < mo) ? A[jj] * A[jj] : 0.0;
      rs += A[jj];
    }
#pragma unroll
    for (int s = 0; s < H40_TS; ++s) {
      const int j = 4 * s + tq;
      double *t = &s_tail[hi][tr][j];
      const double sq = (trowk && j < mo) ? *t * *t : 0.0;
      *t = sq;
      rst += sq;
    }
    rst = quad_sum(rst);
    const double ri = rowk ? rs / m_me : 0.0, rt = trowk ? rst / m_me : 0.0;
    __syncthreads();
    s_u.a.v[hi][r] = ri;
    if (tq == 0) s_u.a.v[hi][R] = rt;
    double g = ri + (tq == 0 ? rt : 0.0), dummy = 0.0;
    half_sum2(g, dummy);
    g = m_me > 0 ? g / m_me : 0.0;
    __syncthreads();
    const double *sv = s_u.a.v[hi];
    CSS_OPAQUE_V(mo);
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) {
      A[jj] = (rowk && jj < mo) ? -0.5 * ((A[jj] - (ri + sv[jj])) + g) : 0.0;
      if ((jj & 7) == 7) {
#pragma unroll
        for (int u = jj - 7; u <= jj; ++u) CSS_PIN(A[u]);
      }
    }
    double f2 = 0;
#pragma unroll
    for (int jj = 0; jj < MP; ++jj) f2 = fma(A[jj], A[jj], f2);
#pragma unroll
    for (int s = 0; s < H40_TS; ++s) {
      const int j = 4 * s + tq;
      double *t = &s_tail[hi][tr][j];
      const double cv = (trowk && j < mo) ? -0.5 * ((*t - (rt + sv[j])) + g) : 0.0;
      *t = cv;
      f2 = fma(cv, cv, f2);
    }
    double dm2 = 0.0;
    half_sum2(f2, dm2);
    /* eigenvalues within rounding of 0 count as 0 (oracle/css_oracle.c, cmds) */
    ztol[0] = 64.0 * M[0] * DBL_EPSILON * sqrt(readlane_f64(f2, 0));
    ztol[1] = 64.0 * M[1] * DBL_EPSILON * sqrt(readlane_f64(f2, 32));
  }

  CSS_PROF(1);
  /* ---- Householder tridiagonalisation of both windows (LAPACK dsytd2, lower) */
#ifndef GD_CSS_SKIP_TRIDIAG
#if CSS_H40_FUSED
  {
    /* (v_j, w_j) pairs over s_u.a.v / w (contiguous, 16-B aligned), column K + 1 over s_u.a.row */
    double2(*s_vw)[MP] = reinterpret_cast<double2(*)[MP]>(&s_u.a.v[0][0]);
    H40Carry cr;
    h40_fused_start(A, s_u.a.row, s_d, s_tail, cr);
    H40FSteps<0>::run(A, M, cr, s_vw, s_u.a.row, s_d, s_e, s_tau, s_tail);
  }
#else
  H40Steps<0>::run(A, M, s_u.a.row, s_u.a.v, s_u.a.w, s_d, s_e, s_tau, s_tail);
#endif
#endif
  __syncthreads();

  CSS_PROF(2);
  /* ---- the two largest eigenvalues of each T */
  double glo[2], ghi[2], btol[2];
  {
    double lo = DBL_MAX, hi_ = -DBL_MAX;
    const double *e = s_e[hi];
    if (rowk) {
      const double rr = (r > 0 ? fabs(e[r - 1]) : 0.0) + (r < m_me - 1 ? fabs(e[r]) : 0.0);
      lo = s_d[hi][r] - rr;
      hi_ = s_d[hi][r] + rr;
    }
    if (tq == 0 && trowk) {
      const double rr = fabs(e[R - 1]) + (R < m_me - 1 ? fabs(e[R]) : 0.0);
      lo = fmin(lo, s_d[hi][R] - rr);
      hi_ = fmax(hi_, s_d[hi][R] + rr);
    }
    for (int k = lane; k < 2 * (MP + 4); k += 64) {
      const int x = k >= MP + 4, kk = x ? k - (MP + 4) : k;
      s_u.a.e2[x][kk] = (kk >= 1 && kk < M[x]) ? fmax(s_e[x][kk - 1] * s_e[x][kk - 1], CSS_E2_FLOOR) : 0.0;
    }
    double nlo = -lo; /* min as a max */
    half_reduce2<OpMax>(nlo, hi_);
    const double l2[2] = {-readlane_f64(nlo, 0), -readlane_f64(nlo, 32)};
    const double h2[2] = {readlane_f64(hi_, 0), readlane_f64(hi_, 32)};
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      glo[x] = ghi[x] = btol[x] = 0.0;
      if (M[x] == 0) continue;
      const double pad = 2.0 * DBL_EPSILON * fmax(fabs(l2[x]), fabs(h2[x])) * M[x] + DBL_MIN;
      glo[x] = l2[x] - pad;
      ghi[x] = h2[x] + pad;
      btol[x] = CSS_BISECT_TOL * fmax(fabs(glo[x]), fabs(ghi[x])) + DBL_MIN;
    }
    for (int k = lane; k < 2 * (MP + 4); k += 64) {
      const int x = k >= MP + 4, kk = x ? k - (MP + 4) : k;
      if (kk >= M[x]) s_d[x][kk] = 2.0 * fabs(ghi[x]) + 2.0 * fabs(glo[x]) + 1.0;
    }
  }
  __syncthreads();
  p40_bisect<!CSS_TWIST>(M[0], M[1], glo, ghi, btol, s_d, s_u.a.e2, s_lam, lane);
  __syncthreads();

  CSS_PROF(3);
  /* ---- eigenvectors of each T: twisted factorisations, or two steps of inverse iteration */
  double y1 = 0.0, y2 = 0.0, y1t = 0.0, y2t = 0.0;
  bool twist_ok = false;
#if CSS_TWIST
  {
    double nz0, nz1;
    twist_ok = twisted_top2<MP, 2>(M, lane, &s_d[0][0], MP + 4, &s_e[0][0], MP, &s_u.c.e2[0][0], MP + 4, &s_lam[0][0],
                                   s_u.c.Q, &s_x[0][0], 2 * MP, nz0, nz1);
    if (twist_ok) {
      const double r1 = 1.0 / sqrt(nz0), r2 = 1.0 / sqrt(nz1);
      y1 = rowk ? s_u.c.Q[hi][0][1][r] * r1 : 0.0;
      y2 = rowk ? s_u.c.Q[hi][1][1][r] * r2 : 0.0;
      y1t = trowk ? s_u.c.Q[hi][0][1][R] * r1 : 0.0;
      y2t = trowk ? s_u.c.Q[hi][1][1][R] * r2 : 0.0;
    }
    __syncthreads();
  }
#endif
  if (!twist_ok) {
    /* one eigenvector at a time in slot 0 (lane x of window x); the first one's unit vector
     * waits in y[x][1] */
#pragma unroll 1
    for (int e = 0; e < 2; ++e) {
      __syncthreads();
      if (lane < 2 && M[lane] > 0)
        invit_factor<MP>(M[lane], e, s_d[lane], s_e[lane], s_lam[lane], s_u.b.lu[lane], s_x[lane], s_u.b.piv[lane],
                         s_u.b.y[lane], 0);
      __syncthreads();
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const double tiny = DBL_EPSILON * fmax(fmax(fabs(glo[x]), fabs(ghi[x])), DBL_MIN);
        for (int k = lane; k < M[x]; k += 64) {
          const double u0 = s_u.b.lu[x][0][0][k];
          s_u.b.lu[x][0][0][k] = fast_rcp(u0 == 0.0 ? tiny : u0);
        }
      }
      double ye = 0.0, yet = 0.0;
#ifdef GD_CSS_SKIP_INVIT
      for (int itn = 0; itn < 0; ++itn) {
#else
      for (int itn = 0; itn < 2; ++itn) {
#endif
        __syncthreads();
        if (lane < 2 && M[lane] > 0) invit_solve<MP>(M[lane], 0, s_u.b.lu[lane], s_x[lane], s_u.b.piv[lane], s_u.b.y[lane]);
        __syncthreads();
        ye = rowk ? s_u.b.y[hi][0][r] : 0.0;
        yet = trowk ? s_u.b.y[hi][0][R] : 0.0;
        double n1 = ye * ye + (tq == 0 ? yet * yet : 0.0), dm = 0.0;
        half_sum2(n1, dm);
        const double r1 = 1.0 / sqrt(n1);
        ye *= r1;
        yet *= r1;
        __syncthreads();
        if (itn == 0) {
          if (rowk) s_u.b.y[hi][0][r] = ye;
          if (tq == 0 && trowk) s_u.b.y[hi][0][R] = yet;
        }
      }
      if (e == 0) {
        y1 = ye;
        y1t = yet;
      } else {
        y2 = ye;
        y2t = yet;
      }
    }
  }
  /* orthogonalise the second vector against the first (close eigenvalues) */
  {
    double dt = y1 * y2 + (tq == 0 ? y1t * y2t : 0.0), dm = 0.0;
    half_sum2(dt, dm);
    y2 = fma(-dt, y1, y2);
    y2t = fma(-dt, y1t, y2t);
    double n = y2 * y2 + (tq == 0 ? y2t * y2t : 0.0);
    dm = 0.0;
    half_sum2(n, dm);
    const double rn = 1.0 / sqrt(n);
    y2 *= rn;
    y2t *= rn;
  }
  /* eigenvalues = Rayleigh quotients y^T T y of the unit vectors (k_css_mds) */
  {
    __syncthreads();
    if (rowk) {
      s_u.b.y[hi][0][r] = y1;
      s_u.b.y[hi][1][r] = y2;
    }
    if (tq == 0 && trowk) {
      s_u.b.y[hi][0][R] = y1t;
      s_u.b.y[hi][1][R] = y2t;
    }
    __syncthreads();
    double t1 = 0.0, t2 = 0.0;
    const double *e = s_e[hi], *dd = s_d[hi];
    const double(*sy)[MP] = s_u.b.y[hi];
    if (rowk) {
      const double el = r > 0 ? e[r - 1] : 0.0, er = r + 1 < m_me ? e[r] : 0.0;
      const int il = r > 0 ? r - 1 : 0, ir = r + 1 < m_me ? r + 1 : r;
      t1 = y1 * (dd[r] * y1 + el * sy[0][il] + er * sy[0][ir]);
      t2 = y2 * (dd[r] * y2 + el * sy[1][il] + er * sy[1][ir]);
    }
    if (tq == 0 && trowk) {
      const double el = e[R - 1], er = R + 1 < m_me ? e[R] : 0.0;
      const int il = R - 1, ir = R + 1 < m_me ? R + 1 : R;
      t1 += y1t * (dd[R] * y1t + el * sy[0][il] + er * sy[0][ir]);
      t2 += y2t * (dd[R] * y2t + el * sy[1][il] + er * sy[1][ir]);
    }
    half_sum2(t1, t2);
    if (r == 0) {
      const double zt = h ? ztol[1] : ztol[0];
      s_lam[hi][0] = fabs(t1) <= zt ? 0.0 : t1;
      s_lam[hi][1] = fabs(t2) <= zt ? 0.0 : t2;
    }
    __syncthreads();
  }

  CSS_PROF(4);
  /* ---- back-transformation y <- H_0 H_1 ... H_{m-3} y per window */
#ifndef GD_CSS_SKIP_BACK
  const double tq0 = tq == 0 ? 1.0 : 0.0;
#pragma unroll
  for (int k = MP - 3; k >= 0; --k) {
    const bool liveA = k <= M[0] - 3, liveB = k <= M[1] - 3;
    if (liveA || liveB) {
      /* a window past its last reflector only needs tau = 0 (its y stays); rows past m hold
       * zero v, and the tail's quad replication is one 0/1 factor (k_css_mds_t80) */
      const bool mine = h ? liveB : liveA;
      const double vk = A[k];
      const double vkt = s_tail[hi][tr][k];
      const double t = mine ? s_tau[hi][k] : 0.0;
      const double vq = vkt * tq0;
      double d1 = fma(vq, y1t, vk * y1);
      double d2 = fma(vq, y2t, vk * y2);
      half_sum2(d1, d2);
      y1 = fma(-(t * d1), vk, y1);
      y2 = fma(-(t * d2), vk, y2);
      y1t = fma(-(t * d1), vkt, y1t);
      y2t = fma(-(t * d2), vkt, y2t);
      asm volatile("" ::: "memory"); /* one s_tau load in flight, not MP */
    }
  }
#endif

  CSS_PROF(5);
  /* ---- X = Q sqrt(L) (css.c:545-556), then calc_dist + css on identity groups */
  {
    const double L1 = sqrt(s_lam[hi][0]), L2 = sqrt(s_lam[hi][1]);
    __syncthreads();
    if (rowk) {
      s_x[hi][2 * r] = y1 * L1 + y2 * 0.0;
      s_x[hi][2 * r + 1] = y1 * 0.0 + y2 * L2;
    }
    if (tq == 0 && trowk) {
      s_x[hi][2 * R] = y1t * L1 + y2t * 0.0;
      s_x[hi][2 * R + 1] = y1t * 0.0 + y2t * L2;
    }
    __syncthreads();
  }
  /* css (css.c:608-647) of both windows at once, each over its own half: the pairs of
   * css_score spread over 32 lanes instead of 64, one half-wave sum for both */
  {
    const int a = h ? Aa[1] : Aa[0], b = h ? Bb[1] : Bb[0], m = h ? M[1] : M[0];
    const double *X = s_x[hi];
    const int ab = a * b;
    const float invb = 1.0f / (float)b;
    double bet = 0.0, win = 0.0;
    if (m > 0) {
      for (int q = r; q < ab; q += 32) {
        const int ii = (int)(((float)q + 0.5f) * invb); /* exact for q < 2^14 (ab <= 400 here) */
        bet += xdist(X, ii, a + (q - ii * b));
      }
      /* consecutive pairs only (Q8), each pre-divided by its group's a^2 (a-1) */
      for (int k = r; k < m - 1; k += 32) {
        if (k < a - 1) win += xdist(X, k, k + 1) / (double)(a * a * (a - 1));
        if (k >= a) win += xdist(X, k, k + 1) / (double)(b * b * (b - 1));
      }
    }
    half_sum2(bet, win);
    const double score = bet / (a * b) - (a + b) * win;
    /* score == -1: the reference's "discarded" marker (css.c:127) */
    if (m > 0 && score != -1.0) {
      const int64_t w = h ? W[1] : W[0];
      const gd_chrom_dev &d = ch[h ? C[1] : C[0]];
      const int64_t wl = w - d.w_base;
      if (r == 0) {
        scores[d.w_out + wl] = score;
        if (!want_x) pvals[d.w_out + wl] = 1.0; /* runs == 0: p = (0 + 1) / (0 + 1) */
      }
      if (want_x) {
        for (int e = r; e < 2 * MP; e += 32) xbuf[w * 2 * MP + e] = (e < 2 * m) ? X[e] : 0.0;
        if (r == 0) status[w] = 1;
      }
    }
  }
  CSS_PROF(6);
}


int gd_css_launch_p40(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s) {
#if CSS_H40
  CSS_PROF_LAUNCH(s);
  hipLaunchKernelGGL(k_css_mds_h40, dim3((unsigned)((wtotal + 1) / 2)), dim3(64), 0, s, d_ch, nchrom, d_pl, planes,
                     lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x, force_literal, scores, p, xbuf, status, flags);
#else
  hipLaunchKernelGGL(k_css_mds_p40, dim3((unsigned)((wtotal + 1) / 2)), dim3(64), 0, s, d_ch, nchrom, d_pl, planes,
                     lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x, force_literal, scores, p, xbuf, status, flags);
#endif
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}
