/*
 * gd_css_t80.hip -- the 65..80-individual CSS MDS tier, one window per wave (k_css_mds_t80; css.c:181-223, 277-366, 505-647)
 */
#include "gd_css_common.h"

/* ------------------------------------------------------------------------ */
/* The 65..80-individual tier in ONE wave (k_css_mds_t80).  Rows 0..63 of the  */
/* matrix live in the VGPRs of lanes 0..63 (80 columns each, as k_css_mds<MP, 1>); */
/* rows 64..79 live in LDS, each worked by a quad of lanes over interleaved      */
/* columns (lane 4r + q holds columns 4s + q of tail row r), so a column group    */
/* dead for the main rows is dead for the tail too and both skip it by the same   */
/* compile-time test.  One wave per window: no workgroup barriers, 2 waves per    */
/* SIMD, 8 windows per CU (the two-wave layout ran 4, three barriers per step).   */
/* ------------------------------------------------------------------------ */
namespace {
constexpr int T80 = 80, T80_MAIN = 64, T80_TS = 20; /* order, VGPR rows, tail columns per lane */
/* tail row stride in doubles: 2 * 84 = 40 (mod 64) dwords, so the 8 tail rows of a
 * 32-lane group start 8 banks apart and a quad's 4 columns fill its 8 banks (a stride of
 * 80 doubles put 4 rows on the same banks: 4-way conflicts on every tail access) */
constexpr int T80_TSTRIDE = 84;

/* Householder steps: one LDS round trip per step (the unfused form, hh_step_static,
 * took two and ran C4 at 5.9 M windows/s against 7.2 M).  Row K of the
 * matrix is read as column K (every lane holds its own entry, symmetric up to rounding),
 * so the reflector's vector needs no single-lane publish: after step K's scalars every lane
 * computes its entry of column K + 1 as it will be after the update (v_{K+1} = 1,
 * w_{K+1} by v_readlane) and publishes it with v_i, w_i; one pass over the row then applies
 * the rank-2 update and accumulates the next step's p = A r, four chains deep.  r and p
 * travel to the next step in registers (T80Carry). */
struct T80Carry {
  double r, p, rt, pt; /* column K entry and p_i of this lane's main row and tail row */
};

/* the rank-2 update of this lane's rows over columns > K and p = A r over columns > K + 1
 * (s_r holds 0 at rows <= K + 1) */
template <int K>
__device__ __forceinline__ void t80_fused_pass(double (&A)[T80], double vi, double wi, double vt, double wt,
                                               const double2 *s_vw, const double *s_r,
                                               double (*s_tail)[T80_TSTRIDE], T80Carry &c) {
  constexpr int MP = T80;
  const int i = css_lane_now(), tr = i >> 2, tq = i & 3;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#ifndef T80_NO_READ2
#define T80_NO_READ2 1
#endif
#ifndef T80_FB
#define T80_FB 4
#endif
  constexpr int FB = T80_FB; /* columns per pinned group (register pressure) */
  /* software-pipelined: group jb + 1's (v, w) and r are loaded before group jb is
   * computed, so a group waits on loads issued one group earlier; the pins' memory
   * clobbers keep the loads of later groups below them (bounded registers) */
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
      /* from K = 63 on every main row is finished (v_i = w_i = 0): no update */
      if (j > K && K + 1 < T80_MAIN) A[j] = fma(-vi, cvw[u].y, fma(-wi, cvw[u].x, A[j]));
    }
#pragma unroll
    for (int u = 0; u < FB; ++u) CSS_PIN(A[FB * jb + u]);
#pragma unroll
    for (int u = 0; u < FB; ++u) {
      const int j = FB * jb + u;
      if (j > K + 1 && K + 1 < T80_MAIN) p[u & 3] = fma(A[j], cr[u], p[u & 3]);
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
#ifndef T80_TG
#define T80_TG 2
#endif
  constexpr int TG = T80_TG, S0 = (K + 1) / 4 / TG * TG; /* tail groups of TG column quads */
  double ct[TG], ctr[TG];
  double2 ctv[TG];
  /* the odd member of each column pair is addressed through an opaque zero, so the two 8-byte
   * reads are not merged into one ds_read2_b64 (8 LDS cycles, MI355X_MICROARCH.md LDS table)
   * but stay two ds_read_b64 (2 cycles each): the pass is LDS-array bound as much as VALU bound */
  int o1 = 0;
#if T80_NO_READ2
  asm volatile("" : "+v"(o1));
#endif
#pragma unroll
  for (int u = 0; u < TG; ++u) {
    const int j = 4 * (S0 + u) + tq + ((u & 1) ? o1 : 0);
    ct[u] = tw[j];
    ctv[u] = s_vw[j];
    ctr[u] = s_r[j];
  }
#pragma unroll
  for (int sg = S0; sg < T80_TS; sg += TG) {
    double nt[TG], ntr[TG];
    double2 ntv[TG];
    if (sg + TG < T80_TS) {
#pragma unroll
      for (int u = 0; u < TG; ++u) {
        const int j = 4 * (sg + TG + u) + tq + ((u & 1) ? o1 : 0);
        nt[u] = tw[j];
        ntv[u] = s_vw[j];
        ntr[u] = s_r[j];
      }
    }
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      const int j = 4 * (sg + u) + tq;
      if (4 * (sg + u) + 3 > K) { /* v_j = w_j = 0 at j <= K: the dead columns stay */
        const double t = fma(-vt, ctv[u].y, fma(-wt, ctv[u].x, ct[u]));
        tw[j] = t;
        if (u & 1)
          t1 = fma(t, ctr[u], t1);
        else
          t0 = fma(t, ctr[u], t0);
      }
    }
    CSS_PIN(t0);
    CSS_PIN(t1);
    if (sg + TG < T80_TS) {
#pragma unroll
      for (int u = 0; u < TG; ++u) {
        ct[u] = nt[u];
        ctv[u] = ntv[u];
        ctr[u] = ntr[u];
      }
    }
  }
  if (tq == (K & 3)) tw[K] = vt;
  c.p = (p[0] + p[1]) + (p[2] + p[3]);
  c.pt = quad_sum(t0 + t1);
}

/* column 0 and p = A r before step 0 */
__device__ __forceinline__ void t80_fused_start(const double (&A)[T80], int m, double2 *s_vw, double *s_r, double *s_d,
                                                double (*s_tail)[T80_TSTRIDE], T80Carry &c) {
  constexpr int MP = T80;
  const int i = css_lane_now(), tr = i >> 2, tq = i & 3, R = T80_MAIN + tr;
  (void)m;
  c.r = A[0];
  c.rt = s_tail[tr][0];
  __syncthreads();
  s_r[i] = i > 0 ? c.r : 0.0;
  if (tq == 0) s_r[R] = c.rt;
  if (i == 0) s_d[0] = c.r;
  __syncthreads();
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 1; j < MP; ++j) {
    p[j & 3] = fma(A[j], s_r[j], p[j & 3]);
    if ((j & 7) == 7) {
#pragma unroll
      for (int u = 0; u < 4; ++u) CSS_PIN(p[u]);
    }
  }
  const double *trw = s_tail[tr];
  double t0 = 0.0, t1 = 0.0;
#pragma unroll
  for (int s = 0; s < T80_TS; ++s) {
    const int j = 4 * s + tq;
    if (s & 1)
      t1 = fma(trw[j], s_r[j], t1);
    else
      t0 = fma(trw[j], s_r[j], t0);
  }
  c.p = (p[0] + p[1]) + (p[2] + p[3]);
  c.pt = quad_sum(t0 + t1);
  (void)s_vw;
}

/* One fused Householder step K <= MP - 3 (hh_step_static's arithmetic) */
template <int K>
__device__ __forceinline__ void t80_fstep(double (&A)[T80], int m, T80Carry &c, double2 *s_vw, double *s_r,
                                          double *s_d, double *s_e, double *s_tau, double (*s_tail)[T80_TSTRIDE]) {
  const int i = css_lane_now(), tr = i >> 2, tq = i & 3, R = T80_MAIN + tr;
  /* rows >= m are zero and stay zero (v_i = w_i = 0 there), as do their r and p entries:
   * only the rows the earlier steps finished (<= K) need masking */
  const double xi = (i > K + 1) ? c.r : 0.0;
  const double xr = (R > K + 1) ? c.rt : 0.0;
  /* |x|^2 and r^T A r in one reduction; a tail row counts once */
  double sigma = xi * xi + (tq == 0 ? xr * xr : 0.0);
  double q = ((i > K) ? c.r * c.p : 0.0) + ((tq == 0 && R > K) ? c.rt * c.pt : 0.0);
  wave_sum2(sigma, q);
  double alpha, pr1, a11;
  if constexpr (K + 1 < T80_MAIN) {
    alpha = readlane_f64(c.r, K + 1);
    pr1 = readlane_f64(c.p, K + 1);
    a11 = readlane_f64(A[K + 1], K + 1);
  } else {
    alpha = readlane_f64(c.rt, 4 * (K + 1 - T80_MAIN));
    pr1 = readlane_f64(c.pt, 4 * (K + 1 - T80_MAIN));
    a11 = s_tail[K + 1 - T80_MAIN][K + 1];
  }
  double tau = 0.0, beta = alpha, scale = 0.0;
  if (sigma != 0.0) {
    beta = -copysign(sqrt_pos(alpha * alpha + sigma), alpha);
    const double rr = fast_rcp(beta * (alpha - beta));
    tau = -(alpha - beta) * (alpha - beta) * rr;
    scale = beta * rr;
  }
  const double Kc = -0.5 * tau * (tau * scale * scale) * fma(beta, fma(beta, a11, -2.0 * pr1), q);
  const double ak1 = A[K + 1];
  const double vi = (i == K + 1) ? 1.0 : xi * scale;
  const double pi = (i > K) ? (tau * scale) * fma(-beta, ak1, c.p) : 0.0;
  const double wi = fma(Kc, vi, pi);
  const double akt = s_tail[tr][K + 1];
  const double vt = (R == K + 1) ? 1.0 : xr * scale;
  const double ptl = (R > K) ? (tau * scale) * fma(-beta, akt, c.pt) : 0.0;
  const double wt = fma(Kc, vt, ptl);
  double wk1;
  if constexpr (K + 1 < T80_MAIN)
    wk1 = readlane_f64(wi, K + 1);
  else
    wk1 = readlane_f64(wt, 4 * (K + 1 - T80_MAIN));
  /* column K + 1 after this step (the update's formula at v_{K+1} = 1) */
  const double rn = fma(-vi, wk1, fma(-wi, 1.0, ak1));
  const double rnt = fma(-vt, wk1, fma(-wt, 1.0, akt));
  __syncthreads();
  if (i == 0) {
    s_e[K] = beta;
    s_tau[K] = tau;
  }
  s_vw[i] = make_double2(vi, wi);
  s_r[i] = i > K + 1 ? rn : 0.0;
  if (tq == 0) {
    s_vw[R] = make_double2(vt, wt);
    s_r[R] = R > K + 1 ? rnt : 0.0;
  }
  if constexpr (K + 1 < T80_MAIN) {
    if (i == K + 1) s_d[K + 1] = rn;
  } else {
    if (i == 4 * (K + 1 - T80_MAIN)) s_d[K + 1] = rnt;
  }
  __syncthreads();
  t80_fused_pass<K>(A, vi, wi, vt, wt, s_vw, s_r, s_tail, c);
  c.r = rn;
  c.rt = rnt;
}

template <int K>
struct T80FSteps {
  static __device__ __forceinline__ void run(double (&A)[T80], int m, T80Carry &c, double2 *s_vw, double *s_r,
                                             double *s_d, double *s_e, double *s_tau, double (*s_tail)[T80_TSTRIDE]) {
    if ((K & 7) == 0 && K >= m) return; /* exits only at block boundaries (hh_step_static) */
    if constexpr (K <= T80 - 3) {
      t80_fstep<K>(A, m, c, s_vw, s_r, s_d, s_e, s_tau, s_tail);
      T80FSteps<K + 1>::run(A, m, c, s_vw, s_r, s_d, s_e, s_tau, s_tail);
    } else {
      /* K = MP - 2: no reflector; e_{MP-2} = column MP - 2 at row MP - 1, d_{MP-1} */
      const int i = css_lane_now();
      const double e = readlane_f64(c.rt, 4 * (T80 - 1 - T80_MAIN));
      __syncthreads();
      if (i == 0) {
        if (K == m - 2) s_e[K] = e;
        s_d[K + 1] = s_tail[T80 - 1 - T80_MAIN][T80 - 1];
      }
    }
  }
};

}  // namespace

__global__ void __launch_bounds__(64, 2)
    k_css_mds_t80(const gd_chrom_dev *ch, int nchrom, const gd_css_planes *pl, const uint32_t *planes,
                  const int32_t *lo_a_, const int32_t *hi_a_, const int32_t *lo_b_, const double *avals,
                  const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *pvals,
                  double *xbuf, uint8_t *status, unsigned *flags) {
  constexpr int MP = T80;
  __shared__ __attribute__((aligned(16))) double s_tail[MP - T80_MAIN][T80_TSTRIDE];
  /* the distance build's and the Householder steps' buffers, reused by inverse iteration */
  __shared__ __attribute__((aligned(16))) union {
    struct {
      double e2[MP + 4]; /* bisection only (after the Householder steps) */
      double r[MP + 2]; /* Householder steps: column K + 1; row means before them */
      double2 vw[MP];   /* Householder steps: (v_j, w_j), 16-B aligned */
      uint64_t mask[2 * MP];
      double vals[MP];
    } a;
    struct {
      double lu[2][3][MP];
      double y[2][MP];
      uint8_t piv[2][MP];
    } b;
    struct {
      double e2[MP + 4]; /* = a.e2: the twisted factorisations read it */
      double Q[2][2][MP];
    } c;
  } s_u;
  __shared__ __attribute__((aligned(16))) double s_d[MP + 4];
  double *s_e2 = s_u.a.e2;
  __shared__ double s_e[MP], s_tau[MP];
  __shared__ double s_x[2 * MP];
  __shared__ int s_tr[MP];
  __shared__ double s_lam[2];
  __shared__ double s_red[4];

  const int tid = threadIdx.x;
  const int i = tid, tr = tid >> 2, tq = tid & 3, R = T80_MAIN + tr;
  for (int k = tid; k < MP; k += 64) s_tr[k] = k;

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
    const bool row = i < m, trow = R < m;
    const gd_css_planes P = pl[c];
    const uint32_t *pa = planes + P.pa, *pb = planes + P.pb;
    const int64_t ra = la / a, rb = lb / b;

    /* ---- regular window?  (k_css_mds) */
    bool literal = force_literal || (la % a) != 0 || (lb % b) != 0;
    if (!literal) {
      int irr = 0;
      for (int k = tid; k * 64 < npos; k += 64) {
        const int nb = min(64, npos - 64 * k);
        const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
        const uint64_t xa = plane_bits64(pa + (int64_t)(2 * a) * P.wa, ra + 64 * k) & tail;
        const uint64_t xb = plane_bits64(pb + (int64_t)(2 * b) * P.wb, rb + 64 * k) & tail;
        irr |= (xa | xb) != 0;
      }
      literal = __syncthreads_or(irr);
    }

    /* ---- compare_all: main row i in A, tail row R's columns 4s + tq into s_tail */
    double A[MP];
    {
      /* the main row's counts accumulate in A itself (exact integers in FP64): an int
       * accumulator array beside A held 80 more VGPRs at the conversion and pushed the
       * kernel into scratch */
      int acct[T80_TS];
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) A[jj] = 0.0;
#pragma unroll
      for (int s = 0; s < T80_TS; ++s) acct[s] = 0;
      if (!literal) {
        for (int k = 0; k * 64 < npos; ++k) {
          const int nb = min(64, npos - 64 * k);
          const uint64_t tail = nb == 64 ? ~0ull : ((1ull << nb) - 1);
          __syncthreads();
          for (int r = tid; r < MP; r += 64) {
            uint64_t Pm = 0, Nm = 0;
            if (r < m) {
              const uint32_t *base = r < a ? pa + (int64_t)(2 * r) * P.wa : pb + (int64_t)(2 * (r - a)) * P.wb;
              const int64_t nw = r < a ? P.wa : P.wb;
              const int64_t rr = (r < a ? ra : rb) + 64 * k;
              Pm = plane_bits64(base, rr) & tail;
              Nm = plane_bits64(base + nw, rr) & tail;
            }
            s_u.a.mask[2 * r] = Pm;
            s_u.a.mask[2 * r + 1] = Nm;
          }
          __syncthreads();
          const uint64_t *mk = s_u.a.mask;
          const uint64_t Pi = mk[2 * i], Ni = mk[2 * i + 1];
#pragma unroll
          for (int jj = 0; jj < MP; ++jj) {
            A[jj] += (double)(__popcll(Pi & mk[2 * jj + 1]) + __popcll(Ni & mk[2 * jj]));
            if ((jj & 7) == 7) {
#pragma unroll
              for (int u = jj - 7; u <= jj; ++u) CSS_PIN(A[u]);
            }
          }
          const uint64_t Pt = mk[2 * R], Nt = mk[2 * R + 1];
#pragma unroll
          for (int s = 0; s < T80_TS; ++s) {
            const int j = 4 * s + tq;
            acct[s] += __popcll(Pt & mk[2 * j + 1]) + __popcll(Nt & mk[2 * j]);
          }
        }
      } else {
        const double *av = avals + d.a_off + la, *bv = bvals + d.b_off + lb;
        for (int k = 0; k < npos; ++k) {
          __syncthreads();
          for (int r = tid; r < m; r += 64)
            s_u.a.vals[r] = r < a ? av[(int64_t)k * a + r] : bv[(int64_t)k * b + (r - a)];
          __syncthreads();
          const double *sv = s_u.a.vals;
          int io = i, ro = R, mo = m, ao = a;
          CSS_OPAQUE_V(io);
          CSS_OPAQUE_V(ro);
          CSS_OPAQUE_S(mo);
          CSS_OPAQUE_S(ao);
          const double vi = sv[io], vr = sv[ro];
#pragma unroll
          for (int jj = 0; jj < MP; ++jj) {
            /* the diagonal never counts: (int)v * v >= 0 */
            if (jj < mo) {
              const double vj = sv[jj];
              /* the reference casts the row element of the larger index within a
               * population and the A element across populations (css.c:281-326) */
              const bool cast_i = ((io < ao) == (jj < ao)) ? (io > jj) : (io < ao);
              const double prod = cast_i ? x86_int(vi) * vj : x86_int(vj) * vi;
              A[jj] += prod == -9.0 ? 1.0 : 0.0;
            }
          }
#pragma unroll
          for (int s = 0; s < T80_TS; ++s) {
            const int j = 4 * s + tq;
            if (j < mo) {
              const double vj = sv[j];
              const bool cast_r = ((ro < ao) == (j < ao)) ? (ro > j) : (ro < ao);
              const double prod = cast_r ? x86_int(vr) * vj : x86_int(vj) * vr;
              acct[s] += prod == -9.0;
            }
          }
        }
        /* rows >= m read stale values: zero them (the popcount path has no bits there) */
#pragma unroll
        for (int jj = 0; jj < MP; ++jj) A[jj] = row ? A[jj] : 0.0;
      }
      /* entries past column m are zero already (no plane bits, or the literal loop's j < m
       * test), as are main rows >= m: only the tail rows are masked */
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int s = 0; s < T80_TS; ++s) {
        const int j = 4 * s + tq;
        s_tail[tr][j] = (trow && j < mo) ? (double)acct[s] : 0.0;
      }
    }

    CSS_PROF(0);
    /* ---- fill_averages (k_css_mds).  The entries are exact integer counts, so "< 1e-5" is
     * "== 0": sum = the plain row sum (zeros add nothing), the valid count = sum of
     * min(v, 1), unval = m^2 - valid -- no per-entry branch or select (the branchy form
     * compiled to ~25 instructions per entry) */
    {
      const int ln_ = css_lane_now();
      const int tr = ln_ >> 2, tq = ln_ & 3;
      double s4[4] = {0.0, 0.0, 0.0, 0.0}, n4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) {
        s4[jj & 3] += A[jj];
        n4[jj & 3] += fmin(A[jj], 1.0);
      }
#pragma unroll
      for (int s = 0; s < T80_TS; ++s) {
        const double t = s_tail[tr][4 * s + tq];
        s4[s & 3] += t;
        n4[s & 3] += fmin(t, 1.0);
      }
      double sum = (s4[0] + s4[1]) + (s4[2] + s4[3]), nz = (n4[0] + n4[1]) + (n4[2] + n4[3]);
      wave_sum2(nz, sum); /* sums of integers: exact in any order */
      const int tot = m * m;
      const int unval = tot - (int)nz;
      if (unval > tot / 2) continue; /* discarded window: outputs untouched */
      const double avg = sum / tot;
      /* rows >= m stay zero; the columns >= m it fills are zeroed by the next pass */
      const double avgr = ln_ < m ? avg : 0.0;
      CSS_OPAQUE_ROW(A);
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) A[jj] = fma(avgr, 1.0 - fmin(A[jj], 1.0), A[jj]);
#pragma unroll
      for (int s = 0; s < T80_TS; ++s) {
        double *t = &s_tail[tr][4 * s + tq];
        *t = fma(avg, 1.0 - fmin(*t, 1.0), *t);
      }
    }

    /* ---- B = -1/2 Z (D o D) Z by double centering */
    double zero_tol;
    {
      const int ln_ = css_lane_now(); /* (as in fill_averages) */
      const int i = ln_, tr = ln_ >> 2, tq = ln_ & 3, R = T80_MAIN + tr;
      const bool row = i < m, trow = R < m;
      double rs = 0, rst = 0;
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) {
        A[jj] = (row && jj < mo) ? A[jj] * A[jj] : 0.0;
        rs += A[jj];
      }
#pragma unroll
      for (int s = 0; s < T80_TS; ++s) {
        const int j = 4 * s + tq;
        double *t = &s_tail[tr][j];
        const double sq = (trow && j < mo) ? *t * *t : 0.0;
        *t = sq;
        rst += sq;
      }
      rst = quad_sum(rst);
      const double ri = row ? rs / m : 0.0, rt = trow ? rst / m : 0.0;
      __syncthreads();
      s_u.a.r[i] = ri;
      if (tq == 0) s_u.a.r[R] = rt;
      const double g = block_sum<1>(ri + (tq == 0 ? rt : 0.0), s_red) / m;
      __syncthreads();
      const double *sv = s_u.a.r;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) {
        A[jj] = (row && jj < mo) ? -0.5 * ((A[jj] - (ri + sv[jj])) + g) : 0.0;
        if ((jj & 7) == 7) {
#pragma unroll
          for (int u = jj - 7; u <= jj; ++u) CSS_PIN(A[u]);
        }
      }
      double f2 = 0;
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) f2 = fma(A[jj], A[jj], f2);
#pragma unroll
      for (int s = 0; s < T80_TS; ++s) {
        const int j = 4 * s + tq;
        double *t = &s_tail[tr][j];
        const double cv = (trow && j < mo) ? -0.5 * ((*t - (rt + sv[j])) + g) : 0.0;
        *t = cv;
        f2 = fma(cv, cv, f2);
      }
      /* eigenvalues within rounding of 0 count as 0 (oracle/css_oracle.c, cmds) */
      zero_tol = 64.0 * m * DBL_EPSILON * sqrt(block_sum<1>(f2, s_red));
    }

    CSS_PROF(1);
    /* ---- Householder tridiagonalisation (LAPACK dsytd2, lower; k_css_mds) */
#ifndef GD_CSS_SKIP_TRIDIAG
    {
      T80Carry cr;
      t80_fused_start(A, m, s_u.a.vw, s_u.a.r, s_d, s_tail, cr);
      T80FSteps<0>::run(A, m, cr, s_u.a.vw, s_u.a.r, s_d, s_e, s_tau, s_tail);
    }
#endif
    __syncthreads();

    CSS_PROF(2);
    /* ---- the two largest eigenvalues of T (k_css_mds) */
    double glo, ghi;
    {
      double lo = DBL_MAX, hi = -DBL_MAX;
      if (row) {
        const double r = (i > 0 ? fabs(s_e[i - 1]) : 0.0) + (i < m - 1 ? fabs(s_e[i]) : 0.0);
        lo = s_d[i] - r;
        hi = s_d[i] + r;
      }
      if (tq == 0 && trow) {
        const double r = fabs(s_e[R - 1]) + (R < m - 1 ? fabs(s_e[R]) : 0.0);
        lo = fmin(lo, s_d[R] - r);
        hi = fmax(hi, s_d[R] + r);
      }
      for (int k = tid; k < MP + 4; k += 64)
        s_e2[k] = (k >= 1 && k < m) ? fmax(s_e[k - 1] * s_e[k - 1], CSS_E2_FLOOR) : 0.0;
      glo = block_reduce<1, OpMin>(lo, s_red);
      ghi = block_reduce<1, OpMax>(hi, s_red);
      const double pad = 2.0 * DBL_EPSILON * fmax(fabs(glo), fabs(ghi)) * m + DBL_MIN;
      glo -= pad;
      ghi += pad;
      for (int k = tid; k < MP + 4; k += 64)
        if (k >= m) s_d[k] = 2.0 * fabs(ghi) + 2.0 * fabs(glo) + 1.0;
    }
    const double bis_tol = CSS_BISECT_TOL * fmax(fabs(glo), fabs(ghi)) + DBL_MIN;
    __syncthreads();
    bisect_top2<true, !CSS_TWIST>(m, glo, ghi, bis_tol, s_d, s_e2, s_lam, tid);
    __syncthreads();

    CSS_PROF(3);
    /* ---- eigenvectors of T: twisted factorisations, or two steps of inverse iteration */
    double y1 = 0.0, y2 = 0.0, y1t = 0.0, y2t = 0.0;
    bool twist_ok = false;
#if CSS_TWIST
    {
      double nz0, nz1;
      const int M1[1] = {m};
      twist_ok = twisted_top2<MP, 1>(M1, tid, s_d, 0, s_e, 0, s_e2, 0, s_lam, &s_u.c.Q, s_x, 0, nz0, nz1);
      if (twist_ok) {
        const double r1 = 1.0 / sqrt(nz0), r2 = 1.0 / sqrt(nz1);
        y1 = row ? s_u.c.Q[0][1][i] * r1 : 0.0;
        y2 = row ? s_u.c.Q[1][1][i] * r2 : 0.0;
        y1t = trow ? s_u.c.Q[0][1][R] * r1 : 0.0;
        y2t = trow ? s_u.c.Q[1][1][R] * r2 : 0.0;
      }
      __syncthreads();
    }
#endif
    if (!twist_ok) {
      if (tid < 2) invit_factor<MP>(m, tid, s_d, s_e, s_lam, s_u.b.lu, s_x, s_u.b.piv, s_u.b.y);
      __syncthreads();
      {
        const double tiny = DBL_EPSILON * fmax(fmax(fabs(glo), fabs(ghi)), DBL_MIN);
        for (int k = tid; k < m; k += 64) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const double u0 = s_u.b.lu[e][0][k];
            s_u.b.lu[e][0][k] = fast_rcp(u0 == 0.0 ? tiny : u0);
          }
        }
      }
#ifdef GD_CSS_SKIP_INVIT
      for (int itn = 0; itn < 0; ++itn) {
#else
      for (int itn = 0; itn < 2; ++itn) {
#endif
        __syncthreads();
        if (tid < 2) invit_solve<MP>(m, tid, s_u.b.lu, s_x, s_u.b.piv, s_u.b.y);
        __syncthreads();
        y1 = row ? s_u.b.y[0][i] : 0.0;
        y2 = row ? s_u.b.y[1][i] : 0.0;
        y1t = trow ? s_u.b.y[0][R] : 0.0;
        y2t = trow ? s_u.b.y[1][R] : 0.0;
        double n1 = y1 * y1 + (tq == 0 ? y1t * y1t : 0.0), n2 = y2 * y2 + (tq == 0 ? y2t * y2t : 0.0);
        wave_sum2(n1, n2);
        const double r1 = 1.0 / sqrt(n1), r2 = 1.0 / sqrt(n2);
        y1 *= r1;
        y2 *= r2;
        y1t *= r1;
        y2t *= r2;
        __syncthreads();
        if (itn == 0) {
          if (row) {
            s_u.b.y[0][i] = y1;
            s_u.b.y[1][i] = y2;
          }
          if (tq == 0 && trow) {
            s_u.b.y[0][R] = y1t;
            s_u.b.y[1][R] = y2t;
          }
        }
      }
    }
    /* orthogonalise the second vector against the first (close eigenvalues) */
    {
      double dt = y1 * y2 + (tq == 0 ? y1t * y2t : 0.0), zero = 0.0;
      wave_sum2(dt, zero);
      y2 = fma(-dt, y1, y2);
      y2t = fma(-dt, y1t, y2t);
      double n2 = y2 * y2 + (tq == 0 ? y2t * y2t : 0.0);
      zero = 0.0;
      wave_sum2(n2, zero);
      const double r2 = 1.0 / sqrt(n2);
      y2 *= r2;
      y2t *= r2;
    }
    /* eigenvalues = Rayleigh quotients y^T T y of the unit vectors (k_css_mds) */
    {
      double(*sy)[MP] = s_u.b.y;
      __syncthreads();
      if (row) {
        sy[0][i] = y1;
        sy[1][i] = y2;
      }
      if (tq == 0 && trow) {
        sy[0][R] = y1t;
        sy[1][R] = y2t;
      }
      __syncthreads();
      double t1 = 0.0, t2 = 0.0;
      if (row) {
        const double el = i > 0 ? s_e[i - 1] : 0.0, er = i + 1 < m ? s_e[i] : 0.0;
        const int il = i > 0 ? i - 1 : 0, ir = i + 1 < m ? i + 1 : i;
        t1 = y1 * (s_d[i] * y1 + el * sy[0][il] + er * sy[0][ir]);
        t2 = y2 * (s_d[i] * y2 + el * sy[1][il] + er * sy[1][ir]);
      }
      if (tq == 0 && trow) {
        const double el = s_e[R - 1], er = R + 1 < m ? s_e[R] : 0.0;
        const int il = R - 1, ir = R + 1 < m ? R + 1 : R;
        t1 += y1t * (s_d[R] * y1t + el * sy[0][il] + er * sy[0][ir]);
        t2 += y2t * (s_d[R] * y2t + el * sy[1][il] + er * sy[1][ir]);
      }
      wave_sum2(t1, t2);
      if (tid == 0) {
        s_lam[0] = fabs(t1) <= zero_tol ? 0.0 : t1;
        s_lam[1] = fabs(t2) <= zero_tol ? 0.0 : t2;
      }
      __syncthreads();
    }

    CSS_PROF(4);
    /* ---- back-transformation y <- H_0 H_1 ... H_{m-3} y; v_k sits in column k */
#ifndef GD_CSS_SKIP_BACK
    /* v_k is zero in rows >= m (k <= m - 3: the steps that left it there saw zero rows), so
     * only the tail's quad replication needs a mask: one factor, no per-step selects */
    const double tq0 = tq == 0 ? 1.0 : 0.0;
#pragma unroll
    for (int k = MP - 3; k >= 0; --k) {
      if (k <= m - 3) {
        const double vk = A[k];
        const double vkt = s_tail[tr][k];
        const double t = s_tau[k];
        const double vq = vkt * tq0;
        double d1 = fma(vq, y1t, vk * y1), d2 = fma(vq, y2t, vk * y2);
        wave_sum2(d1, d2);
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
      const double L1 = sqrt(s_lam[0]), L2 = sqrt(s_lam[1]);
      __syncthreads();
      if (row) {
        s_x[2 * i] = y1 * L1 + y2 * 0.0;
        s_x[2 * i + 1] = y1 * 0.0 + y2 * L2;
      }
      if (tq == 0 && trow) {
        s_x[2 * R] = y1t * L1 + y2t * 0.0;
        s_x[2 * R + 1] = y1t * 0.0 + y2t * L2;
      }
      __syncthreads();
    }
    const double score = css_score<1>(s_tr, a, b, [&](int p, int q) { return xdist(s_x, p, q); }, s_red);
    CSS_PROF(6);
    if (score == -1.0) continue; /* the reference's "discarded" marker (css.c:127) */
    if (tid == 0) {
      scores[d.w_out + wl] = score;
      if (!want_x) pvals[d.w_out + wl] = 1.0; /* runs == 0: p = (0 + 1) / (0 + 1) */
    }
    if (want_x) {
      for (int e = tid; e < 2 * MP; e += 64) xbuf[w * 2 * MP + e] = (e < 2 * m) ? s_x[e] : 0.0;
      if (tid == 0) status[w] = 1;
    }
  }
}


int gd_css_launch_t80(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s) {
  CSS_PROF_LAUNCH(s);
  hipLaunchKernelGGL(k_css_mds_t80, dim3((unsigned)wtotal), dim3(64), 0, s, d_ch, nchrom, d_pl, planes, lo_a, hi_a,
                     lo_b, avals, bvals, wtotal, want_x, force_literal, scores, p, xbuf, status, flags);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}
