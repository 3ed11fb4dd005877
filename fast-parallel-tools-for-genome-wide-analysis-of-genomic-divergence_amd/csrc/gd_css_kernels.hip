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
 *   (the permutation test, significance_treshold, is in gd_css_perm.hip)
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
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_internal.h"

#ifdef GD_CSS_PROFILE
/* diagnostics build only: shader-clock cycles per phase summed over windows (lane 0),
 * accumulated in registers and added to the totals at the last phase (6): a global atomic
 * at every phase boundary would hold up the next vector-memory wait (the counters drain in
 * order) and bill its queueing to the following phase */
__device__ unsigned long long g_css_prof[8];
#define CSS_PROF_INIT                             \
  uint64_t prof_t = __builtin_readcyclecounter(); \
  uint64_t prof_acc[7] = {0, 0, 0, 0, 0, 0, 0}
#define CSS_PROF(ph)                                                                             \
  do {                                                                                           \
    const uint64_t t_ = __builtin_readcyclecounter();                                           \
    prof_acc[ph] += t_ - prof_t;                                                                 \
    prof_t = t_;                                                                                 \
    if ((ph) == 6 && threadIdx.x == 0)                                                           \
      for (int ph_ = 0; ph_ < 7; ++ph_) atomicAdd(&g_css_prof[ph_], (unsigned long long)prof_acc[ph_]); \
  } while (0)
#else
#define CSS_PROF_INIT
#define CSS_PROF(ph)
#endif

/* waves per SIMD the register allocator must reach for k_css_mds<MP> (measured per
 * tier: MP = 24 fits 5 waves without spills, MP = 40 runs best at 4 with a few cold
 * spills) */
#ifndef CSS_STATIC_G1_MAX
#define CSS_STATIC_G1_MAX 64 /* largest one-lane-per-row tier with compile-time-K steps (64: 29.7 -> 18.4 ms per 200k 32+32 windows) */
#endif
#ifndef CSS_STATIC_G2_MAX
#define CSS_STATIC_G2_MAX 80 /* largest G = 2 tier with compile-time-K steps */
#endif
#ifndef CSS_BISECT_TOL
#define CSS_BISECT_TOL 1e-9 /* bisection stops at this fraction of the spectral bound */
#endif
#ifndef CSS_MDS_WAVES
#ifndef CSS_MDS_WAVES_G2
#define CSS_MDS_WAVES_G2 3 /* waves per SIMD of the 80- and 96-individual tiers (diagnostic override) */
#endif
#ifndef CSS_P40
#define CSS_P40 1 /* the 25-40 individual tier two windows per wave (k_css_mds_p40) */
#endif
#ifndef CSS_H40
#define CSS_H40 1 /* the 25-40 tier with one window per half wave (k_css_mds_h40; 0: k_css_mds_p40) */
#endif
#ifndef CSS_H40_FUSED
#define CSS_H40_FUSED 1 /* k_css_mds_h40 with t80's fused Householder step (0: the publish-row form) */
#endif
#ifndef CSS_T80
#define CSS_T80 1 /* the 80-individual tier in one wave with an LDS tail (k_css_mds_t80) */
#endif
#ifndef CSS_G80
#define CSS_G80 1 /* lanes per row of the 80-individual tier (2 measured 7 % slower) */
#endif
#ifndef CSS_MDS_WAVES_40
#define CSS_MDS_WAVES_40 4 /* waves per SIMD of the 25..40 tier (diagnostic override) */
#endif
#define CSS_MDS_WAVES(MP, G) \
  ((MP) <= 24 ? 5 : (MP) <= 40 ? CSS_MDS_WAVES_40 : (MP) <= 64 || (G) == 1 ? 2 : (MP) <= 96 ? CSS_MDS_WAVES_G2 : 2)
#endif

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
/* Pins a value: everything producing it happens before this point and no later
 * LDS load moves above it.  Used once per 8-column group so a group's broadcast
 * loads are consumed before the next group's are issued. */
#define CSS_PIN(x) asm volatile("" : "+v"(x)::"memory")

/* A copy of x the compiler cannot see through: per-column predicates built from it
 * (j < m, j vs lane) are materialised inside the loop that uses them instead of
 * being hoisted out of the window loop as one live SGPR mask per column. */
#define CSS_OPAQUE_S(x) asm volatile("" : "+s"(x))
#define CSS_OPAQUE_V(x) asm volatile("" : "+v"(x))
/* the same for a whole register-resident row: values derived from it before this
 * point (compare masks, partial products) cannot be reused after it */
#define CSS_OPAQUE_ROW(R)                                   \
  do {                                                      \
    _Pragma("unroll") for (int j_ = 0; j_ < MP; ++j_) CSS_OPAQUE_V(R[j_]); \
  } while (0)

/* x86 cvttsd2si: NaN and out-of-range values give INT_MIN */
__device__ __forceinline__ double x86_int(double v) {
  return (v > -2147483649.0 && v < 2147483648.0) ? (double)(int)v : (double)INT_MIN;
}

/* wave64 reductions over DPP (quad_perm, row_ror, row_bcast): the total lands in
 * lane 63 and is read back as a wave-uniform scalar, so every lane holds the same
 * bits and control flow that depends on it stays uniform. */
/* Lanes a row_mask leaves unwritten keep an undefined value (mov_dpp, no "old"
 * operand, so no register has to be zeroed before every DPP move): every
 * reduction below reads its result from lane 63, which only ever combines
 * written lanes; full-mask steps write every lane. */
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp32(uint32_t v, uint32_t ident) {
  (void)ident;
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, ROWMASK, 0xF, false);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp64(double v, double ident) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v), id = __builtin_bit_cast(uint64_t, ident);
  const uint32_t lo = dpp32<CTRL, ROWMASK>((uint32_t)u, (uint32_t)id);
  const uint32_t hi = dpp32<CTRL, ROWMASK>((uint32_t)(u >> 32), (uint32_t)(id >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double lane63(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 63);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
/* v of a wave-uniform lane */
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
/* The lane id, produced by an asm statement so the compiler can neither hoist it nor
 * carry it across the unrolled Householder steps: the row index and the LDS addresses
 * derived from it are rebuilt per step (a few VALU) instead of being kept live through
 * all of them, which at the register limit got them spilled to scratch and reloaded
 * on the serial chain of every step. */
__device__ __forceinline__ int css_lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
struct OpSum {
  static __device__ __forceinline__ double id() { return 0.0; }
  static __device__ __forceinline__ double op(double x, double y) { return x + y; }
};
struct OpMin {
  static __device__ __forceinline__ double id() { return __builtin_huge_val(); }
  static __device__ __forceinline__ double op(double x, double y) { return fmin(x, y); }
};
struct OpMax {
  static __device__ __forceinline__ double id() { return -__builtin_huge_val(); }
  static __device__ __forceinline__ double op(double x, double y) { return fmax(x, y); }
};
template <class Op>
__device__ __forceinline__ double wave_reduce(double v) {
  const double e = Op::id();
  v = Op::op(v, dpp64<0xB1, 0xF>(v, e));
  v = Op::op(v, dpp64<0x4E, 0xF>(v, e));
  v = Op::op(v, dpp64<0x124, 0xF>(v, e));
  v = Op::op(v, dpp64<0x128, 0xF>(v, e));
  v = Op::op(v, dpp64<0x142, 0xA>(v, e));
  v = Op::op(v, dpp64<0x143, 0xC>(v, e));
  return lane63(v);
}
/* two sums at once (independent DPP chains interleave) */
__device__ __forceinline__ void wave_sum2(double &a, double &b) {
  a += dpp64<0xB1, 0xF>(a, 0.0);
  b += dpp64<0xB1, 0xF>(b, 0.0);
  a += dpp64<0x4E, 0xF>(a, 0.0);
  b += dpp64<0x4E, 0xF>(b, 0.0);
  a += dpp64<0x124, 0xF>(a, 0.0);
  b += dpp64<0x124, 0xF>(b, 0.0);
  a += dpp64<0x128, 0xF>(a, 0.0);
  b += dpp64<0x128, 0xF>(b, 0.0);
  a += dpp64<0x142, 0xA>(a, 0.0);
  b += dpp64<0x142, 0xA>(b, 0.0);
  a += dpp64<0x143, 0xC>(a, 0.0);
  b += dpp64<0x143, 0xC>(b, 0.0);
  a = lane63(a);
  b = lane63(b);
}

/* all-reduce over each 16-lane DPP row (every stage combines a lane with its mirror image,
 * so every lane of the row ends with the same bits) and over each 32-lane half (the two rows
 * traded by v_permlane16_swap): VALU latency per stage instead of an LDS round trip per
 * __shfl_xor */
template <class Op>
__device__ __forceinline__ double row_allreduce(double v) {
  v = Op::op(v, dpp64<0xB1, 0xF>(v, 0.0));  /* quad_perm [1,0,3,2] */
  v = Op::op(v, dpp64<0x4E, 0xF>(v, 0.0));  /* quad_perm [2,3,0,1] */
  v = Op::op(v, dpp64<0x141, 0xF>(v, 0.0)); /* row_half_mirror */
  return Op::op(v, dpp64<0x140, 0xF>(v, 0.0)); /* row_mirror */
}
template <class Op>
__device__ __forceinline__ double half_allreduce(double v) {
  v = row_allreduce<Op>(v);
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  return Op::op(__builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]),
                __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]));
}

/* block reductions over NW waves; red must hold 2*NW doubles */
template <int NW, class Op>
__device__ __forceinline__ double block_reduce(double v, double *red) {
  v = wave_reduce<Op>(v);
  if constexpr (NW == 1) {
    return v;
  } else {
    __syncthreads();
    if (css_lane_now() == 0) red[__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6] = v;
    __syncthreads();
    double s = red[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) s = Op::op(s, red[k]);
    return s;
  }
}
template <int NW>
__device__ __forceinline__ double block_sum(double v, double *red) {
  return block_reduce<NW, OpSum>(v, red);
}
template <int NW>
__device__ __forceinline__ void block_sum2(double &a, double &b, double *red) {
  wave_sum2(a, b);
  if constexpr (NW > 1) {
    __syncthreads();
    if (css_lane_now() == 0) {
      const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
      red[wv] = a;
      red[NW + wv] = b;
    }
    __syncthreads();
    double sa = red[0], sb = red[NW];
#pragma unroll
    for (int k = 1; k < NW; ++k) {
      sa += red[k];
      sb += red[NW + k];
    }
    a = sa;
    b = sb;
  }
}

/* 1/x to full precision: hardware estimate + two Newton steps (no IEEE division
 * sequence; used only off the bit-exact path) */
__device__ __forceinline__ double fast_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
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
  const int t = threadIdx.x, ab = a * b, m = a + b;
  const float invb = 1.0f / (float)b;
  const gd_randint db = gd_randint_make((uint32_t)(b > 1 ? b : 2)); /* exact q / b above 2^14 pairs */
  double bet = 0, win = 0;
  for (int q = t; q < ab; q += NT) {
    const int ii = ab <= (1 << 14) ? (int)(((float)q + 0.5f) * invb) /* exact for q < 2^14 */
                                   : (b == 1 ? q : (int)(__umulhi((uint32_t)q, db.magic) >> db.shift));
    const int jj = q - ii * b;
    bet += dist(tracks[ii], tracks[a + jj]);
  }
  /* consecutive pairs only (Q8), each pre-divided by its group's a^2 (a-1) */
  for (int k = t; k < m - 1; k += NT) {
    if (k < a - 1) win += dist(tracks[k], tracks[k + 1]) / (double)(a * a * (a - 1));
    if (k >= a) win += dist(tracks[k], tracks[k + 1]) / (double)(b * b * (b - 1));
  }
  block_sum2<NW>(bet, win, red);
  return bet / (a * b) - (a + b) * win;
}

/* The two largest eigenvalues of T by 33-section bisection, one half-wave per
 * eigenvalue (lanes 0..63 of one wave).  Sturm counts come from the sign changes of
 * the leading principal minors p_k(x) (three-term recurrence, rescaled every 4
 * steps): no division on the serial chain.  d (s_d) and e^2 (s_e2, e_{k-1}^2 at k,
 * s_e2[0] = 0) are padded to a multiple of 4 with decoupled entries above the
 * spectrum. */
template <bool PREFETCH = false>
__device__ __forceinline__ void bisect_top2(int m, double glo, double ghi, double bis_tol, const double *s_d,
                                            const double *s_e2, double *s_lam, int lane) {
  const int m4 = (m + 3) & ~3;
  const int hh = lane >> 5, j = lane & 31;
  const int target = m - 1 - hh; /* ascending index of the eigenvalue */
  double l = glo, u = ghi;
#ifdef GD_CSS_SKIP_BISECT
  for (int it = 0; it < 0; ++it) {
#else
  for (int it = 0; it < 80; ++it) {
#endif
    const double x = l + (u - l) * ((double)(j + 1) * (1.0 / 33.0));
    /* d and e^2 are padded to a multiple of 4 with decoupled entries above the
     * spectrum, so the unrolled groups need no tail */
    double pm = 1.0, pc = 1.0;
    int cnt = 0;
    double2 d01 = *reinterpret_cast<const double2 *>(s_d);
    double2 d23 = *reinterpret_cast<const double2 *>(s_d + 2);
    double2 e01 = *reinterpret_cast<const double2 *>(s_e2);
    double2 e23 = *reinterpret_cast<const double2 *>(s_e2 + 2);
    for (int k = 0; k < m4; k += 4) {
      if constexpr (!PREFETCH) {
        d01 = *reinterpret_cast<const double2 *>(s_d + k);
        d23 = *reinterpret_cast<const double2 *>(s_d + k + 2);
        e01 = *reinterpret_cast<const double2 *>(s_e2 + k);
        e23 = *reinterpret_cast<const double2 *>(s_e2 + k + 2);
      }
      /* PREFETCH (k_css_mds_t80): the next group's operands are loaded first */
      double2 nd01 = d01, nd23 = d23, ne01 = e01, ne23 = e23;
      if constexpr (PREFETCH) {
        const int kn = k + 4 < m4 ? k + 4 : k;
        nd01 = *reinterpret_cast<const double2 *>(s_d + kn);
        nd23 = *reinterpret_cast<const double2 *>(s_d + kn + 2);
        ne01 = *reinterpret_cast<const double2 *>(s_e2 + kn);
        ne23 = *reinterpret_cast<const double2 *>(s_e2 + kn + 2);
      }
      const double dk[4] = {d01.x, d01.y, d23.x, d23.y};
      const double ek[4] = {e01.x, e01.y, e23.x, e23.y}; /* e_{k-1}^2, s_e2[0] = 0 */
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        double pn = fma(dk[uu] - x, pc, -(ek[uu] * pm));
        /* an exactly zero minor takes the sign opposite to its predecessor */
        pn = (pn == 0.0) ? -pc * DBL_MIN : pn;
        cnt += (int)((__double2hiint(pn) ^ __double2hiint(pc)) < 0);
        pm = pc;
        pc = pn;
      }
      const int ex = __builtin_amdgcn_frexp_exp(fmax(fabs(pm), fabs(pc)));
      pm = __builtin_amdgcn_ldexp(pm, -ex);
      pc = __builtin_amdgcn_ldexp(pc, -ex);
      d01 = nd01;
      d23 = nd23;
      e01 = ne01;
      e23 = ne23;
    }
    double nl = cnt <= target ? x : l;
    double nu = cnt <= target ? u : x;
    /* half-wave max / min */
    nl = half_allreduce<OpMax>(nl);
    nu = half_allreduce<OpMin>(nu);
    const bool same = (nl == l && nu == u);
    l = nl;
    u = nu;
    /* a shift within CSS_BISECT_TOL ||T|| is all inverse iteration needs (its two
     * solves gain (shift error / gap)^2 on the eigenvector); the eigenvalue itself
     * comes back to rounding as the Rayleigh quotient below */
    const bool conv = same || (u - l) <= bis_tol;
    if (__all(conv)) break;
  }
  if (j == 0) s_lam[hh] = 0.5 * (l + u);
}

/* eigenvector e of T (0: largest, 1: second): partial-pivot LU of T - lam_e I (U in
 * s_lu[e], multipliers in s_x + e MP, pivots in s_piv[e]) and the start vector in
 * s_y[e]; one lane.  The serial chain carries its running values in registers; LDS
 * holds only read-once factors. */
template <int MP>
__device__ __forceinline__ void invit_factor(int m, int e, const double *s_d, const double *s_e, const double *s_lam,
                                             double (*s_lu)[3][MP], double *s_x, uint8_t (*s_piv)[MP],
                                             double (*s_y)[MP]) {
  const double sig = s_lam[e];
  double *U0 = s_lu[e][0], *U1 = s_lu[e][1], *U2 = s_lu[e][2];
  double *ml = s_x + e * MP; /* elimination multipliers; s_x is free until X is formed */
  uint8_t *pv = s_piv[e];
  double cc0 = s_d[0] - sig, cc1 = m > 1 ? s_e[0] : 0.0;
  /* four steps' operands are loaded together: the stores of a block cannot be crossed
   * by the compiler, so a load per step would wait out its LDS latency on the chain */
  for (int k0 = 0; k0 < m - 1; k0 += 4) {
    double n0v[4], n1v[4], n2v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = min(k0 + u, MP - 2);
      n0v[u] = s_e[k];
      n1v[u] = s_d[k + 1] - sig;
      n2v[u] = (k0 + u + 2 < m) ? s_e[k + 1] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u;
      if (k < m - 1) {
        const double n0 = n0v[u], n1 = n1v[u], n2 = n2v[u];
        const bool sw = fabs(cc0) < fabs(n0);
        const double pvt = sw ? n0 : cc0, oth = sw ? cc0 : n0;
        const double t = (pvt != 0.0) ? oth * fast_rcp(pvt) : 0.0;
        U0[k] = pvt;
        U1[k] = sw ? n1 : cc1;
        U2[k] = sw ? n2 : 0.0;
        ml[k] = t;
        pv[k] = sw;
        const double nc0 = sw ? fma(-t, n1, cc1) : fma(-t, cc1, n1);
        cc1 = sw ? -t * n2 : n2;
        cc0 = nc0;
      }
    }
  }
  U0[m - 1] = cc0;
  /* start vector: deterministic, not orthogonal to anything in practice */
  for (int k = 0; k < m; ++k) {
    const double f = (double)((k * 40503u + 977u * (unsigned)(e + 1)) & 1023u) / 1024.0;
    s_y[e][k] = (e == 0 ? 1.0 : ((k & 1) ? -1.0 : 1.0)) * (0.5 + f);
  }
}

/* one inverse-iteration solve (T - lam_e I) y = y with the factors of invit_factor, in
 * place in s_y[e]; one lane */
template <int MP>
__device__ __forceinline__ void invit_solve(int m, int e, double (*s_lu)[3][MP], const double *s_x,
                                            uint8_t (*s_piv)[MP], double (*s_y)[MP]) {
  double *y = s_y[e];
  const double *R0 = s_lu[e][0], *U1 = s_lu[e][1], *U2 = s_lu[e][2], *ml = s_x + e * MP;
  const uint8_t *pv = s_piv[e];
  double yk = y[0];
  /* operands four steps at a time (invit_factor); y[k + 1] is read before any store
   * reaches it */
  for (int k0 = 0; k0 < m - 1; k0 += 4) {
    double ynv[4], mlv[4];
    int pvv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = min(k0 + u, MP - 2);
      ynv[u] = y[k + 1];
      mlv[u] = ml[k];
      pvv[u] = pv[k];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u;
      if (k < m - 1) {
        double yn = ynv[u];
        if (pvv[u]) {
          const double t = yk;
          yk = yn;
          yn = t;
        }
        y[k] = yk;
        yk = fma(-mlv[u], yk, yn);
      }
    }
  }
  double z1 = yk * R0[m - 1], z2 = 0.0;
  y[m - 1] = z1;
  for (int k0 = m - 2; k0 >= 0; k0 -= 4) {
    double yv[4], u1v[4], u2v[4], r0v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = max(k0 - u, 0);
      yv[u] = y[k];
      u1v[u] = U1[k];
      u2v[u] = U2[k];
      r0v[u] = R0[k];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 - u;
      if (k >= 0) {
        const double z0 = (yv[u] - u1v[u] * z1 - u2v[u] * z2) * r0v[u];
        y[k] = z0;
        z2 = z1;
        z1 = z0;
      }
    }
  }
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
    beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
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
      beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
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
        beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
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

/* sum over the 4 lanes of a quad (every lane gets the same bits) */
__device__ __forceinline__ double quad_sum(double x) {
  x += dpp64<0xB1, 0xF>(x, 0.0); /* quad_perm [1,0,3,2] */
  return x + dpp64<0x4E, 0xF>(x, 0.0); /* quad_perm [2,3,0,1] */
}

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
  constexpr int TG = 2, S0 = (K + 1) / 4 / TG * TG; /* tail groups of TG column quads */
  double ct[TG], ctr[TG];
  double2 ctv[TG];
#pragma unroll
  for (int u = 0; u < TG; ++u) {
    const int j = 4 * (S0 + u) + tq;
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
        const int j = 4 * (sg + TG + u) + tq;
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
  const bool row = i < m, trow = R < m;
  const double xi = (i > K + 1 && row) ? c.r : 0.0;
  const double xr = (R > K + 1 && trow) ? c.rt : 0.0;
  /* |x|^2 and r^T A r in one reduction; a tail row counts once */
  double sigma = xi * xi + (tq == 0 ? xr * xr : 0.0);
  double q = ((i > K && row) ? c.r * c.p : 0.0) + ((tq == 0 && R > K && trow) ? c.rt * c.pt : 0.0);
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
    beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
    const double rr = fast_rcp(beta * (alpha - beta));
    tau = -(alpha - beta) * (alpha - beta) * rr;
    scale = beta * rr;
  }
  const double Kc = -0.5 * tau * (tau * scale * scale) * fma(beta, fma(beta, a11, -2.0 * pr1), q);
  const double ak1 = A[K + 1];
  const double vi = (i == K + 1) ? 1.0 : xi * scale;
  const double pi = (i > K && row) ? (tau * scale) * fma(-beta, ak1, c.p) : 0.0;
  const double wi = fma(Kc, vi, pi);
  const double akt = s_tail[tr][K + 1];
  const double vt = (R == K + 1) ? 1.0 : xr * scale;
  const double ptl = (R > K && trow) ? (tau * scale) * fma(-beta, akt, c.pt) : 0.0;
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
      }
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) A[jj] = (row && jj < mo) ? A[jj] : 0.0;
#pragma unroll
      for (int s = 0; s < T80_TS; ++s) {
        const int j = 4 * s + tq;
        s_tail[tr][j] = (trow && j < mo) ? (double)acct[s] : 0.0;
      }
    }

    CSS_PROF(0);
    /* ---- fill_averages (k_css_mds) */
    {
      /* the lane indices rebuilt for this phase (css_lane_now): kept live from the kernel's
       * start they were spilled at the Householder steps' register peak and reloaded here */
      const int ln_ = css_lane_now();
      const int i = ln_, tr = ln_ >> 2, tq = ln_ & 3;
      const bool row = i < m, trow = T80_MAIN + tr < m;
      int unval = 0;
      double sum = 0;
      int mo = m;
      CSS_OPAQUE_S(mo);
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) {
        if (row && jj < mo) {
          if (A[jj] < 0.00001)
            ++unval;
          else
            sum += A[jj];
        }
      }
#pragma unroll
      for (int s = 0; s < T80_TS; ++s) {
        const int j = 4 * s + tq;
        const double t = s_tail[tr][j];
        if (trow && j < mo) {
          if (t < 0.00001)
            ++unval;
          else
            sum += t;
        }
      }
      double unv = (double)unval;
      wave_sum2(unv, sum); /* sums of integers: exact in any order */
      unval = (int)unv;
      const int tot = m * m;
      if (unval > tot / 2) continue; /* discarded window: outputs untouched */
      const double avg = sum / tot;
      CSS_OPAQUE_ROW(A);
#pragma unroll
      for (int jj = 0; jj < MP; ++jj) A[jj] = fma(avg, 1.0 - fmin(A[jj], 1.0), A[jj]);
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
      for (int k = tid; k < MP + 4; k += 64) s_e2[k] = (k >= 1 && k < m) ? s_e[k - 1] * s_e[k - 1] : 0.0;
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
    bisect_top2<true>(m, glo, ghi, bis_tol, s_d, s_e2, s_lam, tid);
    __syncthreads();

    CSS_PROF(3);
    /* ---- eigenvectors of T: two steps of inverse iteration (k_css_mds) */
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
    double y1 = 0.0, y2 = 0.0, y1t = 0.0, y2t = 0.0;
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
#pragma unroll
    for (int k = MP - 3; k >= 0; --k) {
      if (k <= m - 3) {
        const double vk = row ? A[k] : 0.0;
        const double vkt = trow ? s_tail[tr][k] : 0.0;
        const double t = s_tau[k];
        double d1 = vk * y1 + (tq == 0 ? vkt * y1t : 0.0), d2 = vk * y2 + (tq == 0 ? vkt * y2t : 0.0);
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

/* the Householder scalars of one window from its reduced |x|^2 (sigma), r^T A r (q),
 * (A r)_{K+1} (pr1) and A_{K+1,K+1} (a11) -- hh_step_static's recurrences */
__device__ __forceinline__ void hh_scalars(double alpha, double sigma, double q, double pr1, double a11, double *tau,
                                           double *beta, double *scale, double *Kc) {
  double t = 0.0, be = alpha, sc = 0.0;
  if (sigma != 0.0) {
    be = -copysign(sqrt(alpha * alpha + sigma), alpha);
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
        pn = (pn == 0.0) ? -pc * DBL_MIN : pn;
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
template <class Op>
__device__ __forceinline__ void half_reduce2(double &a, double &b) {
  a = Op::op(a, dpp64<0xB1, 0xF>(a, 0.0)); /* quad_perm [1,0,3,2] */
  b = Op::op(b, dpp64<0xB1, 0xF>(b, 0.0));
  a = Op::op(a, dpp64<0x4E, 0xF>(a, 0.0)); /* quad_perm [2,3,0,1] */
  b = Op::op(b, dpp64<0x4E, 0xF>(b, 0.0));
  a = Op::op(a, dpp64<0x141, 0xF>(a, 0.0)); /* row_half_mirror: quad 0 <-> quad 1 of each 8 */
  b = Op::op(b, dpp64<0x141, 0xF>(b, 0.0));
  a = Op::op(a, dpp64<0x140, 0xF>(a, 0.0)); /* row_mirror: the two 8-lane groups of a row */
  b = Op::op(b, dpp64<0x140, 0xF>(b, 0.0));
  /* rows 0 + 1 and 2 + 3: both operands of the swap are the row sums, so lane i of row 0
   * and lane i of row 1 add the same two values in the same order */
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const auto al = __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ua, false, false);
  const auto ah = __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ua >> 32), false, false);
  const auto bl = __builtin_amdgcn_permlane16_swap((uint32_t)ub, (uint32_t)ub, false, false);
  const auto bh = __builtin_amdgcn_permlane16_swap((uint32_t)(ub >> 32), (uint32_t)(ub >> 32), false, false);
  a = Op::op(__builtin_bit_cast(double, ((uint64_t)ah[0] << 32) | al[0]),
             __builtin_bit_cast(double, ((uint64_t)ah[1] << 32) | al[1]));
  b = Op::op(__builtin_bit_cast(double, ((uint64_t)bh[0] << 32) | bl[0]),
             __builtin_bit_cast(double, ((uint64_t)bh[1] << 32) | bl[1]));
}
__device__ __forceinline__ void half_sum2(double &a, double &b) { half_reduce2<OpSum>(a, b); }

/* a half-uniform value of lane L of each half (L wave-uniform) */
__device__ __forceinline__ double half_lane(double v, int L, bool h) {
  const double v0 = readlane_f64(v, L), v1 = readlane_f64(v, 32 + L);
  return h ? v1 : v0;
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
  constexpr int FB = 4; /* columns per pinned group */
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
  const int mine = h ? M[1] : M[0];
  const bool row = r < mine, trow = R < mine;
  const double xi = (r > K + 1 && row) ? c.r : 0.0;
  const double xr = (R > K + 1 && trow) ? c.rt : 0.0;
  /* |x|^2 and r^T A r of each window in one half-wave sum; a tail row counts once */
  double sigma = xi * xi + (tq == 0 ? xr * xr : 0.0);
  double q = ((r > K && row) ? c.r * c.p : 0.0) + ((tq == 0 && R > K && trow) ? c.rt * c.pt : 0.0);
  half_sum2(sigma, q);
  double alpha, pr1, a11;
  if constexpr (K + 1 < H40_MAIN) {
    alpha = half_lane(c.r, K + 1, h);
    pr1 = half_lane(c.p, K + 1, h);
    a11 = half_lane(A[K + 1], K + 1, h);
  } else {
    alpha = half_lane(c.rt, 4 * (K + 1 - H40_MAIN), h);
    pr1 = half_lane(c.pt, 4 * (K + 1 - H40_MAIN), h);
    a11 = s_tail[hi][K + 1 - H40_MAIN][K + 1];
  }
  double tau, beta, scale, Kc;
  hh_scalars(alpha, sigma, q, pr1, a11, &tau, &beta, &scale, &Kc);
  const double ak1 = A[K + 1];
  const double vi = (r == K + 1) ? 1.0 : xi * scale;
  const double pi = (r > K && row) ? (tau * scale) * fma(-beta, ak1, c.p) : 0.0;
  const double wi = fma(Kc, vi, pi);
  const double akt = s_tail[hi][tr][K + 1];
  const double vt = (R == K + 1) ? 1.0 : xr * scale;
  const double ptl = (R > K && trow) ? (tau * scale) * fma(-beta, akt, c.pt) : 0.0;
  const double wt = fma(Kc, vt, ptl);
  double wk1;
  if constexpr (K + 1 < H40_MAIN)
    wk1 = half_lane(wi, K + 1, h);
  else
    wk1 = half_lane(wt, 4 * (K + 1 - H40_MAIN), h);
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
    int un = 0;
    double sm = 0;
    int mo = mm;
    CSS_OPAQUE_V(mo);
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
    for (int s = 0; s < H40_TS; ++s) {
      const int j = 4 * s + tq;
      const double t = s_tail[hi][tr][j];
      if (trow && j < mo) {
        if (t < 0.00001)
          ++un;
        else
          sm += t;
      }
    }
    double us = (double)un, ss = sm;
    half_sum2(us, ss); /* sums of integers: exact in any order */
    const double u2[2] = {readlane_f64(us, 0), readlane_f64(us, 32)};
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      if (M[x] != 0 && (int)u2[x] > (M[x] * M[x]) / 2) M[x] = 0; /* discarded window: outputs untouched */
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
      s_u.a.e2[x][kk] = (kk >= 1 && kk < M[x]) ? s_e[x][kk - 1] * s_e[x][kk - 1] : 0.0;
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
  p40_bisect(M[0], M[1], glo, ghi, btol, s_d, s_u.a.e2, s_lam, lane);
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
    y1 = rowk ? s_u.b.y[hi][0][r] : 0.0;
    y2 = rowk ? s_u.b.y[hi][1][r] : 0.0;
    y1t = trowk ? s_u.b.y[hi][0][R] : 0.0;
    y2t = trowk ? s_u.b.y[hi][1][R] : 0.0;
    double n1 = y1 * y1 + (tq == 0 ? y1t * y1t : 0.0), n2 = y2 * y2 + (tq == 0 ? y2t * y2t : 0.0);
    half_sum2(n1, n2);
    const double r1 = 1.0 / sqrt(n1), r2 = 1.0 / sqrt(n2);
    y1 *= r1;
    y2 *= r2;
    y1t *= r1;
    y2t *= r2;
    __syncthreads();
    if (itn == 0) {
      if (rowk) {
        s_u.b.y[hi][0][r] = y1;
        s_u.b.y[hi][1][r] = y2;
      }
      if (tq == 0 && trowk) {
        s_u.b.y[hi][0][R] = y1t;
        s_u.b.y[hi][1][R] = y2t;
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
#pragma unroll
  for (int k = MP - 3; k >= 0; --k) {
    const bool liveA = k <= M[0] - 3, liveB = k <= M[1] - 3;
    if (liveA || liveB) {
      const bool mine = h ? liveB : liveA;
      const double vk = (rowk && mine) ? A[k] : 0.0;
      const double vkt = (trowk && mine) ? s_tail[hi][tr][k] : 0.0;
      const double t = mine ? s_tau[hi][k] : 0.0;
      double d1 = vk * y1 + (tq == 0 ? vkt * y1t : 0.0);
      double d2 = vk * y2 + (tq == 0 ? vkt * y2t : 0.0);
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
        beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
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

/* ------------------------------------------------------------------------ */
int gd_css_tier(int m) {
  static const int tiers[] = {24, 40, 64, 80, 96, 128};
  for (int t : tiers)
    if (m <= t) return t;
  /* the general path: any tier value above GD_CSS_TIER_MAX, the xbuf row width / 2 */
  if (m <= GD_CSS_BIG_MAX) return (m + 7) & ~7;
  return 0;
}

static int launch_big(int mp, const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, double *slab, hipStream_t s) {
  const int ld = gd_css_big_ld(mp);
  const int64_t per = gd_css_big_slab_per_wg(mp), grid = gd_css_big_grid(wtotal, mp);
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

static int launch_p40(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s) {
#if CSS_H40
  hipLaunchKernelGGL(k_css_mds_h40, dim3((unsigned)((wtotal + 1) / 2)), dim3(64), 0, s, d_ch, nchrom, d_pl, planes,
                     lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x, force_literal, scores, p, xbuf, status, flags);
#else
  hipLaunchKernelGGL(k_css_mds_p40, dim3((unsigned)((wtotal + 1) / 2)), dim3(64), 0, s, d_ch, nchrom, d_pl, planes,
                     lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x, force_literal, scores, p, xbuf, status, flags);
#endif
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

static int launch_t80(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                      const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                      double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s) {
  hipLaunchKernelGGL(k_css_mds_t80, dim3((unsigned)wtotal), dim3(64), 0, s, d_ch, nchrom, d_pl, planes, lo_a, hi_a,
                     lo_b, avals, bvals, wtotal, want_x, force_literal, scores, p, xbuf, status, flags);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

template <int MP, int G>
static int launch_tier(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl, const uint32_t *planes,
                       const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                       const double *bvals, int64_t wtotal, int want_x, int force_literal, double *scores, double *p,
                       double *xbuf, uint8_t *status, unsigned *flags, hipStream_t s) {
  constexpr int NT = CssShape<MP, G>::NT;
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
#ifdef GD_CSS_PROFILE
  {
    static const unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_css_prof), z, sizeof z, 0, hipMemcpyHostToDevice, s);
  }
  struct Dump {
    hipStream_t s;
    ~Dump() {
      unsigned long long h[8];
      (void)hipStreamSynchronize(s);
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_css_prof), sizeof h);
      fprintf(stderr, "css-prof cycles: D %llu fill+center %llu tridiag %llu bisect %llu invit %llu back %llu score %llu\n",
              h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
    }
  } dump{s};
#endif
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
          st = launch_p40(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x1, force_literal,
                          scores, p, xbuf, status, flags, s);
          break;
#else
        CSS_TIER(40, 1)
#endif
        CSS_TIER(64, 1)
#if CSS_T80
        case 80:
          st = launch_t80(d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x1, force_literal,
                          scores, p, xbuf, status, flags, s);
          break;
#else
        CSS_TIER(80, CSS_G80)
#endif
        CSS_TIER(96, 2)
        CSS_TIER(128, 2)
        default:
          if (mp <= GD_CSS_TIER_MAX || mp > GD_CSS_BIG_MAX) return GD_ERR_SIZE;
          st = launch_big(mp, d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, wtotal, want_x1, force_literal,
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
