#pragma once
/*
 * gd_css_common.h -- device helpers shared by the CSS MDS kernels (statistics/css/).
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
static __device__ unsigned long long g_css_prof[8];
/* each kernel's translation unit owns its counters: reset before a launch, dumped
 * after it (CSS_PROF_LAUNCH in the launcher) */
struct CssProfDump {
  hipStream_t s;
  explicit CssProfDump(hipStream_t s_) : s(s_) {
    static const unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_css_prof), z, sizeof z, 0, hipMemcpyHostToDevice, s);
  }
  ~CssProfDump() {
    unsigned long long h[8];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_css_prof), sizeof h);
    fprintf(stderr, "css-prof cycles: D %llu fill+center %llu tridiag %llu bisect %llu invit %llu back %llu score %llu\n",
            h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
  }
};
#define CSS_PROF_LAUNCH(s) CssProfDump css_prof_dump_(s)
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
#define CSS_PROF_LAUNCH(s)
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
#ifndef CSS_TWIST
#define CSS_TWIST 1 /* eigenvectors by twisted factorisations (0: pivoted-LU inverse iteration only) */
#endif
#define CSS_E2_FLOOR 1e-300 /* floor of e_k^2 in the Sturm arrays (bisect_top2<.., false>, twisted_top2) */
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
/* v_cndmask_b32 with a constant lane mask in SGPRs: lanes whose bit is set take t, the
 * others f (no compare, no VCC) */
__device__ __forceinline__ double sel_mask(double f, double t, uint64_t mask) {
  const uint64_t uf = __builtin_bit_cast(uint64_t, f), ut = __builtin_bit_cast(uint64_t, t);
  uint32_t lo, hi;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(lo) : "v"((uint32_t)uf), "v"((uint32_t)ut), "s"(mask));
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(uf >> 32)), "v"((uint32_t)(ut >> 32)), "s"(mask));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
/* f64 all-reduce step across the two 16-lane rows of each 32-lane half (permlane16_swap)
 * and across the two halves (permlane32_swap): both operands of a swap are the same
 * value, so partners add the same two numbers */
__device__ __forceinline__ double swap16_sum(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const auto l = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  return __builtin_bit_cast(double, ((uint64_t)h[0] << 32) | l[0]) +
         __builtin_bit_cast(double, ((uint64_t)h[1] << 32) | l[1]);
}
__device__ __forceinline__ double swap32_sum(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const auto l = __builtin_amdgcn_permlane32_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto h = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  return __builtin_bit_cast(double, ((uint64_t)h[0] << 32) | l[0]) +
         __builtin_bit_cast(double, ((uint64_t)h[1] << 32) | l[1]);
}
#ifndef CSS_SUM2_LDS
#define CSS_SUM2_LDS 0 /* measured slower (C4 9.92 -> 9.62 M windows/s): LDS latency on the chain */
#endif
/* Two wave sums in ONE reduction chain.  The first step splits the work by lane bit 3:
 * lanes 0-7 of every row keep a, lanes 8-15 keep b, and each lane receives the value of its
 * class from its row_mirror partner (lane 15 - i, the other class).  The remaining steps
 * (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror = lane ^ 7, then the row and half swaps)
 * never cross bit 3, so each lane ends with the full sum of its class and every lane of a
 * class holds the same bits (each step adds the same two values on both partners).  26 VALU
 * where two separate DPP chains took 40. */
__device__ __forceinline__ void wave_sum2(double &a, double &b) {
  constexpr uint64_t B3 = 0xFF00FF00FF00FF00ull; /* lanes with bit 3 set: class b */
  double v = sel_mask(a, b, B3);
  const double send = sel_mask(b, a, B3);
  v += dpp64<0x140, 0xF>(send, 0.0); /* row_mirror */
  v += dpp64<0xB1, 0xF>(v, 0.0);     /* quad_perm [1,0,3,2] */
  v += dpp64<0x4E, 0xF>(v, 0.0);     /* quad_perm [2,3,0,1] */
  v += dpp64<0x141, 0xF>(v, 0.0);    /* row_half_mirror */
#if CSS_SUM2_LDS
  /* the cross-row steps through the LDS crossbar (ds_swizzle lane ^ 16, ds_bpermute lane ^ 32):
   * one VALU add each instead of two copies, two swaps and the add */
  {
    uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t l16 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)u, 0x401F);
    const uint32_t h16 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(u >> 32), 0x401F);
    v += __builtin_bit_cast(double, ((uint64_t)h16 << 32) | l16);
    u = __builtin_bit_cast(uint64_t, v);
    const int src = (int)((__lane_id() ^ 32u) << 2);
    const uint32_t l32 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)u);
    const uint32_t h32 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(u >> 32));
    v += __builtin_bit_cast(double, ((uint64_t)h32 << 32) | l32);
  }
#else
  v = swap32_sum(swap16_sum(v));
#endif
  a = readlane_f64(v, 0);
  b = readlane_f64(v, 8);
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

/* sqrt of a positive normal x: the hardware reciprocal-sqrt estimate and the Newton
 * corrections of the compiler's sqrt sequence, without its zero / infinity / denormal
 * handling (ldexp scaling, class test, selects): 10 VALU instead of 17.  Callers guarantee
 * x > 0 (the Householder steps form it only for sigma != 0) */
__device__ __forceinline__ double sqrt_pos(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  double s = x * r, h = 0.5 * r;
  const double e = fma(-h, s, 0.5);
  s = fma(s, e, s);
  h = fma(h, e, h);
  double d = fma(-s, s, x);
  s = fma(d, h, s);
  d = fma(-s, s, x);
  return fma(d, h, s);
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
/* ZFIX = false: the serial chain is the FMA alone.  An exactly zero minor then counts as
 * positive (one sign change across it and its successor -e^2 p_{k-1} either way), which
 * needs every e_k^2 of the matrix floored at CSS_E2_FLOOR (a zero minor followed by e^2 = 0
 * would zero the rest of the chain); the floor moves no eigenvalue by more than 1e-150. */
template <bool PREFETCH = false, bool ZFIX = true>
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
        if constexpr (ZFIX) pn = (pn == 0.0) ? -pc * DBL_MIN : pn;
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
 * s_lu[slot], multipliers in s_x + slot MP, pivots in s_piv[slot]) and the start vector in
 * s_y[slot], slot = e unless given (one eigenvector at a time in one buffer); one lane.  The serial chain carries its running values in registers; LDS
 * holds only read-once factors. */
template <int MP>
__device__ __forceinline__ void invit_factor(int m, int e, const double *s_d, const double *s_e, const double *s_lam,
                                             double (*s_lu)[3][MP], double *s_x, uint8_t (*s_piv)[MP],
                                             double (*s_y)[MP], int slot = -1) {
  const int sl = slot < 0 ? e : slot;
  const double sig = s_lam[e];
  double *U0 = s_lu[sl][0], *U1 = s_lu[sl][1], *U2 = s_lu[sl][2];
  double *ml = s_x + sl * MP; /* elimination multipliers; s_x is free until X is formed */
  uint8_t *pv = s_piv[sl];
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
    s_y[sl][k] = (e == 0 ? 1.0 : ((k & 1) ? -1.0 : 1.0)) * (0.5 + f);
  }
}

/* one inverse-iteration solve (T - lam_e I) y = y with the factors of invit_factor, in
 * place in s_y[e]; one lane */
template <int MP>
__device__ __forceinline__ void invit_solve(int m, int e, double (*s_lu)[3][MP], const double *s_x,
                                            uint8_t (*s_piv)[MP], double (*s_y)[MP]) { /* e: the slot */
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

/* two all-reduces over each 32-lane half at once (every lane of a half ends with the same bits) */
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
#ifndef CSS_HALF_SPLIT
#define CSS_HALF_SPLIT 1
#endif
/* two sums over each 32-lane half, every lane of a half ending with both (the same bits):
 * CSS_HALF_SPLIT runs them as ONE chain split by lane bit 3 (wave_sum2's scheme), then the
 * row_mirror partner hands each lane the other class's sum -- 27 VALU instead of 34 */
__device__ __forceinline__ void half_sum2(double &a, double &b) {
#if CSS_HALF_SPLIT
  constexpr uint64_t B3 = 0xFF00FF00FF00FF00ull;
  double v = sel_mask(a, b, B3);
  const double send = sel_mask(b, a, B3);
  v += dpp64<0x140, 0xF>(send, 0.0); /* row_mirror */
  v += dpp64<0xB1, 0xF>(v, 0.0);     /* quad_perm [1,0,3,2] */
  v += dpp64<0x4E, 0xF>(v, 0.0);     /* quad_perm [2,3,0,1] */
  v += dpp64<0x141, 0xF>(v, 0.0);    /* row_half_mirror */
  v = swap16_sum(v);
  const double o = dpp64<0x140, 0xF>(v, 0.0);
  a = sel_mask(v, o, B3);
  b = sel_mask(o, v, B3);
#else
  half_reduce2<OpSum>(a, b);
#endif
}

/* Eigenvectors of T for the shifts sig0 / sig1 (the two bisection results) by twisted
 * factorisations T - sig I = N_r Delta_r N_r^T (Parlett & Dhillon's solution of
 * Wilkinson's problem), W windows per wave (1, or 2 on the halves), rows k = lane, lane + 64/W:
 *   - the leading minors p+_k = (d_k - sig) p+_{k-1} - e_{k-1}^2 p+_{k-2} and the trailing
 *     minors p-_k: four serial chains per window (eigenvector x direction) on lanes 0..3
 *     of the window whose only dependent operation is the FMA (rescaled by a power of two
 *     every 4 steps); each step stores its minor, and the pivots D_k = p_k / p_{k-1} are
 *     formed later on every row in parallel (twist_prev: the rescale exponent is a function
 *     of the two stored minors before it, so it is recomputed, not stored);
 *   - gamma_k = D+_k + D-_k - (d_k - sig) on every row, r = argmin |gamma_k|;
 *   - z_r = 1, z_k = prod_{j=k}^{r-1} (-e_j / D+_j) above r and prod_{j=r+1}^{k} (-e_{j-1} / D-_j)
 *     below it: the multipliers on every row, the products as four segmented scans per
 *     window (16 / W lanes each: NB walking steps per lane, a DPP row_shr scan of the block
 *     products, the block applied);
 *   - sig += gamma_r / |z|^2, the Rayleigh quotient of z ((T - sig I) z = gamma_r e_r).
 * Two rounds.  From the bisection shift (within CSS_BISECT_TOL ||T||) the first gives
 * |z - q| ~ shift error / gap and a Rayleigh shift accurate to its square; the second
 * converges to rounding (worst 4e-13 against LAPACK on 6,000 synthetic 40+40 / 20+20
 * windows, where two pivoted-LU inverse-iteration solves reach 3e-12).  This replaces
 * invit_factor's pivoted elimination (compare, select, reciprocal and FMA on the chain)
 * and invit_solve's 2 x 2m steps.
 * Per window x: s_d + x sdS, s_e + x seS, s_e2 + x se2S (e_{k-1}^2 floored at CSS_E2_FLOOR
 * at k = 1 .. m - 1, 0 at k = 0 and k = m), s_lam[2x + e] the shifts; s_rev + x srS (2 MP
 * doubles of free scratch) takes d and e^2 in backward order so both chain directions walk
 * upward.  s_Q[x][e][0][k] = p+_k, s_Q[x][e][1][t] = p-_k at t = m - 1 - k; on return
 * s_Q[x][e][1][k] holds z (z_r = 1) and nz_e = |z|^2 of the lane's window.  False
 * (wave-uniform) when a pivot, multiplier or norm is not finite -- an exactly singular
 * leading or trailing minor, or a product out of range: the caller falls back to
 * pivoted-LU inverse iteration. */
__device__ __forceinline__ double dpp_shr_f64(double v, int n) { /* n = 1, 2, 4, 8 */
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  uint32_t lo, hi;
  /* lanes whose source lies before their 16-lane row keep 1.0 (the product identity) */
  switch (n) {
    case 1:
      lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)u, 0x111, 0xF, 0xF, false);
      hi = __builtin_amdgcn_update_dpp(0x3ff00000u, (uint32_t)(u >> 32), 0x111, 0xF, 0xF, false);
      break;
    case 2:
      lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)u, 0x112, 0xF, 0xF, false);
      hi = __builtin_amdgcn_update_dpp(0x3ff00000u, (uint32_t)(u >> 32), 0x112, 0xF, 0xF, false);
      break;
    case 4:
      lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)u, 0x114, 0xF, 0xF, false);
      hi = __builtin_amdgcn_update_dpp(0x3ff00000u, (uint32_t)(u >> 32), 0x114, 0xF, 0xF, false);
      break;
    default:
      lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)u, 0x118, 0xF, 0xF, false);
      hi = __builtin_amdgcn_update_dpp(0x3ff00000u, (uint32_t)(u >> 32), 0x118, 0xF, 0xF, false);
  }
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

/* the pivot p_t / p_{t-1} of a chain's step t, p_{t-1} brought to step t's scale (the chains
 * rescale after steps 3, 7, 11, ... by the exponent of max(|p_{t-2}|, |p_{t-1}|)) */
__device__ __forceinline__ double twist_pivot(const double *Q, int t) {
  const double p = Q[t];
  if (t == 0) return p;
  double q = Q[t - 1];
  if ((t & 3) == 0) q = __builtin_amdgcn_ldexp(q, -__builtin_amdgcn_frexp_exp(fmax(fabs(Q[t - 2]), fabs(q))));
  return p * fast_rcp(q);
}

template <int MP, int W>
__device__ __forceinline__ bool twisted_top2(const int *M, int lane, const double *s_d, int sdS, const double *s_e,
                                             int seS, const double *s_e2, int se2S, const double *s_lam,
                                             double (*s_Q)[2][2][MP], double *s_rev, int srS, double &nz0,
                                             double &nz1) {
  static_assert(W == 1 || W == 2, "one window per wave or per half wave");
  constexpr int G = 64 / W;               /* lanes per window */
  constexpr int NR = (MP + G - 1) / G;    /* rows per lane */
  constexpr int LS = 16 / W;              /* lanes per scan segment (4 segments per window) */
  constexpr int NB = (MP + LS - 1) / LS;  /* walking steps per scan lane */
  const int x = W == 1 ? 0 : lane / G, ll = lane % G;
  const int m = W == 1 ? M[0] : (x ? M[1] : M[0]);
  const double *dX = s_d + x * sdS, *eX = s_e + x * seS, *e2X = s_e2 + x * se2S;
  double *revX = s_rev + x * srS;
  double(*Q)[2][MP] = s_Q[x];
  double sig0 = s_lam[2 * x], sig1 = s_lam[2 * x + 1];
  for (int k = ll; k < m; k += G) {
    revX[k] = dX[m - 1 - k];
    revX[MP + k] = e2X[m - k];
  }
  __syncthreads();
  for (int rd = 0; rd < 2; ++rd) {
    /* chains: lane 2e + dir of the window, step t = row t (dir 0) or row m - 1 - t (dir 1) */
    if (ll < 4) {
      const int e = ll >> 1, dir = ll & 1;
      const double sig = e ? sig1 : sig0;
      const double *dd = dir ? revX : dX, *ee = dir ? revX + MP : e2X;
      double *out = Q[e][dir];
      const int mc = max(m, 1);
      double pm = 1.0, pc = 1.0;
      double dv[4], ev[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        dv[u] = dd[min(u, mc - 1)];
        ev[u] = ee[min(u, mc - 1)];
      }
      for (int t0 = 0; t0 < m; t0 += 4) {
        double nd[4], ne[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          nd[u] = dd[min(t0 + 4 + u, mc - 1)];
          ne[u] = ee[min(t0 + 4 + u, mc - 1)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (t0 + u < m) {
            const double pn = fma(dv[u] - sig, pc, -(ev[u] * pm));
            out[t0 + u] = pn;
            pm = pc;
            pc = pn;
          }
        }
        const int ex = __builtin_amdgcn_frexp_exp(fmax(fabs(pm), fabs(pc)));
        pm = __builtin_amdgcn_ldexp(pm, -ex);
        pc = __builtin_amdgcn_ldexp(pc, -ex);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          dv[u] = nd[u];
          ev[u] = ne[u];
        }
      }
    }
    __syncthreads();
    /* pivots of the lane's rows (registers), twist indices: the smallest |gamma_k| (a NaN
     * never compares smaller) */
    double Dp0[NR], Dm0[NR], Dp1[NR], Dm1[NR];
    double g0 = __builtin_huge_val(), g1 = __builtin_huge_val();
    int i0 = 0, i1 = 0;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const int k = ll + G * q;
      Dp0[q] = Dm0[q] = Dp1[q] = Dm1[q] = 1.0;
      if (k < m) {
        Dp0[q] = twist_pivot(Q[0][0], k);
        Dm0[q] = twist_pivot(Q[0][1], m - 1 - k);
        Dp1[q] = twist_pivot(Q[1][0], k);
        Dm1[q] = twist_pivot(Q[1][1], m - 1 - k);
        const double dk = dX[k];
        const double a0 = fabs(Dp0[q] + Dm0[q] - (dk - sig0)), a1 = fabs(Dp1[q] + Dm1[q] - (dk - sig1));
        if (a0 < g0) {
          g0 = a0;
          i0 = k;
        }
        if (a1 < g1) {
          g1 = a1;
          i1 = k;
        }
      }
    }
    double mn0 = g0, mn1 = g1;
    if constexpr (W == 1) {
      mn0 = wave_reduce<OpMin>(g0);
      mn1 = wave_reduce<OpMin>(g1);
    } else {
      half_reduce2<OpMin>(mn0, mn1);
    }
    if (__any(m > 0 && !(mn0 < __builtin_huge_val() && mn1 < __builtin_huge_val()))) return false;
    const uint64_t bl0 = __ballot(g0 == mn0), bl1 = __ballot(g1 == mn1);
    int r0, r1;
    if constexpr (W == 1) {
      r0 = __builtin_amdgcn_readlane(i0, __builtin_ctzll(bl0));
      r1 = __builtin_amdgcn_readlane(i1, __builtin_ctzll(bl1));
    } else {
      /* each half's first lane holding its minimum (a half with m = 0 has every bit set:
       * inf == inf) */
      const int a0 = __builtin_amdgcn_readlane(i0, __builtin_ctzll(bl0 | (1ull << 31)));
      const int c0 = __builtin_amdgcn_readlane(i0, 32 + __builtin_ctzll((bl0 >> 32) | (1ull << 31)));
      const int a1 = __builtin_amdgcn_readlane(i1, __builtin_ctzll(bl1 | (1ull << 31)));
      const int c1 = __builtin_amdgcn_readlane(i1, 32 + __builtin_ctzll((bl1 >> 32) | (1ull << 31)));
      r0 = x ? c0 : a0;
      r1 = x ? c1 : a1;
    }
    double gr0 = 0.0, gr1 = 0.0;
    if (m > 0) {
      gr0 = twist_pivot(Q[0][0], r0) + twist_pivot(Q[0][1], m - 1 - r0) - (dX[r0] - sig0);
      gr1 = twist_pivot(Q[1][0], r1) + twist_pivot(Q[1][1], m - 1 - r1) - (dX[r1] - sig1);
    }
    /* multipliers into Q[e][0][k] (every minor was read above): -e_k / D+_k above the twist,
     * -e_{k-1} / D-_k below it */
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const int k = ll + G * q;
      if (k < m) {
        const double ek = k + 1 < m ? eX[k] : 0.0, ekm = k > 0 ? eX[k - 1] : 0.0;
        Q[0][0][k] = k < r0 ? -ek * fast_rcp(Dp0[q]) : -ekm * fast_rcp(Dm0[q]);
        Q[1][0][k] = k < r1 ? -ek * fast_rcp(Dp1[q]) : -ekm * fast_rcp(Dm1[q]);
      }
    }
    __syncthreads();
    /* z into Q[e][1][k] by segmented scans: segment (e, dir) of the window (LS lanes) walks
     * away from r_e, NB steps per lane */
    {
      const int seg = (ll / LS) & 3, e = seg >> 1, dir = seg & 1, ls = ll % LS;
      const int r = e ? r1 : r0, cnt = m > 0 ? (dir ? m - 1 - r : r) : 0, ks = dir ? 1 : -1;
      const double *Gm = Q[e][0];
      double *Z = Q[e][1];
      double c[NB];
      double run = 1.0;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int t = NB * ls + j;
        const double g = t < cnt ? Gm[r + ks * (t + 1)] : 1.0;
        run *= g;
        c[j] = run;
      }
      double v = run;
#pragma unroll
      for (int sh = 1; sh < LS; sh <<= 1) {
        const double o = dpp_shr_f64(v, sh);
        v *= (LS == 16 || ls >= sh) ? o : 1.0;
      }
      double ex = dpp_shr_f64(v, 1); /* the product of the segment's lower lanes' blocks */
      if (LS != 16 && ls == 0) ex = 1.0;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int t = NB * ls + j;
        if (t < cnt) Z[r + ks * (t + 1)] = ex * c[j];
      }
      if (m > 0 && dir == 0 && ls == 0) Z[r] = 1.0;
    }
    __syncthreads();
    double s0 = 0.0, s1 = 0.0;
    for (int k = ll; k < m; k += G) {
      const double z0 = Q[0][1][k], z1 = Q[1][1][k];
      s0 = fma(z0, z0, s0);
      s1 = fma(z1, z1, s1);
    }
    if constexpr (W == 1)
      wave_sum2(s0, s1);
    else
      half_sum2(s0, s1);
    if (__any(m > 0 && !(s0 < __builtin_huge_val() && s1 < __builtin_huge_val()))) return false; /* NaN fails too */
    nz0 = s0;
    nz1 = s1;
    if (m > 0) {
      sig0 += gr0 / s0;
      sig1 += gr1 / s1;
    }
  }
  return true;
}

/* sum over the 4 lanes of a quad (every lane gets the same bits) */
__device__ __forceinline__ double quad_sum(double x) {
  x += dpp64<0xB1, 0xF>(x, 0.0); /* quad_perm [1,0,3,2] */
  return x + dpp64<0x4E, 0xF>(x, 0.0); /* quad_perm [2,3,0,1] */
}

}  // namespace

