/*
 * gd_css_perm.hip -- the CSS permutation test (significance_treshold, css.c:675-752)
 * on the MDS coordinates the score kernels leave in xbuf.
 *
 * One workgroup of NWV waves per window (windows pulled from a work counter: the
 * early exit makes their cost uneven), 64 * NWV permutations per pass, one per lane:
 *  1. draws: lane t of wave v (permutation q = 64 v + t of the pass) starts at draw
 *     q (m - 1) of the pass via an affine LCG jump and applies its Fisher-Yates swaps
 *     to an identity column sigma_q of its wave's LDS byte matrix (a rejected draw,
 *     probability ~m/2^31, sends the pass through the serial generator, which records
 *     each permutation's start state).
 *  2. tracks: F_q = F_{q-1} o sigma_q, 64 steps per wave, the waves in turn (the
 *     carry F between them in LDS); F is held one element per lane and gathered with
 *     ds_bpermute; F_q overwrites the dead column sigma_q.
 *  3. score of every lane's F_q: the between-group sum over the smaller group G as
 *     sum_{x in G} R_x - 2 sum_{x<y in G} S_xy (R = row sums of S), read from the
 *     packed lower triangle of S in LDS, plus the consecutive within-group pairs
 *     (Q8).  The observed score is the same function of the identity tracks, so
 *     ties are decided identically for observed and permuted scores.
 *  4. hits are counted in permutation order (one ballot per wave), so the early exit
 *     stops exactly where the serial loop would.
 * The tracks are reset to the identity per window and every window draws from its
 * own nrand48 stream (deviation 1).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_internal.h"

/* A copy of the lane id the compiler cannot see through: lane-derived addresses are
 * rebuilt inside each phase instead of being hoisted out of the window and pass
 * loops as ~100 live VGPRs. */
#define PERM_OPAQUE(x) asm volatile("" : "+v"(x))

#ifdef GD_PERM_PROFILE
/* diagnostics build only: shader-clock cycles per phase summed over workgroups (thread 0),
 * accumulated in registers and added to the global totals once per workgroup at exit (an
 * atomic per phase boundary queued behind every other workgroup's and then held up the
 * next vmcnt wait, the work queue's, which showed as queue time) */
#include <cstdio>
__device__ unsigned long long g_perm_prof[8];
#define PERM_PROF_INIT                                  \
  uint64_t prof_t = __builtin_readcyclecounter();      \
  uint64_t prof_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define PERM_PROF(ph)                                  \
  do {                                                 \
    const uint64_t t_ = __builtin_readcyclecounter(); \
    prof_acc[ph] += t_ - prof_t;                       \
    prof_t = t_;                                       \
  } while (0)
#define PERM_PROF_FLUSH                                                                           \
  do {                                                                                            \
    if (threadIdx.x == 0)                                                                         \
      for (int ph_ = 0; ph_ < 8; ++ph_) atomicAdd(&g_perm_prof[ph_], (unsigned long long)prof_acc[ph_]); \
  } while (0)
#else
#define PERM_PROF_INIT
#define PERM_PROF(ph)
#define PERM_PROF_FLUSH
#endif

namespace {

__device__ __forceinline__ int perm_chrom_of(const gd_chrom_dev *ch, int nchrom, int64_t w) {
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

/* calc_dist (css.c:573-587) of points i, j of X (m x 2, row-major) */
__device__ __forceinline__ double perm_xdist(const double *X, int i, int j) {
  const double dx = X[2 * i] - X[2 * j], dy = X[2 * i + 1] - X[2 * j + 1];
  return sqrt(dx * dx + dy * dy);
}

#ifndef PERM_CHAINS
#define PERM_CHAINS 1 /* composition chains per wave (1 or 2), see k_css_perm phase 2 */
#endif
/* Diagnostics builds for per-phase counters (tools/perm_phase_pmc.sh; outputs are wrong in
 * them): PERM_DIAG_NOEXIT runs every window's full mcR permutations (no early exit, so every
 * build does the same passes); PERM_DIAG_SKIP bit 1 skips the Fisher-Yates draws (the
 * identity permutations stay), bit 2 the compositions, bit 4 the scores (no hits). */
#ifndef PERM_DIAG_NOEXIT
#define PERM_DIAG_NOEXIT 0
#endif
#ifndef PERM_DIAG_SKIP
#define PERM_DIAG_SKIP 0
#endif
#ifndef PERM_S16_PAIRS
#define PERM_S16_PAIRS 1 /* the fp16 matrix from each unordered pair once (0: every entry) */
#endif
#ifndef PERM_MFMA
#define PERM_MFMA 1 /* the permutation score on the matrix cores up to 80 individuals */
#endif

/* Row stride of the byte matrices: row k holds byte k of every lane's column.  68
 * bytes (17 dwords, odd) put the 64 rows a composition step writes, one per lane,
 * on distinct LDS banks; 64 bytes put them all on two. */
#define PERM_ROW 68

/* waves per workgroup and the LDS carve-up */
template <int MP>
struct PermShape {
  static constexpr int TRI = MP * (MP + 1) / 2 + 1; /* packed triangle + padding row + zero */
  static constexpr int HALF = MP / 2;               /* largest smaller-group size */
#ifndef PERM_NWV_LARGE
#define PERM_NWV_LARGE 2 /* waves per workgroup above 64 individuals */
#endif
  static constexpr int NWV = MP <= 64 ? 4 : PERM_NWV_LARGE;
  static constexpr int NT = 64 * NWV;
  static constexpr int SIG = MP * PERM_ROW; /* one wave's byte matrix */
  static constexpr int MEM = HALF * 64;     /* one wave's member lists (byte k of lane l at k*64 + l) */
  /* The matrix-core score (score_mfma) for cohorts up to 80: S scaled by a power of two
   * into one fp16 matrix, MT 32-row tiles x KT 16-deep k steps of v_mfma_f32_32x32x16_f16;
   * row stride RS bytes,
   * an odd multiple of 16, so the 16-byte A-fragment reads of 16 consecutive rows hit
   * distinct bank groups */
  static constexpr bool MF = PERM_MFMA && MP <= 80;
  static constexpr int MT = (MP + 31) / 32, KT = (MP + 15) / 16;
  static constexpr int RS = KT * 32 + 16;
  /* rows of the fp16 matrix: the last row tile's rows at and past MP read row MP, which stays
   * zero (score_mfma clamps the fragment row), so the rows MP + 1 .. 32 MT - 1 take no LDS:
   * at 80 individuals 81 rows instead of 96, and with the members' serial-stream start states
   * computed per lane and no FP64-triangle alias the workgroup fits 6 per CU instead of 5 */
  static constexpr int S16ROWS = MT * 32 > MP ? MP + 1 : MT * 32;
  static constexpr int S16 = S16ROWS * RS; /* bytes of the fp16 matrix */
  /* region U: the FP64 triangle while a window is set up; then either the FP32 triangle,
   * the byte matrices and the member lists (FP32 score), or the fp16 matrix,
   * the byte matrices and the serial-stream start states (matrix-core score) */
  static constexpr int OFF_SIG = MF ? S16 : (TRI * 4 + 15) / 16 * 16;
  static constexpr int OFF_MEM = OFF_SIG + NWV * SIG;
  /* matrix-core tiers: score_exact_wave's 256-byte scratch per wave; FP32 tiers: the member
   * lists, which the serial-stream start states alias */
  static constexpr int MEMB = MF ? NWV * 256 : NWV * MEM;
  static constexpr int UBYTES = MF ? OFF_MEM + MEMB : (OFF_MEM + MEMB > TRI * 8 ? OFF_MEM + MEMB : TRI * 8);
  static_assert(MF || MEMB >= (NT + 1) * 8, "the serial-stream start states alias the member lists");
};

/* packed lower triangle with one zero row appended: pair (x, y), x != y, at
 * T(max) + min, T(h) = h(h-1)/2; index MP is a padding individual with S = 0, and
 * the pair (MP, MP) lands on the extra zero entry at the end.  Byte offsets of T(x)
 * for the FP64 (tri8) and FP32 (tri4) copies. */
__device__ __forceinline__ uint32_t tri8(uint32_t x) { return (x * (x - 1u) >> 1) << 3; }
__device__ __forceinline__ uint32_t tri4(uint32_t x) { return (x * (x - 1u) >> 1) << 2; }

/* S(x, y) for two individuals given their tri8 forms */
__device__ __forceinline__ double s_pair(const double *S, uint32_t x, uint32_t tx, uint32_t y, uint32_t ty) {
  const uint32_t off = x > y ? tx + (y << 3) : ty + (x << 3);
  return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(S) + off);
}

/* css() of one track array in FP64.  track(k): entry k of the track array; member(k):
 * member k of the smaller group G in ascending order, the padding individual MP for
 * k >= g; sxy(x, y), x < y: S(x, y) (0 when y is the padding individual).  The
 * consecutive within-group pairs (css.c:627-642) are summed in track order; the
 * between-group sum over G is sum_{x in G} R_x - 2 sum_{x<y in G} S_xy with the members
 * ascending, visited in 8x8 blocks, so it is a function of the SET G alone: every
 * permutation that keeps the groups' sets gets the observed value bit for bit. */
template <int MP, bool UNROLL, class TRK, class MEMB, class SXY>
__device__ __forceinline__ double score_exact(TRK track, MEMB member, SXY sxy, const double *R, int a, int b,
                                              double inva, double invb) {
  constexpr int NB = (PermShape<MP>::HALF + 7) / 8;
  const int m = a + b;
  double wa = 0.0, wb = 0.0;
  uint32_t prev = track(0);
#pragma unroll 4
  for (int k = 1; k < m; ++k) {
    const uint32_t cur = track(k);
    const double e = sxy(min(prev, cur), max(prev, cur));
    if (k < a) wa += e;
    if (k > a) wb += e;
    prev = cur;
  }
  double sr = 0.0, q0 = 0.0, q1 = 0.0, q2 = 0.0, q3 = 0.0;
  if constexpr (UNROLL) {
    /* the observed score (once per window, S from the triangle): many loads in flight */
#pragma unroll 1
    for (int K = 0; K < NB; ++K) {
      uint32_t xk[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        xk[u] = member(8 * K + u);
        sr += R[xk[u]];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
#pragma unroll
        for (int v = u + 1; v < 8; ++v) {
          const double e = sxy(xk[u], xk[v]);
          if ((u + v) & 1)
            q0 += e;
          else
            q1 += e;
        }
        asm volatile("" ::: "memory");
      }
#pragma unroll 1
      for (int L = K + 1; L < NB; ++L) {
        uint32_t xl[8];
#pragma unroll
        for (int v = 0; v < 8; ++v) xl[v] = member(8 * L + v);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
          for (int v = 0; v < 8; ++v) {
            const double e = sxy(xk[u], xl[v]);
            if (v & 1)
              q3 += e;
            else
              q2 += e;
          }
          asm volatile("" ::: "memory");
        }
      }
    }
  } else {
    /* rolled (the rare ambiguous lanes, S from the coordinates); the additions reach
     * each accumulator in the same order */
#pragma unroll 1
    for (int K = 0; K < NB; ++K) {
#pragma unroll 1
      for (int u = 0; u < 8; ++u) sr += R[member(8 * K + u)];
#pragma unroll 1
      for (int u = 0; u < 8; ++u) {
        const uint32_t xu = member(8 * K + u);
#pragma unroll 1
        for (int v = u + 1; v < 8; ++v) {
          const double e = sxy(xu, member(8 * K + v));
          if ((u + v) & 1)
            q0 += e;
          else
            q1 += e;
        }
      }
#pragma unroll 1
      for (int L = K + 1; L < NB; ++L)
#pragma unroll 1
        for (int u = 0; u < 8; ++u) {
          const uint32_t xu = member(8 * K + u);
#pragma unroll 1
          for (int v = 0; v < 8; ++v) {
            const double e = sxy(xu, member(8 * L + v));
            if (v & 1)
              q3 += e;
            else
              q2 += e;
          }
        }
    }
  }
  const double bet = sr - 2.0 * ((q0 + q1) + (q2 + q3));
  return bet / (double)(a * b) - (double)(a + b) * (wa * inva + wb * invb);
}

/* The same score from the FP32 copy of S, with a bound on its distance to the FP64
 * value score_exact returns: est, err with |score_exact - est| <= err.  Every S
 * entry is >= 0, so a sum of n FP32-rounded terms is within (n + 2) 2^-24 of its
 * computed value (representation + recursive summation), plus 2^-125 per term for
 * flushed subnormals; the FP64 sums and the final arithmetic of both versions add
 * < 1e-11 of the magnitudes involved.  Reads the track from column `col` (byte k
 * at col[k*PERM_ROW]) and writes G's members ascending to `mcol` (the track stays intact
 * for score_exact).  sr, the row-sum term, is summed exactly as score_exact sums it. */
template <int MP>
__device__ __forceinline__ void score_f32(const float *S32, const double *R, const uint8_t *col, const uint8_t *fmap,
                                          bool mapped, uint8_t *mcol, int a, int b, double inva, double invb,
                                          double &est, double &err) {
  constexpr int NB = (PermShape<MP>::HALF + 7) / 8;
  const int m = a + b;
  const int g = a <= b ? a : b, off = a <= b ? 0 : a;
  const char *Sb = reinterpret_cast<const char *>(S32);
  auto s_at = [&](uint32_t off4) { return *reinterpret_cast<const float *>(Sb + off4); };
  /* consecutive pairs inside each group, and G as a bit set */
  float wa = 0.f, wb = 0.f;
  uint64_t lo = 0, hi = 0;
  auto add_member = [&](uint32_t x) {
    lo |= x < 64 ? 1ull << (x & 63u) : 0ull;
    if constexpr (MP > 64) hi |= x >= 64 ? 1ull << (x & 63u) : 0ull;
  };
  /* track entry k: the column byte, through the wave's map when its compositions started
   * from the identity (`mapped` is wave-uniform) */
  auto track = [&](int k) -> uint32_t {
    const uint32_t c = col[k * PERM_ROW];
    return mapped ? (uint32_t)fmap[c] : c;
  };
  /* split at the group boundary (G is group A iff ga, wave-uniform): no per-entry selects */
  const bool ga = off == 0;
  uint32_t prev = track(0), tprev = tri4(prev);
  auto pair_next = [&](uint32_t cur, uint32_t tcur) {
    const float e = s_at(prev > cur ? tprev + (cur << 2) : tcur + (prev << 2));
    prev = cur;
    tprev = tcur;
    return e;
  };
  if (ga && g > 0) add_member(prev);
#pragma unroll 4
  for (int k = 1; k < a; ++k) {
    const uint32_t cur = track(k);
    wa += pair_next(cur, tri4(cur));
    if (ga) add_member(cur);
  }
  if (a > 0 && a < m) { /* the pair across the boundary counts for neither group */
    prev = track(a);
    tprev = tri4(prev);
    if (!ga) add_member(prev);
  }
#pragma unroll 4
  for (int k = a + 1; k < m; ++k) {
    const uint32_t cur = track(k);
    wb += pair_next(cur, tri4(cur));
    if (!ga) add_member(cur);
  }
  /* the members, ascending: the set bits of lo, then those of hi (per-lane trip counts;
   * one find-first-set per member instead of both words' in every step) */
  int k = 0;
  while (lo != 0) {
    mcol[k * 64] = (uint8_t)__builtin_ctzll(lo);
    lo &= lo - 1;
    ++k;
  }
  if constexpr (MP > 64) {
    if constexpr (MP - 64 <= 32) {
      uint32_t h = (uint32_t)hi;
      while (h != 0) {
        mcol[k * 64] = (uint8_t)(64u + (uint32_t)__builtin_ctz(h));
        h &= h - 1;
        ++k;
      }
    } else {
      while (hi != 0) {
        mcol[k * 64] = (uint8_t)(64u + (uint32_t)__builtin_ctzll(hi));
        hi &= hi - 1;
        ++k;
      }
    }
  }
  auto member = [&](int k) -> uint32_t { return k < g ? (uint32_t)mcol[k * 64] : (uint32_t)MP; };
  /* gathers in pairs, summed with packed FP32 adds (v_pk_add_f32) */
  typedef float f2 __attribute__((ext_vector_type(2)));
  double sr = 0.0;
  f2 qa = {0.f, 0.f}, qb = {0.f, 0.f};
#pragma unroll 1
  for (int K = 0; K < NB; ++K) {
    uint32_t xk4[8], tk[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t x = member(8 * K + u);
      sr += R[x];
      xk4[u] = x << 2;
      tk[u] = tri4(x);
    }
#pragma unroll
    for (int u = 0; u < 7; ++u) {
#pragma unroll
      for (int v = u + 1; v < 8; v += 2) {
        f2 e;
        e.x = s_at(tk[v] + xk4[u]); /* x_u < x_v */
        e.y = v + 1 < 8 ? s_at(tk[v + 1] + xk4[u]) : 0.f;
        qa += e;
      }
      if (u & 1) asm volatile("" ::: "memory"); /* a bounded number of gathers in flight */
    }
#pragma unroll 1
    for (int L = K + 1; L < NB; ++L) {
      uint32_t tl[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) tl[v] = tri4(member(8 * L + v));
#pragma unroll
      for (int u = 0; u < 8; ++u) {
#pragma unroll
        for (int v = 0; v < 8; v += 2) {
          f2 e;
          e.x = s_at(tl[v] + xk4[u]); /* every member of block K < every member of block L */
          e.y = s_at(tl[v + 1] + xk4[u]);
          qb += e;
        }
        if (u & 1) asm volatile("" ::: "memory");
      }
    }
  }
  const double q = (double)((qa.x + qa.y) + (qb.x + qb.y)), dwa = (double)wa, dwb = (double)wb;
  const double ab = (double)(a * b), apb = (double)(a + b);
  est = (sr - 2.0 * q) / ab - apb * (dwa * inva + dwb * invb);
  constexpr double U = 0x1p-24 * 1.001, SUB = 0x1p-125;
  const double nq = (double)(g * (g - 1) / 2 + 4);
  const double eq = nq * (U * q + SUB), ewa = (a + 2) * (U * dwa + SUB), ewb = (b + 2) * (U * dwb + SUB);
  const double mag = (fabs(sr) + 2.0 * q) / ab + apb * (dwa * inva + dwb * invb);
  err = 2.0 * eq / ab + apb * (ewa * inva + ewb * invb) + 1e-11 * mag;
}

typedef _Float16 pm_f16x8 __attribute__((ext_vector_type(8)));
typedef float pm_f32x16 __attribute__((ext_vector_type(16)));

/* The score of every lane's track on the matrix cores (the between-group sum of
 * css.c:608-647 as a bilinear form).  With x_p the indicator of group A under
 * permutation p, bet_p = sum_{i in A, j in B} S_ij = x_p^T S (1 - x_p): one wave forms
 * Y = S (1 - X) for its 64 permutations (X: individuals x permutations, 0/1, exact in
 * fp16) as v_mfma_f32_32x32x16_f16 products with S scaled by a power of two sc (its
 * largest entry to [2^14, 2^15)) and rounded to fp16, then bet_p = sum_i X_ip Y_ip from
 * the accumulator tiles (lane l holds column l & 31, rows (reg & 3) + 8 (reg >> 2) +
 * 4 (l >> 5) of each 32 x 32 tile).  The consecutive within-group pairs (Q8) are gathered
 * from the same matrix.  Error bound, u = 2^-24: an entry is within 2^-10 of its scaled
 * value plus 2^-14 absolute (entries below fp16's smallest normal 2^-14 are stored as 0,
 * so the bound holds whether or not the matrix cores keep fp16 denormals; a float
 * rounding first); the products with
 * 0/1 are exact; each Y entry takes <= 16 KT fp32 roundings and each dot <= 32 MT + 1
 * more, so |bet - est| <= (2^-10 + u (16 KT + 32 MT + 4)) bet + a b 2^-14 / sc; the pair
 * sums likewise with their term counts.  est and err as score_f32: |score_exact - est|
 * <= err, and the few lanes inside the bound recompute in FP64. */
template <int MP>
__device__ __forceinline__ void score_mfma(const char *s16, const uint2 *lut, const uint8_t *col, const uint8_t *fmap,
                                           bool mapped, int a, int b, double inva, double invb, double inv_sc,
                                           int lane, double &est, double &err) {
  using SH = PermShape<MP>;
  constexpr int MT = SH::MT, KT = SH::KT, RS = SH::RS;
  static_assert(MP <= 96, "score_mfma keeps members 64.. in one 32-bit word");
  static_assert(SH::MT <= 3, "score_mfma's row tiles take their mask words from (lo, hi)");
  const int m = a + b;
  uint64_t lo = 0, hi = 0;
  auto s_at = [&](uint32_t x, uint32_t y) -> float {
    return (float)*reinterpret_cast<const _Float16 *>(s16 + __umul24(x, (uint32_t)RS) + 2 * y);
  };
  uint32_t hi32 = 0; /* members 64 .. MP - 1 (MP <= 96) */
  auto add = [&](uint32_t x) {
    const uint64_t t = 1ull << (x & 63u);
    if constexpr (MP > 64) {
      const bool h = x >= 64u;
      lo |= h ? 0ull : t;
      hi32 |= h ? (uint32_t)t : 0u;
    } else {
      lo |= t;
    }
  };
  /* group A's members and the consecutive pairs, 16 track entries at a time: the
   * entries' loads, their map lookups and the pair gathers each go out as one batch
   * (one wait per batch instead of a round trip per entry) */
  float wa = 0.f, wb = 0.f;
  uint32_t prev = 0;
  constexpr int CK = 16; /* rows m .. MP - 1 of the byte matrix hold 0 (sig_identity) */
  auto batch = [&](int k0) {
    if (k0 < m) {
      uint32_t c[CK];
#pragma unroll
      for (int i = 0; i < CK; ++i) c[i] = k0 + i < MP ? (uint32_t)col[(k0 + i) * PERM_ROW] : 0u;
      if (mapped) {
#pragma unroll
        for (int i = 0; i < CK; ++i) c[i] = fmap[c[i]];
      }
      float e[CK];
#pragma unroll
      for (int i = 0; i < CK; ++i) e[i] = s_at(i == 0 ? prev : c[i - 1], c[i]);
#pragma unroll
      for (int i = 0; i < CK; ++i) {
        const int k = k0 + i;
        if (k >= 1 && k < a) wa += e[i];
        if (k > a && k < m) wb += e[i];
        if (k < a) add(c[i]);
      }
      prev = c[CK - 1];
    }
  };
  /* Above 64 individuals the batches run as a loop: unrolled, the compiler hoisted every
   * (k < a), (k > a), (k < m) test of the MP entries out of the permutation loop as SGPR
   * masks and spilled them to VGPR lanes (467 SGPR spills at 80, a v_readlane per use);
   * rolled, the tests are scalar compares in the loop (C5 shape 8.40-8.43 -> 8.07-8.16 ms per
   * 50k windows).  At 40 the unrolled form stays ahead (20+20 with mcR 1000: 15.86 against
   * 16.06 ms per 200k windows). */
  if constexpr (MP > 64) {
#pragma unroll 1
    for (int k0 = 0; k0 < MP; k0 += CK) batch(k0);
  } else {
#pragma unroll
    for (int k0 = 0; k0 < MP; k0 += CK) batch(k0);
  }
  hi = hi32;
  const uint64_t vlo = m >= 64 ? ~0ull : ((1ull << m) - 1), vhi = m > 64 ? ((1ull << (m - 64)) - 1) : 0ull;
  const uint64_t clo = ~lo & vlo, chi = ~hi & vhi; /* group B = the complement within m */
  /* the masks of the two permutations whose columns this lane's fragments carry */
  const int r = lane & 31, h = lane >> 5;
  auto pull = [](uint64_t v, int src) -> uint64_t {
    const uint32_t l = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)v);
    const uint32_t u = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)(v >> 32));
    return ((uint64_t)u << 32) | l;
  };
  uint64_t cm[2][2], am[2][2];
  cm[0][0] = pull(clo, r);
  cm[1][0] = pull(clo, 32 + r);
  am[0][0] = pull(lo, r);
  am[1][0] = pull(lo, 32 + r);
  if constexpr (MP > 64) {
    cm[0][1] = pull(chi, r);
    cm[1][1] = pull(chi, 32 + r);
    am[0][1] = pull(hi, r);
    am[1][1] = pull(hi, 32 + r);
  } else {
    cm[0][1] = cm[1][1] = am[0][1] = am[1][1] = 0;
  }
  /* one 32 x 32 output tile at a time (16 accumulators live): for each column tile n and
   * row tile t, the k steps accumulate, then the tile's rows of this lane's column enter
   * the dot with X */
  float own = 0.f, send = 0.f;
#pragma unroll 1
  for (int n = 0; n < 2; ++n) {
    const uint64_t c0 = n ? cm[1][0] : cm[0][0], c1 = n ? cm[1][1] : cm[0][1];
    const uint64_t a0 = n ? am[1][0] : am[0][0], a1 = n ? am[1][1] : am[0][1];
    float part = 0.f;
#pragma unroll 1
    for (int t = 0; t < MT; ++t) {
      pm_f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int k0 = kt * 16 + 8 * h; /* this lane's 8 k of the step */
        const uint64_t c = k0 < 64 ? c0 >> k0 : c1 >> (k0 - 64);
        const uint2 l4 = lut[c & 15u], h4 = lut[(c >> 4) & 15u];
        uint4 v;
        v.x = l4.x;
        v.y = l4.y;
        v.z = h4.x;
        v.w = h4.y;
        const pm_f16x8 bf = __builtin_bit_cast(pm_f16x8, v);
        const int arow = SH::S16ROWS < MT * 32 ? min(t * 32 + r, MP) : t * 32 + r; /* row MP is zero */
        const pm_f16x8 ah =
            __builtin_bit_cast(pm_f16x8, *reinterpret_cast<const uint4 *>(s16 + arow * RS + 2 * k0));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bf, acc, 0, 0, 0);
        if (kt & 1) asm volatile("" ::: "memory"); /* two k steps of fragment loads in flight */
      }
      /* accumulator e holds row t * 32 + 4 h + (e & 3) + 8 (e >> 2) of this lane's column:
       * its membership bit from the tile's 32-bit word of the A-mask, as an all-ones /
       * zero mask (one sign-extending bit-field extract) ANDed into the float */
      const uint32_t W = t == 0 ? (uint32_t)a0 : (t == 1 ? (uint32_t)(a0 >> 32) : (uint32_t)a1);
      const uint32_t Wh = W >> (4 * h);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const uint32_t msk = (uint32_t)__builtin_amdgcn_sbfe((int)Wh, (e & 3) + 8 * (e >> 2), 1);
        part += __uint_as_float(__float_as_uint(acc[e]) & msk);
      }
    }
    if (n == h)
      own = part;
    else
      send = part;
  }
  /* the other row half of this lane's column comes from lane ^ 32 */
  const float q = own + __shfl_xor(send, 32);
  const double ab = (double)(a * b), apb = (double)(a + b);
  const double dq = (double)q * inv_sc, dwa = (double)wa * inv_sc, dwb = (double)wb * inv_sc;
  est = dq / ab - apb * (dwa * inva + dwb * invb);
  constexpr double U = 0x1p-24, REP = 0x1p-10, SUB = 0x1p-14;
  const double ebet = (REP + U * (16 * KT + 32 * MT + 4)) * dq * 1.001 + SUB * ab * inv_sc;
  const double ewa = (REP + U * (a + 4)) * dwa * 1.001 + SUB * a * inv_sc;
  const double ewb = (REP + U * (b + 4)) * dwb * 1.001 + SUB * b * inv_sc;
  const double mag = dq / ab + apb * (dwa * inva + dwb * invb);
  err = ebet / ab + apb * (ewa * inva + ewb * invb) + 1e-11 * mag;
}

/* every lane's column of one wave's byte matrix := identity (rows k < m; row k is
 * 64 bytes of k), rows m .. MP - 1 := 0 (score_mfma reads whole 16-row batches) */
template <int MP>
__device__ __forceinline__ void sig_identity(uint8_t *sig, int m, int lane) {
  PERM_OPAQUE(lane);
  for (int q = lane; q < MP * 16; q += 64) {
    const uint32_t k = (uint32_t)(q >> 4);
    *reinterpret_cast<uint32_t *>(sig + (q >> 4) * PERM_ROW + (q & 15) * 4) = k < (uint32_t)m ? k * 0x01010101u : 0u;
  }
}

/* random_int_nrand48(n) constants for 2 <= n <= 128 from the magic number alone
 * (gd_randint_make): shift = ceil(log2 n) - 1, and the rejection limit
 * RAND_MAX - 2^31 mod n from (2^31 - 1) mod n.  n is wave-uniform, so this is
 * scalar work; the magic comes from a 4-byte-per-n LDS table. */
__device__ __forceinline__ gd_randint perm_rd(uint32_t n, uint32_t magic) {
  gd_randint d;
  d.n = n;
  d.magic = magic;
  d.shift = 31u - (uint32_t)__clz((int)(n - 1u)); /* ceil(log2 n) - 1 */
  const uint32_t q = (uint32_t)(((uint64_t)0x7FFFFFFFu * magic) >> 32) >> d.shift;
  const uint32_t t = 0x7FFFFFFFu - q * n + 1u; /* (2^31 - 1) mod n + 1 */
  d.limit = GD_RAND_MAX - (t == n ? 0u : t);
  return d;
}

#ifndef PERM_FY_UNROLL
#define PERM_FY_UNROLL 1 /* Fisher-Yates steps unrolled with literal constants (fy_fast_unrolled) */
#endif
#ifndef PERM_FY_PIPE
#define PERM_FY_PIPE 0 /* software-pipelined Fisher-Yates (reads one step ahead, forwarded): measured
                        * slower (the draw phase is issue-bound; forwarding adds 4 VALU per step) */
#endif

/* the magic number of n from VGPR lanes (lane l holds mag[l] in vm0, mag[64 + l] in vm1;
 * n wave-uniform): no LDS round trip in the draw chain */
__device__ __forceinline__ uint32_t perm_mag(uint32_t vm0, uint32_t vm1, int n) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)vm0, n & 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)vm1, n & 63);
  return n < 64 ? lo : hi;
}

/* One nrand48 step on y = x << 16 (mod 2^64), as the FET draw loop takes it (gd_fet_fast.hip
 * FW_STEP): ylo's low 16 bits are 0, so the high word a_lo yhi + 5 ylo + hi(a_lo ylo + c16)
 * is one v_mad_u64_u32 whose addend 5 ylo + hi(...) is a v_mad_u32_u24 of ylo >> 16
 * (14 issue cycles against 16 for the compiler's mul_lo / lshl_add / add3 form) */
#ifndef PERM_LCG_MAD
#define PERM_LCG_MAD 0 /* measured neutral to slower here (C5 shape) */
#endif
__device__ __forceinline__ void perm_lcg_step(uint64_t &y) {
#if PERM_LCG_MAD
  const uint32_t ylo = (uint32_t)y, yhi = (uint32_t)(y >> 32);
  const uint64_t t = (uint64_t)ylo * 0xDEECE66Du + (GD_LCG_C << 16);
  const uint32_t s = __umul24(ylo >> 16, 5u << 16) + (uint32_t)(t >> 32);
  uint64_t acc;
  asm volatile("" : "=v"(acc)); /* a fresh pair: its high word is don't-care */
  acc = (acc & 0xFFFFFFFF00000000ull) | s;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(yhi), "s"(0xDEECE66Du) : "vcc");
  y = ((uint64_t)(uint32_t)acc << 32) | (uint32_t)t;
#else
  y = y * GD_LCG_A + (GD_LCG_C << 16);
#endif
}

/* the draw of a straight-line step as an opaque 32-bit value (PERM_R_FENCE): otherwise the
 * compiler folds (y >> 33) > limit into a 64-bit compare of y against a per-step 64-bit
 * constant, hoists the 2 (MP - 1) constant words out of the permutation loop and spills them
 * (80: 187 -> 71 SGPR spills) */
#ifndef PERM_R_FENCE
#define PERM_R_FENCE 1
#endif
/* Fisher-Yates swaps of random_shuffle (css.c:700-706) on the lane's column, draws
 * from state x (no rejection: the caller checks); returns true if a draw would have
 * been rejected.
 *
 * Software-pipelined: step n swaps positions n - 1 and j_n.  The two reads of step
 * n - 1 are issued before the two writes of step n (LDS is in order per wave, so they
 * see every write up to step n + 1), and step n's writes are forwarded in registers:
 * position n - 2 or j_{n-1} holds u_n iff it equals j_n (position n - 1, written with
 * v_n, is never read again).  Each step then waits for reads issued one step earlier
 * instead of a full read -> write round trip.  The loop body is two steps with their
 * own registers (A, B), so no loaded value is copied across the back edge (a copy
 * would wait for the load). */
__device__ __forceinline__ bool fy_fast(uint8_t *col, uint64_t x, int m, uint32_t vm0, uint32_t vm1) {
  bool rej = false;
  /* the LCG on y = x << 16 (mod 2^64): no 48-bit mask, the draw is y >> 33 */
  uint64_t y = x << 16;
  auto draw = [&](int n) -> uint32_t { /* j_n = r mod n (n >= 2, wave-uniform) */
    const gd_randint rd = perm_rd((uint32_t)n, perm_mag(vm0, vm1, n));
    y = y * GD_LCG_A + (GD_LCG_C << 16);
    const uint32_t r = (uint32_t)(y >> 33);
    rej |= r > rd.limit;
    return r - (__umulhi(r, rd.magic) >> rd.shift) * (uint32_t)n;
  };
  auto at = [&](uint32_t k) -> uint8_t * { return col + __umul24(k, (uint32_t)PERM_ROW); };
#if PERM_FY_PIPE
  if (m < 2) return false;
  int n = __builtin_amdgcn_readfirstlane(m);
  /* at the top of step n: jA = j_n with its reads (urA, vrA) in flight, jN = j_{n-1}
   * drawn; step n issues the reads of step n - 1, draws j_{n-2}, then (the reads of
   * step n now two draws old) forwards and writes.  sched_barrier keeps the compiler
   * from hoisting the forwarding (and its wait) above the next reads and draw. */
  uint32_t jA = draw(n);
  uint8_t urA = *at((uint32_t)(n - 1)), vrA = *at(jA);
  uint32_t jN = n > 2 ? draw(n - 1) : 0u;
  uint32_t jp = 0xFFFFFFFFu; /* the previous step's j and u (none yet) */
  uint8_t up = 0;
#define FY_STEP(J, UR, V, URN, VRN, N)                                       \
  do {                                                                      \
    const uint32_t jn_ = jN;                                                \
    URN = *at((uint32_t)((N) - 2));                                         \
    VRN = *at(jn_);                                                         \
    jN = draw((N) - 2);                                                     \
    __builtin_amdgcn_sched_barrier(0);                                      \
    const uint8_t u_ = jp == (uint32_t)((N) - 1) ? up : UR;                 \
    const uint8_t v_ = jp == J ? up : V;                                    \
    *at((uint32_t)((N) - 1)) = v_;                                          \
    *at(J) = u_;                                                            \
    jp = J;                                                                 \
    up = u_;                                                                \
    J = jn_;                                                                \
  } while (0)
  uint8_t urB, vrB;
  for (; n > 4; n -= 2) { /* draws j_{n-2}, j_{n-3} >= 2 */
    FY_STEP(jA, urA, vrA, urB, vrB, n);
    FY_STEP(jA, urB, vrB, urA, vrA, n - 1);
  }
#undef FY_STEP
  { /* finish step n (2 <= n <= 4), then the last steps unpipelined */
    const uint8_t u = jp == (uint32_t)(n - 1) ? up : urA, v = jp == jA ? up : vrA;
    *at((uint32_t)(n - 1)) = v;
    *at(jA) = u;
  }
  for (int k = n - 1; k >= 2; --k) {
    const uint32_t j = k == n - 1 ? jN : draw(k);
    const uint8_t u = *at((uint32_t)(k - 1)), v = *at(j);
    *at((uint32_t)(k - 1)) = v;
    *at(j) = u;
  }
#else
  /* steps n >= 64 read their magic from vm1, the rest from vm0: one readlane per step */
  auto step = [&](int n, uint32_t mg) {
    const gd_randint rd = perm_rd((uint32_t)n, mg);
    perm_lcg_step(y);
    const uint32_t r = (uint32_t)(y >> 33);
    rej |= r > rd.limit;
    const uint32_t j = r - (__umulhi(r, rd.magic) >> rd.shift) * (uint32_t)n;
    const uint8_t u = *at((uint32_t)(n - 1)), v = *at(j);
    *at((uint32_t)(n - 1)) = v;
    *at(j) = u;
  };
  int n = __builtin_amdgcn_readfirstlane(m);
  for (; n >= 64; --n) step(n, (uint32_t)__builtin_amdgcn_readlane((int)vm1, n - 64));
  for (; n >= 2; --n) step(n, (uint32_t)__builtin_amdgcn_readlane((int)vm0, n));
#endif
  return rej;
}

/* random_int_nrand48 constants of a compile-time n (gd_randint_make's formulas) */
struct PmRd {
  uint32_t magic, shift, limit;
};
constexpr PmRd pm_rd_const(uint32_t n) {
  uint32_t l = 0;
  while ((1ull << l) < n) ++l;
  PmRd d{0u, 0u, 0x7FFFFFFFu - (uint32_t)(0x80000000ull % n)};
  if (l) {
    d.magic = (uint32_t)(((1ull << (31 + l)) + n - 1) / n);
    d.shift = l - 1;
  }
  return d;
}

/* fy_fast with every step unrolled (PERM_FY_UNROLL): step n's magic number, shift and
 * rejection limit are literals and its row n - 1 an immediate LDS offset, so a step is
 * the LCG, the remainder, one address and the swap -- no readlane, no scalar
 * arithmetic.  Taken when the window fills its tier (m == MP, e.g. 40 + 40); other
 * cohorts run the loop (fy_fast). */
template <int N, bool FENCE>
__device__ __forceinline__ void fy_step(uint8_t *col, uint64_t &y, bool &rej) {
  constexpr PmRd rd = pm_rd_const((uint32_t)N);
  perm_lcg_step(y);
  uint32_t r = (uint32_t)(y >> 33);
  if constexpr (FENCE) asm("" : "+v"(r));
  rej |= r > rd.limit;
  const uint32_t j = r - (__umulhi(r, rd.magic) >> rd.shift) * (uint32_t)N;
  uint8_t *pn = col + (N - 1) * PERM_ROW;
  uint8_t *pj = col + __umul24(j, (uint32_t)PERM_ROW);
  const uint8_t u = *pn, v = *pj;
  *pn = v;
  *pj = u;
}
template <int N, bool FENCE>
__device__ __forceinline__ void fy_steps(uint8_t *col, uint64_t &y, bool &rej) {
  if constexpr (N >= 2) {
    fy_step<N, FENCE>(col, y, rej);
    fy_steps<N - 1, FENCE>(col, y, rej);
  }
}
/* a full tier (m == MP): the steps n = MP .. 2 as one straight line */
template <int MP>
__device__ __forceinline__ bool fy_fast_unrolled(uint8_t *col, uint64_t x) {
  bool rej = false;
  uint64_t y = x << 16;
  fy_steps<MP, (PERM_R_FENCE != 0) && MP <= 80>(col, y, rej); /* at 96 the fence cost registers: 2 -> 1 wave */
  return rej;
}

/* the same with random_int_nrand48's redraw loop (css.c:675-690) */
__device__ __forceinline__ void fy_exact(uint8_t *col, uint64_t x, int m) {
  for (int s = 0; s < m - 1; ++s) {
    const int n = __builtin_amdgcn_readfirstlane(m - s);
    const gd_randint rd = gd_randint_make((uint32_t)n);
    uint32_t r;
    do {
      x = gd_lcg_next(x);
      r = gd_lcg_value(x);
    } while (r > rd.limit);
    const int j = (int)gd_randint_mod(&rd, r);
    const uint8_t u = col[(n - 1) * PERM_ROW], v = col[j * PERM_ROW];
    col[(n - 1) * PERM_ROW] = v;
    col[j * PERM_ROW] = u;
  }
}


/* the exact serial stream (random_int_nrand48's redraws, css.c:675-690) advanced over q whole
 * permutations of m - 1 draws each: a permutation's start state, derived by its own lane (the
 * rare rejection path) */
__device__ __forceinline__ uint64_t serial_advance(uint64_t y, int q, int m, uint32_t vm0, uint32_t vm1) {
  for (int p = 0; p < q; ++p)
    for (int s = 0; s < m - 1; ++s) {
      const int n = __builtin_amdgcn_readfirstlane(m - s);
      const gd_randint rd = perm_rd((uint32_t)n, perm_mag(vm0, vm1, n));
      do y = gd_lcg_next(y);
      while (gd_lcg_value(y) > rd.limit);
    }
  return y;
}

/* sum over the wave, the same value in every lane (an xor butterfly: both lanes of a
 * pair add the same two operands) */
__device__ __forceinline__ double pw_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

/* The exact FP64 css() (css.c:608-647) of one track array, computed by the whole wave
 * (matrix-core tiers, <= 80 individuals): the observed score (identity tracks) and the
 * rare permutations whose matrix-core estimate lies within its error bound of it.
 *   consecutive within-group pairs (Q8): entry k = lane (and lane + 64) with entry k - 1;
 *   between-group sum over the pairs (A_i, B_j) of the groups' members in ascending
 *   order, pair p = i b + j dealt to lane p mod 64 and summed in p order per lane;
 *   both reduced by the butterfly.
 * A function of the order within each group and of the groups' SETS only, so every
 * permutation that keeps them gets the observed value bit for bit (ties are decided
 * identically for observed and permuted scores).  Distances from the coordinates
 * (calc_dist, css.c:573-587; symmetric bit for bit).  ent(k): track entry k < m;
 * lst: 256 bytes of the wave's LDS scratch; rb: random_int constants of n = b. */
template <int MP, class ENT>
__device__ double score_exact_wave(ENT ent, const double *X, int a, int b, double inva, double invb, int lane,
                                   uint8_t *lst, const gd_randint &rb) {
  static_assert(MP <= 80, "score_exact_wave's scratch holds 80 individuals per list");
  const int m = a + b;
  const uint32_t t0 = lane < m ? ent(lane) : 0u;
  const uint32_t t1 = (MP > 64 && lane + 64 < m) ? ent(lane + 64) : 0u;
  double wa = 0.0, wb = 0.0;
  {
    const uint32_t p0 = (uint32_t)__shfl_up((int)t0, 1);
    const int k = lane;
    if (k >= 1 && k < m && k != a) {
      const double e = perm_xdist(X, (int)p0, (int)t0);
      if (k < a)
        wa = e;
      else
        wb = e;
    }
  }
  if constexpr (MP > 64) {
    const uint32_t s63 = (uint32_t)__shfl((int)t0, 63), su = (uint32_t)__shfl_up((int)t1, 1);
    const uint32_t p1 = lane == 0 ? s63 : su;
    const int k = lane + 64;
    if (k < m && k != a) {
      const double e = perm_xdist(X, (int)p1, (int)t1);
      if (k < a)
        wa += e;
      else
        wb += e;
    }
  }
  wa = pw_sum(wa);
  wb = pw_sum(wb);
  /* membership flags (LDS in issue order within the wave), then the members ascending:
   * rank = set lanes below in the ballot */
  uint8_t *fl = lst, *la = lst + 96, *lb = lst + 176;
  if (lane < m) fl[t0] = (uint8_t)(lane < a);
  if (MP > 64 && lane + 64 < m) fl[t1] = (uint8_t)(lane + 64 < a);
  __builtin_amdgcn_wave_barrier();
  const bool v0 = lane < m, v1 = MP > 64 && lane + 64 < m;
  const bool in0 = v0 && fl[lane] != 0, in1 = v1 && fl[(MP > 64 ? lane + 64 : lane)] != 0;
  const uint64_t A0 = __ballot(in0), A1 = __ballot(in1), B0 = __ballot(v0 && !in0), B1 = __ballot(v1 && !in1);
  const uint64_t below = (1ull << lane) - 1ull;
  if (in0) la[__popcll(A0 & below)] = (uint8_t)lane;
  if (v0 && !in0) lb[__popcll(B0 & below)] = (uint8_t)lane;
  if (in1) la[__popcll(A0) + __popcll(A1 & below)] = (uint8_t)(lane + 64);
  if (v1 && !in1) lb[__popcll(B0) + __popcll(B1 & below)] = (uint8_t)(lane + 64);
  __builtin_amdgcn_wave_barrier();
  double bet = 0.0;
  const int nab = a * b;
  for (int p = lane; p < nab; p += 64) {
    const uint32_t i = b == 1 ? (uint32_t)p : (__umulhi((uint32_t)p, rb.magic) >> rb.shift);
    const uint32_t j = (uint32_t)p - i * (uint32_t)b;
    bet += perm_xdist(X, la[i], lb[j]);
  }
  bet = pw_sum(bet);
  return bet / (double)(a * b) - (double)(a + b) * (wa * inva + wb * invb);
}

}  // namespace

#ifdef PERM_COUNT_AMBIGUOUS
__device__ unsigned long long g_perm_amb[2];
#endif
#ifdef PERM_WAVES_PER_SIMD /* diagnostic: register-allocation target */
#define PERM_WPE __attribute__((amdgpu_waves_per_eu(PERM_WAVES_PER_SIMD, PERM_WAVES_PER_SIMD)))
#else
#define PERM_WPE
#endif
template <int MP>
__global__ void __launch_bounds__(PermShape<MP>::NT) PERM_WPE
    k_css_perm(const gd_chrom_dev *ch, int nchrom, const double *xbuf, const uint8_t *status, int64_t wtotal,
               int treshold, int runs, double *pvals, unsigned *wq, int force_exact) {
  using SH = PermShape<MP>;
  constexpr int TRI = SH::TRI, NWV = SH::NWV, NT = SH::NT, P = 64 * NWV, SIG = SH::SIG;
  __shared__ __attribute__((aligned(16))) char s_U[SH::UBYTES];
  /* the window's MDS coordinates (FP64 distances on demand): the FP32 tiers stage them in
   * LDS; the matrix-core tiers read them in place (xbuf; the window setup and the rare
   * near-tie recomputes only), which keeps their workgroup at 6 per CU */
  __shared__ double s_Xl[SH::MF ? 1 : 2 * MP];
  __shared__ double s_R[SH::MF ? 1 : MP + 1]; /* row sums: the FP32 score's tiers only */
  __shared__ uint64_t s_hit[NWV];
  __shared__ uint8_t s_car[MP > 64 ? 128 : 64];
  __shared__ uint8_t s_gend[NWV * PERM_CHAINS * MP]; /* each chain's last composition */
  __shared__ uint8_t s_fs[NWV * PERM_CHAINS * MP];   /* each chain's map: the tracks before its first permutation */
  __shared__ int64_t s_w;
  double *s_S = reinterpret_cast<double *>(s_U); /* FP64 triangle: window setup only */
  float *s_S32 = reinterpret_cast<float *>(s_U);  /* FP32 triangle: the permutation passes */
  uint64_t *s_st = reinterpret_cast<uint64_t *>(s_U + SH::OFF_MEM); /* serial start states (FP32 tiers, draw phase only) */
  __shared__ uint64_t s_next; /* the serial stream after a pass (matrix-core tiers' rejection path) */
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ uint2 s_lut[16]; /* 4 indicator bits -> 4 bf16 (0 or 1.0): score_mfma's B fragments */
  if (tid < 16) /* fp16 1.0 = 0x3C00 */
    s_lut[tid] = make_uint2((tid & 1 ? 0x3C00u : 0u) | (tid & 2 ? 0x3C000000u : 0u),
                            (tid & 4 ? 0x3C00u : 0u) | (tid & 8 ? 0x3C000000u : 0u));
  __syncthreads();
  /* the magic numbers in VGPR lanes for fy_fast (kept for the kernel's life; the opaque
   * use completes the loads here, so the draw loop carries no LDS wait for them) */
  uint32_t vm0 = lane <= MP ? gd_randint_make(lane < 1 ? 1u : (uint32_t)lane).magic : 0u;
  uint32_t vm1 = lane + 64 <= MP ? gd_randint_make((uint32_t)(lane + 64)).magic : 0u;
  PERM_OPAQUE(vm0);
  PERM_OPAQUE(vm1);
  const char *s16 = s_U; /* score_mfma: the scaled fp16 matrix */
  uint8_t *my_sig = reinterpret_cast<uint8_t *>(s_U + SH::OFF_SIG) + wave * SIG;
  uint8_t *my_mem = reinterpret_cast<uint8_t *>(s_U + SH::OFF_MEM) + wave * SH::MEM;
  /* score_exact_wave's scratch (matrix-core tiers): 256 bytes per wave over the serial
   * start states, which are dead outside the draw phase */
  uint8_t *my_lst = reinterpret_cast<uint8_t *>(s_U + SH::OFF_MEM) + wave * 256;
  static_assert(!SH::MF || NWV * 256 <= SH::MEMB, "score_exact_wave scratch");

  PERM_PROF_INIT;
  for (;;) {
    __syncthreads();
    if (tid == 0) s_w = (int64_t)atomicAdd(wq, 1u);
    __syncthreads();
    const int64_t w = s_w;
    if (w >= wtotal) {
      PERM_PROF_FLUSH;
      break;
    }
    if (!status[w]) continue;
    PERM_PROF(5); /* work queue and status */
    const int c = perm_chrom_of(ch, nchrom, w);
    const gd_chrom_dev &d = ch[c];
    const int a = d.asize, b = d.bsize, m = a + b, m1 = m - 1;
    const int64_t wl = w - d.w_base;

    const double inva = a > 1 ? 1.0 / (double)(a * a * (a - 1)) : 0.0;
    const double invb = b > 1 ? 1.0 / (double)(b * b * (b - 1)) : 0.0;
    const int g = a <= b ? a : b, goff = a <= b ? 0 : a;
    double obs, inv_sc = 1.0; /* score_mfma: S was scaled by 1 / inv_sc */
    int ln = tid;
    PERM_OPAQUE(ln);
    const double *s_X = SH::MF ? xbuf + w * 2 * MP : s_Xl;
    if constexpr (SH::MF) {
      /* matrix-core tiers: no FP64 triangle.  The scale from the coordinates' bounding
       * box (its diagonal D >= every distance, D < 2^ex), then the scaled fp16 matrix of
       * S, zero outside m x m and on the diagonal, and the observed score by the wave */
      double x0 = __builtin_inf(), x1 = -__builtin_inf(), y0 = __builtin_inf(), y1 = -__builtin_inf();
      for (int i = lane; i < m; i += 64) {
        x0 = fmin(x0, s_X[2 * i]);
        x1 = fmax(x1, s_X[2 * i]);
        y0 = fmin(y0, s_X[2 * i + 1]);
        y1 = fmax(y1, s_X[2 * i + 1]);
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        x0 = fmin(x0, __shfl_xor(x0, o));
        x1 = fmax(x1, __shfl_xor(x1, o));
        y0 = fmin(y0, __shfl_xor(y0, o));
        y1 = fmax(y1, __shfl_xor(y1, o));
      }
      PERM_PROF(7); /* the coordinates and their bounding box */
      const double dmax = sqrt((x1 - x0) * (x1 - x0) + (y1 - y0) * (y1 - y0));
      int ex = 0;
      if (dmax > 0.0) (void)frexp(dmax, &ex);
      const double sc = ldexp(1.0, 15 - ex);
      inv_sc = ldexp(1.0, ex - 15);
      /* in FP32 (fp16 keeps 11 bits: the FP32 distance's ~2^-22 is inside the bound) */
      const float scf = (float)sc;
      constexpr int KC = SH::KT * 16;
#if PERM_S16_PAIRS
      /* zero the whole matrix (padding rows and columns, the diagonal), then every
       * unordered pair once, written to both (x, y) and (y, x): S is symmetric bit for bit
       * (dx and dy only change sign) */
      for (int e = ln; e < SH::S16 / 16; e += NT) reinterpret_cast<uint4 *>(s_U)[e] = make_uint4(0u, 0u, 0u, 0u);
      __syncthreads();
      for (int e = ln; e < m * (m - 1) / 2; e += NT) {
        /* pair e = T(h) + l, h > l: h from the float root of 8e + 1 (within one of the true
         * row for e < 2^24), then corrected */
        int h = (int)((1.0f + __fsqrt_rn(8.0f * (float)e + 1.0f)) * 0.5f);
        if (h * (h - 1) / 2 > e)
          --h;
        else if (h * (h + 1) / 2 <= e)
          ++h;
        const int l = e - h * (h - 1) / 2;
        const float dx = (float)(s_X[2 * h] - s_X[2 * l]), dy = (float)(s_X[2 * h + 1] - s_X[2 * l + 1]);
        float v = __fsqrt_rn(dx * dx + dy * dy) * scf;
        if (v < 0x1p-14f) v = 0.f; /* no fp16 denormals (score_mfma's SUB) */
        const _Float16 hv = (_Float16)v;
        *reinterpret_cast<_Float16 *>(s_U + h * SH::RS + 2 * l) = hv;
        *reinterpret_cast<_Float16 *>(s_U + l * SH::RS + 2 * h) = hv;
      }
#else
      for (int e = ln; e < SH::MT * 32 * KC; e += NT) {
        const int row = e / KC, k = e - row * KC;
        float v = 0.f;
        if (row < m && k < m && row != k) {
          const float dx = (float)(s_X[2 * row] - s_X[2 * k]), dy = (float)(s_X[2 * row + 1] - s_X[2 * k + 1]);
          v = __fsqrt_rn(dx * dx + dy * dy) * scf;
          if (v < 0x1p-14f) v = 0.f; /* no fp16 denormals (score_mfma's SUB) */
        }
        *reinterpret_cast<_Float16 *>(s_U + row * SH::RS + 2 * k) = (_Float16)v;
      }
#endif
      PERM_PROF(6); /* the fp16 matrix */
      const gd_randint rb = gd_randint_make((uint32_t)(b > 1 ? b : 2));
      obs = score_exact_wave<MP>([](int k) { return (uint32_t)k; }, s_X, a, b, inva, invb, lane, my_lst, rb);
      if (tid < m) s_car[tid] = (uint8_t)tid; /* tracks := identity */
      __syncthreads();
    } else {
      /* S (packed triangle, zero rows for individuals >= m) and its row sums */
      for (int e = ln; e < 2 * m; e += NT) s_Xl[e] = xbuf[w * 2 * MP + e];
      __syncthreads();
      /* entry e = T(h) + l of the triangle, e strided over the threads (independent
       * entries, no per-row loop): h from the float root of 8e + 1 (within one of the
       * true row for e < 2^24), then corrected */
      #pragma unroll 4
      for (int e = ln; e < TRI - 1; e += NT) {
        int h = (int)((1.0f + __fsqrt_rn(8.0f * (float)e + 1.0f)) * 0.5f);
        if (h * (h - 1) / 2 > e)
          --h;
        else if (h * (h + 1) / 2 <= e)
          ++h;
        const int l = e - h * (h - 1) / 2;
        const double v = (h < m && l < m) ? perm_xdist(s_X, h, l) : 0.0;
        s_S[e] = v;
      }
      if (tid == 0) s_S[TRI - 1] = 0.0;
      __syncthreads();
      for (int r = ln; r <= MP; r += NT) {
        double acc = 0.0;
        if (r < m) {
          const uint32_t tr = tri8((uint32_t)r);
          /* j ascending, eight loads in flight */
#pragma unroll 1
          for (int j0 = 0; j0 < m; j0 += 8) {
            double e[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const int j = j0 + t;
              e[t] = j < m ? s_pair(s_S, (uint32_t)r, tr, (uint32_t)j, tri8((uint32_t)j)) : 0.0;
            }
#pragma unroll
            for (int t = 0; t < 8; ++t)
              if (j0 + t < m && j0 + t != r) acc += e[t];
          }
        }
        s_R[r] = acc;
      }
      if (tid < m) s_car[tid] = (uint8_t)tid; /* tracks := identity */
      __syncthreads();

      /* the observed score: identity tracks, from the FP64 triangle */
      obs = score_exact<MP, true>(
          [](int k) { return (uint32_t)k; },
          [&](int k) { return k < g ? (uint32_t)(goff + k) : (uint32_t)MP; },
          [&](uint32_t x, uint32_t y) {
            return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(s_S) + tri8(y) + (x << 3));
          },
          s_R, a, b, inva, invb);
      /* FP32 copy of the triangle over the head of the FP64 one, in chunks (the FP32
       * entries of chunk j overlap only FP64 entries of chunks <= j, read before) */
      {
        constexpr int CH = 8;
#pragma unroll 1
        for (int e0 = 0; e0 < TRI; e0 += CH * NT) {
          float v[CH];
#pragma unroll
          for (int i = 0; i < CH; ++i) {
            const int e = e0 + i * NT + ln;
            v[i] = e < TRI ? (float)s_S[e] : 0.f;
          }
          __syncthreads();
#pragma unroll
          for (int i = 0; i < CH; ++i) {
            const int e = e0 + i * NT + ln;
            if (e < TRI) s_S32[e] = v[i];
          }
          __syncthreads();
        }
      }
    }
    PERM_PROF(0);

    uint64_t base = gd_window_state(d.seed, GD_STREAM_CSS, wl + d.w_first);
    const gd_affine Jq = gd_lcg_jump((uint64_t)tid * (uint64_t)m1), JP = gd_lcg_jump((uint64_t)P * (uint64_t)m1);
    int hits = 0, nsc = 0;
    bool done = !(treshold > 0 && runs > 0);
    while (!done) {
      /* 1. draws and Fisher-Yates swaps on sigma_q, q = tid */
      __syncthreads();
      sig_identity<MP>(my_sig, m, lane);
      __syncthreads();
      int lq = lane;
      PERM_OPAQUE(lq);
      uint8_t *col = my_sig + lq;
#if PERM_DIAG_SKIP & 1
      const bool rej = false;
#elif PERM_FY_UNROLL
      /* (not at 64: the straight line raised that tier's VGPRs 160 -> 196, 3 -> 2 waves per SIMD) */
      const bool rej = (MP != 64 && m == MP) ? fy_fast_unrolled<MP>(col, gd_affine_apply(Jq, base))
                                             : fy_fast(col, gd_affine_apply(Jq, base), m, vm0, vm1);
#else
      const bool rej = fy_fast(col, gd_affine_apply(Jq, base), m, vm0, vm1);
#endif
      if (__syncthreads_or(rej)) {
        /* exact serial stream: the start state of every permutation of the pass */
        uint64_t mine;
        if constexpr (SH::MF) {
          /* every thread derives its own (a rare path: no LDS table of start states) */
          mine = serial_advance(base, tid, m, vm0, vm1);
          if (tid == NT - 1) s_next = serial_advance(mine, 1, m, vm0, vm1);
        } else {
          if (tid == 0) {
            uint64_t y = base;
            for (int q = 0; q < P; ++q) {
              s_st[q] = y;
              y = serial_advance(y, 1, m, vm0, vm1);
            }
            s_st[P] = y;
          }
          __syncthreads();
          mine = s_st[tid];
        }
        __syncthreads();
        sig_identity<MP>(my_sig, m, lane);
        __syncthreads();
        fy_exact(col, mine, m);
        base = SH::MF ? s_next : s_st[P];
      } else {
        base = gd_affine_apply(JP, base);
      }
      __syncthreads();
      PERM_PROF(1);

      /* 2. compositions, all waves at once; lane i owns rows i and i + 64.  The wave's 64
       * permutations form PERM_CHAINS chains of consecutive ones (chain u = CH v + c holds
       * q = 64 v + (64 / CH) c + t), composed side by side: with PERM_CHAINS == 1 wave 0
       * composes F_q = F_{q-1} o sigma_q from the carried tracks and wave v > 0 composes
       * G_t = G_{t-1} o sigma_{64v+t} from the identity, its tracks F_{64v+t} = Fs_v o G_t
       * read through the map s_fs[v]; with PERM_CHAINS == 2 every chain starts from the
       * identity and every lane reads through its chain's map (Fs_0 = the carried tracks),
       * which halves the chain of dependent ds_bpermutes */
      if (!(PERM_DIAG_SKIP & 2)) {
        constexpr int CH = PERM_CHAINS, TL = 64 / CH;
        uint32_t pf0[16], pf1[16];
        int li = lane;
        PERM_OPAQUE(li);
        const bool r0 = li < m, r1 = MP > 64 && li + 64 < m;
        /* above 64 individuals lane i carries F(i) and F(i + 64) as the low two bytes of
         * one word, so one ds_bpermute per row fetches whichever of the two is wanted */
        const uint32_t ident = (uint32_t)li | (MP > 64 ? (uint32_t)(li + 64) << 8 : 0u);
        uint32_t car[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) car[c] = ident;
        if (CH == 1 && wave == 0) car[0] = (uint32_t)s_car[li] | (MP > 64 ? (uint32_t)s_car[li + 64] << 8 : 0u);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          pf0[q] = r0 ? *reinterpret_cast<const uint32_t *>(my_sig + li * PERM_ROW + 4 * q) : 0u;
          pf1[q] = r1 ? *reinterpret_cast<const uint32_t *>(my_sig + (li + 64) * PERM_ROW + 4 * q) : 0u;
        }
        /* F_q(i) for q = t .. t+3 leave as one dword per row (bytes t .. t+3 of row i) */
        uint32_t w0[CH], w1[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) w0[c] = w1[c] = 0u;
#pragma unroll
        for (int t = 0; t < TL; ++t) {
#pragma unroll
          for (int c = 0; c < CH; ++c) {
            const int q = TL * c + t;
            const uint32_t s0 = __builtin_amdgcn_ubfe(pf0[q >> 2], 8 * (q & 3), 8);
            uint32_t n0, n1 = 0;
            if constexpr (MP > 64) {
              /* ds_bpermute reads lane (addr >> 2) mod 64; entry s >= 64 is byte 1 of lane
               * s - 64's word: bit field (8 (s >> 6), 8) */
              const uint32_t s1 = __builtin_amdgcn_ubfe(pf1[q >> 2], 8 * (q & 3), 8);
              const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(s0 << 2), (int)car[c]);
              const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(s1 << 2), (int)car[c]);
              n0 = __builtin_amdgcn_ubfe(a0, (s0 >> 3) & 8u, 8);
              n1 = __builtin_amdgcn_ubfe(a1, (s1 >> 3) & 8u, 8);
              w1[c] |= n1 << (8 * (q & 3));
            } else {
              n0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(s0 << 2), (int)car[c]);
            }
            w0[c] |= n0 << (8 * (q & 3));
            if ((q & 3) == 3) {
              if (r0) *reinterpret_cast<uint32_t *>(my_sig + li * PERM_ROW + (q & ~3)) = w0[c];
              if (MP > 64 && r1) *reinterpret_cast<uint32_t *>(my_sig + (li + 64) * PERM_ROW + (q & ~3)) = w1[c];
              w0[c] = 0;
              w1[c] = 0;
            }
            car[c] = n0 | (n1 << 8);
          }
        }
        /* each chain's last composition */
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          uint8_t *gend = s_gend + (CH * wave + c) * MP;
          if (r0) gend[li] = (uint8_t)car[c];
          if (r1) gend[li + 64] = (uint8_t)(car[c] >> 8);
        }
      }
      __syncthreads();
      /* the chain across the chains, wave 0 alone (LDS in issue order: each step reads what
       * the previous one wrote).  PERM_CHAINS == 1: Fs_1 = F_63, Fs_v = Fs_{v-1} o G^{v-1}_63;
       * PERM_CHAINS == 2: Fs_0 = the carried tracks, Fs_u = Fs_{u-1} o G^{u-1}_end.  The carry
       * into the next pass is the last map composed with the last chain's end. */
      if (!(PERM_DIAG_SKIP & 2) && wave == 0) {
        constexpr int NCH = NWV * PERM_CHAINS, U0 = PERM_CHAINS == 1 ? 1 : 0;
        for (int u = U0; u < NCH; ++u) {
          for (int i = lane; i < m; i += 64)
            s_fs[u * MP + i] = u == 0 ? s_car[i] : (U0 == 1 && u == 1) ? s_gend[i]
                                                                        : s_fs[(u - 1) * MP + s_gend[(u - 1) * MP + i]];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        for (int i = lane; i < m; i += 64)
          s_car[i] = NCH == 1 ? s_gend[i] : s_fs[(NCH - 1) * MP + s_gend[(NCH - 1) * MP + i]];
      }
      __syncthreads();
      PERM_PROF(2);
      /* 3. scores of the P permuted track arrays from the FP32 triangle; a lane whose
       * estimate lies within its error bound of obs recomputes the FP64 score with S
       * from the coordinates (the same values the FP64 triangle held), so every hit is
       * decided exactly as score_exact decides it.  4. in-order hit count */
      int lc = lane;
      PERM_OPAQUE(lc);
      const uint8_t *tcol = my_sig + lc;
      uint8_t *mcol = my_mem + lc;
      double est, err;
      /* the lane's chain map (PERM_CHAINS == 1: wave-uniform, none for wave 0) */
      const bool mapped = !(PERM_DIAG_SKIP & 2) && (PERM_CHAINS > 1 || __builtin_amdgcn_readfirstlane(wave) > 0);
      const uint8_t *fmap = s_fs + (PERM_CHAINS * wave + lc / (64 / PERM_CHAINS)) * MP;
      if constexpr ((PERM_DIAG_SKIP & 4) != 0) {
        est = -1e300; /* no hits */
        err = 0.0;
      } else if constexpr (SH::MF) {
        score_mfma<MP>(s16, s_lut, tcol, fmap, mapped, a, b, inva, invb, inv_sc, lane, est, err);
      } else {
        score_f32<MP>(s_S32, s_R, tcol, fmap, mapped, mcol, a, b, inva, invb, est, err);
      }
      if (force_exact) err = __builtin_inf();
      int hit = est - obs > err ? 1 : (obs - est > err ? 0 : -1);
#ifdef PERM_COUNT_AMBIGUOUS /* diagnostics: ambiguous lanes and wave-passes that ran the FP64 path */
      if (hit < 0) atomicAdd(&g_perm_amb[0], 1ull);
      if (__any(hit < 0) && lane == 0) atomicAdd(&g_perm_amb[1], 1ull);
#endif
      if constexpr (SH::MF) {
        /* the rare lanes inside the bound: exact score by the whole wave, one lane at a time */
        uint64_t amb = __ballot(hit < 0);
        if (amb) {
          const gd_randint rb = gd_randint_make((uint32_t)(b > 1 ? b : 2));
          while (amb) {
            const int L = __builtin_ctzll(amb);
            amb &= amb - 1;
            const uint8_t *cl = my_sig + L;
            const uint8_t *fmL = s_fs + (PERM_CHAINS * wave + L / (64 / PERM_CHAINS)) * MP;
            const double sc = score_exact_wave<MP>(
                [&](int k) {
                  const uint32_t c = cl[k * PERM_ROW];
                  return mapped ? (uint32_t)fmL[c] : c;
                },
                s_X, a, b, inva, invb, lane, my_lst, rb);
            if (lane == L) hit = sc >= obs;
          }
        }
      } else if (__any(hit < 0)) {
        if (hit < 0) {
          const double sc = score_exact<MP, false>(
              [&](int k) {
                const uint32_t c = tcol[k * PERM_ROW];
                return mapped ? (uint32_t)fmap[c] : c;
              },
              [&](int k) { return k < g ? (uint32_t)mcol[k * 64] : (uint32_t)MP; },
              [&](uint32_t x, uint32_t y) { return y < (uint32_t)m ? perm_xdist(s_X, (int)y, (int)x) : 0.0; }, s_R,
              a, b, inva, invb);
          hit = sc >= obs;
        }
      }
#ifdef GD_PERM_PROFILE
      __syncthreads();
      PERM_PROF(3);
#endif
      const int valid = min(P, runs - nsc);
      const uint64_t H = __ballot(tid < valid && hit > 0);
      if (lane == 0) s_hit[wave] = H;
      __syncthreads();
      for (int v = 0; v < NWV && !done; ++v) {
        const uint64_t Hv = s_hit[v];
        const int vv = min(64, max(0, valid - 64 * v)); /* valid permutations of wave v */
        const int need = treshold - hits;
        if (!PERM_DIAG_NOEXIT && __popcll(Hv) >= need) {
          uint64_t h = Hv;
          for (int k = 1; k < need; ++k) h &= h - 1;
          nsc += __ffsll((unsigned long long)h); /* position of the need-th hit, + 1 */
          hits = treshold;
          done = true;
        } else {
          hits += __popcll(Hv);
          nsc += vv;
          done = nsc >= runs;
        }
      }
    }
    PERM_PROF(4);
    if (tid == 0) pvals[d.w_out + wl] = (hits + 1) * 1.0 / (nsc + 1);
  }
}

/* ------------------------------------------------------------------------ */
/* The general path (GD_CSS_TIER_MAX < m <= GD_CSS_BIG_MAX): one workgroup of 4 */
/* waves per window (pulled from the work counter), 64 permutations per pass.    */
/* Wave 0 draws them (lane q: Fisher-Yates on its own 16-bit LDS column, start   */
/* state by jump-ahead, the serial stream when a draw is rejected, as            */
/* k_css_perm); the workgroup composes F_q = F_{q-1} o sigma_q row-parallel (one */
/* barrier per step, F_q written over sigma_q); each wave scores every fourth     */
/* track in FP64 with the lanes splitting the a b between-group pairs (S in the   */
/* workgroup's global slab, computed once per window from X); hits are counted in */
/* permutation order, so the early exit stops where the serial loop stops.  The   */
/* observed score is the same function of the identity tracks.                    */
/* ------------------------------------------------------------------------ */
namespace {
/* permutations per pass: 64, 32 at the 1024 tier, 16 at 2048 (the u16 matrix is MP x P) */
template <int MP>
constexpr int pb_p() { return MP > 1024 ? 16 : MP > 512 ? 32 : 64; }

/* Fisher-Yates of random_shuffle (css.c:700-706) on column `col` (stride PB_P), draws
 * from state x without rejection; true if a draw would have been rejected */
template <int PB_P>
__device__ __forceinline__ bool fy_big_fast(uint16_t *col, uint64_t x, int m, const uint32_t *mag) {
  bool rej = false;
  uint64_t y = x << 16;
  for (int s = 0; s < m - 1; ++s) {
    const int n = __builtin_amdgcn_readfirstlane(m - s);
    const gd_randint rd = perm_rd((uint32_t)n, __builtin_amdgcn_readfirstlane(mag[n]));
    y = y * GD_LCG_A + (GD_LCG_C << 16);
    const uint32_t r = (uint32_t)(y >> 33);
    rej |= r > rd.limit;
    const int j = (int)(r - (__umulhi(r, rd.magic) >> rd.shift) * (uint32_t)n);
    const uint16_t u = col[(n - 1) * PB_P], v = col[j * PB_P];
    col[(n - 1) * PB_P] = v;
    col[j * PB_P] = u;
  }
  return rej;
}

/* the same with random_int_nrand48's redraw loop (css.c:675-690) */
template <int PB_P>
__device__ __forceinline__ void fy_big_exact(uint16_t *col, uint64_t x, int m, const uint32_t *mag) {
  for (int s = 0; s < m - 1; ++s) {
    const int n = __builtin_amdgcn_readfirstlane(m - s);
    const gd_randint rd = perm_rd((uint32_t)n, __builtin_amdgcn_readfirstlane(mag[n]));
    uint32_t r;
    do {
      x = gd_lcg_next(x);
      r = gd_lcg_value(x);
    } while (r > rd.limit);
    const int j = (int)gd_randint_mod(&rd, r);
    const uint16_t u = col[(n - 1) * PB_P], v = col[j * PB_P];
    col[(n - 1) * PB_P] = v;
    col[j * PB_P] = u;
  }
}

__device__ __forceinline__ double pb_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

/* css() (css.c:608-647) of one track array by one wave: S(x, y) at y ld + x.
 * The consecutive within-group pairs (Q8) in track order; the between-group sum over the
 * pairs (A_i, B_j) of the two groups' members in ascending order, pair p = i b + j dealt
 * to lane p mod 64 and summed in p order per lane (score_exact_wave's order): a function
 * of the groups' SETS, so a permutation that keeps them scores the observed value bit for
 * bit and its tie is decided as at the register tiers.  fl: m membership bytes, la / lb:
 * the members ascending (the wave's LDS scratch). */
template <class TRK>
__device__ __forceinline__ double pb_score(TRK track, const double *S, int ld, int a, int b, double inva, double invb,
                                           int lane, uint8_t *fl, uint16_t *la, uint16_t *lb) {
  const int ab = a * b, m = a + b;
  for (int k = lane; k < m; k += 64) fl[track(k)] = (uint8_t)(k < a);
  __builtin_amdgcn_wave_barrier();
  const uint64_t below = (1ull << lane) - 1ull;
  int na = 0, nb = 0;
  for (int i0 = 0; i0 < m; i0 += 64) {
    const int i = i0 + lane;
    const bool v = i < m, in = v && fl[i] != 0;
    const uint64_t A = __ballot(in), B = __ballot(v && !in);
    if (in) la[na + __popcll(A & below)] = (uint16_t)i;
    if (v && !in) lb[nb + __popcll(B & below)] = (uint16_t)i;
    na += __popcll(A);
    nb += __popcll(B);
  }
  __builtin_amdgcn_wave_barrier();
  double bet = 0.0, wa = 0.0, wb = 0.0;
  int ii = lane / b, jj = lane - (lane / b) * b;
#pragma unroll 4
  for (int p = lane; p < ab; p += 64) {
    bet += S[(int64_t)lb[jj] * ld + la[ii]];
    jj += 64;
    while (jj >= b) {
      jj -= b;
      ++ii;
    }
  }
  for (int k = lane; k < m - 1; k += 64) {
    const double e = S[(int64_t)track(k + 1) * ld + track(k)];
    if (k < a - 1) wa += e;
    if (k >= a) wb += e;
  }
  bet = pb_wave_sum(bet);
  wa = pb_wave_sum(wa);
  wb = pb_wave_sum(wb);
  __builtin_amdgcn_wave_barrier(); /* the scratch is rewritten by the wave's next score */
  return bet / (double)ab - (double)m * (wa * inva + wb * invb);
}
}  // namespace

template <int MP>
__global__ void __launch_bounds__(256)
    k_css_perm_big(const gd_chrom_dev *ch, int nchrom, const double *xbuf, int xstride, const uint8_t *status,
                   int64_t wtotal, int treshold, int runs, double *pvals, unsigned *wq, double *slab,
                   int64_t slab_per_wg, int ld) {
  constexpr int NT = 256, P = pb_p<MP>();
  __shared__ uint16_t s_sig[MP * P]; /* element k of column q at k P + q */
  __shared__ uint16_t s_F[2][MP];    /* the carried tracks, double-buffered while composing */
  __shared__ double s_X[2 * MP];
  __shared__ uint32_t s_mag[MP + 1];
  __shared__ uint64_t s_st[P + 1];
  __shared__ int s_hitq[P];
  __shared__ double s_obs;
  __shared__ int64_t s_w;
  __shared__ int s_ctl[3]; /* hits, permutations run, done */
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  /* pb_score's scratch over s_X (dead once S is in the slab): per wave MP u16 for the
   * members ascending (group A's, then group B's at offset a) and MP membership bytes */
  static_assert(NT / 64 * 3 * MP <= (int)sizeof(s_X), "pb_score scratch");
  uint16_t *s_ls = reinterpret_cast<uint16_t *>(s_X) + wave * MP;
  uint8_t *s_fl = reinterpret_cast<uint8_t *>(s_X) + (NT / 64) * 2 * MP + wave * MP;
  double *S = slab + (int64_t)blockIdx.x * slab_per_wg;
  for (int n = tid; n <= MP; n += NT) s_mag[n] = gd_randint_make(n < 1 ? 1u : (uint32_t)n).magic;

  for (;;) {
    __syncthreads();
    if (tid == 0) s_w = (int64_t)atomicAdd(wq, 1u);
    __syncthreads();
    const int64_t w = s_w;
    if (w >= wtotal) break;
    if (!status[w]) continue;
    const int c = perm_chrom_of(ch, nchrom, w);
    const gd_chrom_dev &d = ch[c];
    const int a = d.asize, b = d.bsize, m = a + b, m1 = m - 1;
    if (m > MP || m > ld) continue; /* the MDS stage flagged it and wrote no coordinates */
    const int64_t wl = w - d.w_base;
    for (int e = tid; e < 2 * m; e += NT) s_X[e] = xbuf[w * xstride + e];
    for (int i = tid; i < m; i += NT) s_F[0][i] = (uint16_t)i; /* tracks := identity */
    __syncthreads();
    /* S = calc_dist(X) (css.c:573-587), symmetric bit for bit */
    for (int e = tid; e < m * m; e += NT) {
      const int x = e % m, y = e / m;
      S[(int64_t)y * ld + x] = x == y ? 0.0 : perm_xdist(s_X, x, y);
    }
    __threadfence_block();
    __syncthreads();
    const double inva = a > 1 ? 1.0 / (double)(a * a * (a - 1)) : 0.0;
    const double invb = b > 1 ? 1.0 / (double)(b * b * (b - 1)) : 0.0;
    if (wave == 0) {
      const double o = pb_score([](int k) { return k; }, S, ld, a, b, inva, invb, lane, s_fl, s_ls, s_ls + a);
      if (lane == 0) s_obs = o;
    }
    if (tid == 0) {
      s_ctl[0] = 0;
      s_ctl[1] = 0;
      s_ctl[2] = !(treshold > 0 && runs > 0);
    }
    __syncthreads();
    const double obs = s_obs;
    uint64_t base = gd_window_state(d.seed, GD_STREAM_CSS, wl + d.w_first);
    const gd_affine Jq = gd_lcg_jump((uint64_t)lane * (uint64_t)m1), JP = gd_lcg_jump((uint64_t)P * (uint64_t)m1);
    int cur = 0;
    while (!s_ctl[2]) {
      /* 1. draws: wave 0, lane q -> sigma_q in column q */
      uint16_t *col = s_sig + lane;
      bool rej = false;
      if (wave == 0 && lane < P) {
        for (int k = 0; k < m; ++k) col[k * P] = (uint16_t)k;
        rej = fy_big_fast<P>(col, gd_affine_apply(Jq, base), m, s_mag);
      }
      if (__syncthreads_or(rej)) {
        if (tid == 0) {
          uint64_t y = base;
          for (int q = 0; q < P; ++q) {
            s_st[q] = y;
            for (int s2 = 0; s2 < m1; ++s2) {
              const gd_randint rd = perm_rd((uint32_t)(m - s2), s_mag[m - s2]);
              do y = gd_lcg_next(y);
              while (gd_lcg_value(y) > rd.limit);
            }
          }
          s_st[P] = y;
        }
        __syncthreads();
        if (wave == 0 && lane < P) {
          for (int k = 0; k < m; ++k) col[k * P] = (uint16_t)k;
          fy_big_exact<P>(col, s_st[lane], m, s_mag);
        }
        base = s_st[P];
      } else {
        base = gd_affine_apply(JP, base);
      }
      __syncthreads();
      /* 2. compositions F_q = F_{q-1} o sigma_q, F_q over sigma_q */
      for (int q = 0; q < P; ++q) {
        for (int i = tid; i < m; i += NT) {
          const uint16_t v = s_F[cur][s_sig[i * P + q]];
          s_F[cur ^ 1][i] = v;
          s_sig[i * P + q] = v;
        }
        cur ^= 1;
        __syncthreads();
      }
      /* 3. scores: wave v takes tracks v, v + 4, ... */
      for (int q = wave; q < P; q += NT / 64) {
        const double sc = pb_score([&](int k) { return (int)s_sig[k * P + q]; }, S, ld, a, b, inva, invb, lane,
                                   s_fl, s_ls, s_ls + a);
        if (lane == 0) s_hitq[q] = sc >= obs;
      }
      __syncthreads();
      /* 4. hits in permutation order, early exit at the treshold-th hit */
      if (tid == 0) {
        int hits = s_ctl[0], nsc = s_ctl[1];
        const int valid = min(P, runs - nsc);
        bool done = false;
        for (int q = 0; q < valid && !done; ++q) {
          hits += s_hitq[q];
          ++nsc;
          done = hits >= treshold;
        }
        s_ctl[0] = hits;
        s_ctl[1] = nsc;
        s_ctl[2] = done || nsc >= runs;
      }
      __syncthreads();
    }
    if (tid == 0) pvals[d.w_out + wl] = (s_ctl[0] + 1) * 1.0 / (s_ctl[1] + 1);
  }
}

template <int MP>
static int launch_perm(const gd_chrom_dev *d_ch, int nchrom, const double *xbuf, const uint8_t *status, int64_t wtotal,
                       int treshold, int runs, double *p, unsigned *wq, hipStream_t s) {
  /* GD_PERM_EXACT=1: every permuted score in FP64 (checks that the FP32 pre-filter
   * changes no p-value) */
  const char *fe = getenv("GD_PERM_EXACT");
  const int force_exact = fe && fe[0] == '1' ? 1 : 0;
  const unsigned grid = (unsigned)std::min<int64_t>(wtotal, 256 * 16);
  hipLaunchKernelGGL(k_css_perm<MP>, dim3(grid), dim3(PermShape<MP>::NT), 0, s, d_ch, nchrom, xbuf, status, wtotal,
                     treshold, runs, p, wq, force_exact);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

int gd_css_perm_launch(int mp, const gd_chrom_dev *d_ch, int nchrom, const double *xbuf, const uint8_t *status,
                       int64_t wtotal, int treshold, int runs, double *p, unsigned *wq, double *slab, hipStream_t s) {
#ifdef GD_PERM_PROFILE
  {
    static const unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_perm_prof), z, sizeof z, 0, hipMemcpyHostToDevice, s);
  }
  struct Dump {
    hipStream_t s;
    ~Dump() {
      unsigned long long h[8];
      (void)hipStreamSynchronize(s);
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_perm_prof), sizeof h);
      fprintf(stderr,
              "perm-prof cycles: setup %llu draws %llu compose %llu score %llu hits %llu (setup parts: queue+status %llu "
              "coordinates %llu fp16 matrix %llu; the rest is the observed score)\n",
              h[0], h[1], h[2], h[3], h[4], h[5], h[7], h[6]);
    }
  } dump{s};
#endif
#ifdef PERM_COUNT_AMBIGUOUS
  struct DumpAmb {
    hipStream_t s;
    ~DumpAmb() {
      unsigned long long h[2];
      (void)hipStreamSynchronize(s);
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_perm_amb), sizeof h);
      fprintf(stderr, "perm ambiguous lanes %llu, wave-passes with an FP64 recompute %llu (cumulative)\n", h[0], h[1]);
    }
  } dump_amb{s};
#endif
  switch (mp) {
    case 24: return launch_perm<24>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 40: return launch_perm<40>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 64: return launch_perm<64>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 80: return launch_perm<80>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 96: return launch_perm<96>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 128: return launch_perm<128>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
  }
  if (mp > GD_CSS_TIER_MAX && mp <= GD_CSS_BIG_MAX) {
    const unsigned grid = (unsigned)gd_css_big_grid(wtotal, mp);
    const int64_t per = gd_css_big_slab_per_wg(mp);
    const int ld = gd_css_big_ld(mp);
    if (mp <= 256)
      hipLaunchKernelGGL(k_css_perm_big<256>, dim3(grid), dim3(256), 0, s, d_ch, nchrom, xbuf, 2 * mp, status, wtotal,
                         treshold, runs, p, wq, slab, per, ld);
    else if (mp <= 512)
      hipLaunchKernelGGL(k_css_perm_big<512>, dim3(grid), dim3(256), 0, s, d_ch, nchrom, xbuf, 2 * mp, status, wtotal,
                         treshold, runs, p, wq, slab, per, ld);
    else if (mp <= 1024)
      hipLaunchKernelGGL(k_css_perm_big<1024>, dim3(grid), dim3(256), 0, s, d_ch, nchrom, xbuf, 2 * mp, status,
                         wtotal, treshold, runs, p, wq, slab, per, ld);
    else
      hipLaunchKernelGGL(k_css_perm_big<2048>, dim3(grid), dim3(256), 0, s, d_ch, nchrom, xbuf, 2 * mp, status,
                         wtotal, treshold, runs, p, wq, slab, per, ld);
    return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
  }
  return GD_ERR_SIZE;
}
