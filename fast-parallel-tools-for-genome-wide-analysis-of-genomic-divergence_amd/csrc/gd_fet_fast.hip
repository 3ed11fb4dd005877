/*
 * gd_fet_fast.hip -- fast window path of the FET scan: window percentile and the
 * 100-replicate bootstrap stddev (cFisher.c:136-144, 547-597) without sorting.
 *
 * Why it is exact.  percentile() sorts the window's SNP scores S ascending and the
 * bootstrap draws indices into that SORTED array (Q6, cFisher.c:188,194,569).  The
 * sorted replicate therefore equals S evaluated at the sorted sampled indices, so
 * its idx-th and (idx+1)-th elements are S[t_{m-1}] and S[t_{m-2}], where t_0 >=
 * t_1 >= ... are the sampled indices in descending order and m = n - idx
 * (m ~ 3-4 at perc 0.95).  Each lane keeps the MT largest indices of its
 * replicate in registers (one v_med3_i32 per slot per draw); no sort, no histogram.
 * The window's top-KTOP scores are ranked once into LDS (a bitonic sort across
 * the window's 8 lanes for n <= 64).
 *
 * Parallel RNG.  nrand48 is x -> (a x + c) mod 2^48; lane q of a window starts
 * its replicates at stream position 13*q*n via an affine jump (gd_lcg_jump), so
 * the 8 lanes of a window reproduce the reference's single sequential stream.
 * A rejected draw (r > RAND_MAX - 2^31 mod n, probability ~n/2^31) would shift
 * every later draw: such a window is handed to the literal general path, as are
 * windows with NaN scores, n < 2, n > NFAST, m > 8, misaligned A/B rows, or a
 * replicate whose order statistic falls below the ranked top-KTOP.
 *
 * Layout: 256-thread workgroup = 32 consecutive windows of one chromosome x 8
 * lanes; lanes run 13 of the window's 100 replicates (the last 9).  Windows are assigned
 * to lane groups in order of n, so the windows sharing a wave run loops of similar
 * length.  The SNP scores the 32 windows touch (a contiguous row span) are staged
 * in LDS once.  Per draw: 4 VALU for the LCG step (FW_DRAW), 2 for an order key
 * that sorts like r mod n (fw_key: no remainder is formed inside the loop), MT (4, 5
 * or 8, chosen per wave) for the order statistics, 1/2 for the rejection maximum.
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_fet_rows.h"
#include "gd_internal.h"

#ifndef FW_WPB
#define FW_WPB 32    /* windows per workgroup (sorted by (m, n) into waves of 8; 64 measured slower) */
#endif
#define FW_TPW 8     /* lanes per window (10 and 4 measured 35% / 22% slower) */
#define FW_RPT 12    /* whole replicates per lane: 8*12 = 96 */
#define FW_HALF (FW_TPW / 2) /* replicates 96..99 drawn as halves by lane pairs (2j, 2j + 1) */
#define FW_KTOP 24   /* ranked top scores kept per window (P(needing more) < 1e-9 per replicate) */
#define FW_NFAST 256 /* largest window handled here */
#ifndef FW_SPAN
#define FW_SPAN 1024 /* staged SNP rows per workgroup (32 windows need ~400 at 50 SNPs/window) */
#endif
#ifndef FW_STAGE_U
#define FW_STAGE_U 4 /* 16-byte loads in flight per lane while staging the span */
#endif
#define FW_MAXREJ 8  /* rejected draws tracked per window before giving up */

#define FW_BAD_GENERAL 1 /* hand the window to the literal general path */
#define FW_BAD_REJECT 2  /* a draw was rejected: redo with corrected offsets (B') */

#ifdef GD_FET_PROFILE
/* diagnostics build only: shader-clock cycles per phase summed over workgroups (thread 0) */
__device__ unsigned long long g_fet_prof[8];
#define FW_PROF_INIT uint64_t prof_t = __builtin_readcyclecounter()
#define FW_PROF(ph)                                                   \
  do {                                                                \
    if (threadIdx.x == 0) {                                           \
      const uint64_t t_ = __builtin_readcyclecounter();              \
      atomicAdd(&g_fet_prof[ph], (unsigned long long)(t_ - prof_t)); \
      prof_t = t_;                                                    \
    }                                                                 \
  } while (0)
#else
#define FW_PROF_INIT
#define FW_PROF(ph)
#endif

namespace {

__device__ __forceinline__ int chrom_of_fast(const gd_chrom_dev *ch, int nchrom, int64_t g) {
  int lo = 0, hi = nchrom - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ch[mid].w_base <= g)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

/* median of three; with a >= b it is the insertion step max(b, min(a, v)) */
__device__ __forceinline__ int med3i(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

template <int MT>
__device__ __forceinline__ void top_insert(int (&K)[MT], int v) {
#pragma unroll
  for (int i = MT - 1; i > 0; --i) K[i] = med3i(K[i - 1], K[i], v);
  K[0] = max(K[0], v);
}

/* r mod n for n >= 2 (gd_randint_mod without the n == 1 mask) */
__device__ __forceinline__ int fmod_n(uint32_t r, uint32_t magic, uint32_t shift, uint32_t n) {
  const uint32_t q = __umulhi(r, magic) >> shift;
  return (int)(r - q * n);
}

/* The LCG runs on y = x << 16 (mod 2^64): y' = a*y + (c << 16) keeps the 48-bit
 * nrand48 state in the top 48 bits, so no masking is needed and the 31-bit draw
 * x' >> 17 is simply the high word >> 1.  Per step: one v_mad_u64_u32, one
 * v_mul_lo_u32, one v_lshl_add (a's high part is 5), one v_add3. */
#define FW_C16 (GD_LCG_C << 16)

/* one LCG step on the 32-bit halves of y: lo*a_lo + c16 as one v_mad_u64_u32,
 * the high word gets hi*a_lo (v_mul_lo_u32) and lo*5 (a's high part; v_lshl_add) */
#ifndef FW_LCG_MAD
#define FW_LCG_MAD 1
#endif
/* MAD: the same step as two v_mad_u64_u32 and one v_mad_u32_u24 (+ a shift): ylo's low 16
 * bits are 0 (y = x << 16), so 5 ylo + hi(t) = (ylo >> 16) (5 << 16) + hi(t) is a 24-bit
 * multiply-add, and a_lo yhi + that is the low word of one v_mad_u64_u32 whose addend is a
 * fresh register pair (its high word is don't-care: only the low word of the result is
 * used).  14 issue cycles per step against 16 (ubench: the multiplies and VOP3 adds are
 * 4-cycle instructions, the shift 2). */
template <bool MAD>
__device__ __forceinline__ void fw_step(uint32_t &ylo, uint32_t &yhi, uint32_t a_lo) {
  const uint64_t t = (uint64_t)ylo * 0xDEECE66Du + FW_C16;
  if constexpr (MAD) {
    const uint32_t s = __umul24(ylo >> 16, 5u << 16) + (uint32_t)(t >> 32);
    uint64_t acc;
    asm volatile("" : "=v"(acc)); /* a fresh pair, high word undefined */
    acc = (acc & 0xFFFFFFFF00000000ull) | s;
    asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(yhi), "s"(a_lo) : "vcc");
    yhi = (uint32_t)acc;
  } else {
    yhi = (uint32_t)(t >> 32) + yhi * 0xDEECE66Du + ylo * 5u;
  }
  ylo = (uint32_t)t;
}
/* the MAD step where the top list holds at most FW_LCG_MAD_MT keys (4: nearly every wave); in
 * the MT = 5 / 8 loops its extra registers pushed the 7-wave kernel into scratch (2-4 VGPRs,
 * ~0.2 GB of scratch traffic per C2 scan) */
#define FW_STEP() fw_step<FW_LCG_MAD && (MT <= FW_LCG_MAD_MT)>(ylo, yhi, a_lo)
#ifndef FW_LCG_MAD_MT
#define FW_LCG_MAD_MT 4
#endif
#define FW_LCG_DECL const uint32_t a_lo = __builtin_amdgcn_readfirstlane(0xDEECE66Du)

/* Order key of a draw without the remainder.  The draw is r = yhi >> 1 and the
 * sampled index r mod n; yhi = 2r + (yhi & 1) gives yhi mod 2n = 2 (r mod n) + bit,
 * so ordering by u mod D (u = yhi, D = 2n) orders the sampled indices.  With
 * M = ceil(2^64 / D) (Lemire's fastmod constant), L = M*u mod 2^64 equals
 * (u mod D) 2^64/D + e with 0 <= e < u < 2^32, so key = L >> 32 grows strictly with
 * u mod D (consecutive residues lie >= 2^32/D >= 2^23 apart) and
 * u mod D = ((key + 1) D) >> 32.  Two VALU per draw (v_mul_hi_u32, v_mad_u64_u32)
 * instead of the remainder's four. */
__device__ __forceinline__ uint32_t fw_key(uint32_t u, uint32_t m_lo, uint32_t m_hi) {
  return __umulhi(m_lo, u) + m_hi * u;
}
__device__ __forceinline__ int fw_key_index(uint32_t key, uint32_t D) {
  return (int)((((uint64_t)key + 1) * D) >> 33); /* (u mod D) >> 1 = r mod n */
}
__device__ __forceinline__ int64_t fw_key16_index(uint32_t key, uint32_t D) {
  return (int64_t)((((uint64_t)key + 1) * D) >> 17); /* the same from a 16-bit key (~0: no key) */
}

/* FW_KEY16: the top list holds 16-bit keys (the low halves of its registers) and inserts with
 * v_min_u16 / v_max_u16, 2-cycle instructions (ubench), 2 MT - 1 of them, where the u32 form
 * issues MT 4-cycle v_med3_u32 / v_max_u32.  The key's low 16 bits suffice when M is taken as
 * M16 = ceil(2^48 / D) = ceil(M / 2^16): then (M16 u mod 2^64) >> 32 has bits 32..47 of
 * M16 u mod 2^48 in its low half, key16 = floor(2^16 frac(u / D + e)) with 0 <= e < 2^-16, so
 * consecutive residues lie >= 2^16 / D - 1 >= 127 apart (D <= 512) and
 * u mod D = ((key16 + 1) D) >> 16 (tests/test_fet_key.py pins both for every n).  Off by
 * default: bit-exact on the FET GPU suite, but C2 2.36-2.39 against 2.34-2.35 ms/step (the
 * seven 16-bit ops cost more than the four VOP3 ones they replace in this instruction mix). */
#ifndef FW_KEY16
#define FW_KEY16 0
#endif
__device__ __forceinline__ uint32_t min16(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t max16(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int MT>
__device__ __forceinline__ void top_insert_u(uint32_t (&K)[MT], uint32_t v) {
#if FW_KEY16
  /* the value displaced from slot i moves on to slot i + 1 */
#pragma unroll
  for (int i = 0; i < MT - 1; ++i) {
    const uint32_t t = min16(K[i], v);
    K[i] = max16(K[i], v);
    v = t;
  }
  K[MT - 1] = max16(K[MT - 1], v);
#else
#pragma unroll
  for (int i = MT - 1; i > 0; --i) K[i] = max(min(K[i - 1], K[i]), min(max(K[i - 1], K[i]), v)); /* v_med3_u32 */
  K[0] = max(K[0], v);
#endif
}

/* one draw: advance, order key, insert into the top-MT list */
#define FW_DRAW(MT)                          \
  do {                                       \
    FW_STEP();                               \
    ymax = max(ymax, yhi);                   \
    top_insert_u<MT>(K, fw_key(yhi, mlo, mhi)); \
  } while (0)

/* The index pair a replicate reads from the window's ranked top scores (ranks
 * a - base and b - base, each < FW_KTOP), kept in LDS per replicate: phase C rebuilds
 * the replicate values from them, so the draw loop holds no per-replicate registers. */
__device__ __forceinline__ uint16_t rix_pack(int a, int b, int base) {
  return (uint16_t)(max(a - base, 0) | (max(b - base, 0) << 8));
}

/* Draws `len` values of one replicate (wave-uniform bounds lo8 <= len <= hi) into the
 * top-MT list K */
template <int MT>
__device__ __forceinline__ void draw_rep(uint32_t &ylo, uint32_t &yhi, uint32_t (&K)[MT], int len, int lo8, int hi,
                                         uint32_t mlo, uint32_t mhi, uint32_t &ymax) {
#pragma unroll
  for (int i = 0; i < MT; ++i) K[i] = 0u;
  FW_LCG_DECL;
  int j = 0;
  for (; j < lo8; j += 8) {
    FW_DRAW(MT);
    FW_DRAW(MT);
    FW_DRAW(MT);
    FW_DRAW(MT);
    FW_DRAW(MT);
    FW_DRAW(MT);
    FW_DRAW(MT);
    FW_DRAW(MT);
  }
  for (; j < hi; ++j)
    if (j < len) FW_DRAW(MT);
}

/* The rank pair of order statistics m-1, m-2 of a replicate's top list, packed as
 * rix_pack does, in four VALU: the index recovery (key + 1) D >> 33 and the
 * subtraction of base are one v_mad_u64_u32 each, scaled by 2^7 so that rank - base
 * lands in byte 1 of the high word (D 2^7 = 256 n < 2^17, (key + 1) D 2^7 < 2^49), and
 * one v_perm_b32 joins the two bytes.  A rank below base leaves a wrapped byte, but
 * its window goes to the general path: wkey keeps the smallest key read (keys grow
 * with the index), checked once per lane.  MU > 0: the wave's common m, the register
 * picks are static; MU = 0: per-lane m. */
template <int MT, int MU>
__device__ __forceinline__ uint16_t pick_rix(const uint32_t (&K)[MT], int m, uint32_t D7, uint64_t add7,
                                             uint32_t &wkey) {
  uint32_t ka = K[0], kb = K[0];
  if (MU > 0) {
    ka = K[MU - 1];
    kb = K[MU >= 2 ? MU - 2 : 0];
  } else {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (i == m - 1) ka = K[i];
      if (i == m - 2) kb = K[i];
    }
  }
#if FW_KEY16
  /* (key16 + 1) D 2^7 - base 2^24 (mod 2^32): rank - base in byte 3 (the product is below 2^33,
   * the fraction below 2^24, so the wrap keeps the byte) */
  ka &= 0xFFFFu;
  kb &= 0xFFFFu;
  wkey = min(wkey, ka);
  const uint32_t a32 = (uint32_t)add7;
  const uint32_t ha = __umul24(ka, D7) + a32, hb = __umul24(kb, D7) + a32;
  return (uint16_t)__builtin_amdgcn_perm(hb, ha, 0x0C0C0703u);
#else
  wkey = min(wkey, ka); /* a = t_{m-1} <= b = t_{m-2}: the lowest index read */
  const uint32_t ha = (uint32_t)(((uint64_t)ka * D7 + add7) >> 32), hb = (uint32_t)(((uint64_t)kb * D7 + add7) >> 32);
  return (uint16_t)__builtin_amdgcn_perm(hb, ha, 0x0C0C0501u);
#endif
}

/* Lane q's replicates: whole replicates 12q .. 12q + 11 from y (stream position 12qn),
 * then half of replicate 96 + q/2 from yh (its first floor(n/2) draws for even q, the
 * rest for odd q); the lane pair merges its two top lists (DPP quad_perm [1,0,3,2])
 * and the even lane stores the replicate's rank pair.  8 lanes x 12.5 replicates: no
 * idle replicate slot (13 per lane left 4 of 104 idle).  The draw loops run
 * wave-uniform trip counts (scalar loop control): lo8 = 8 floor(min / 8) draws
 * unrolled by 8 for every lane, then draws up to the wave's largest count with lanes
 * past their own masked off.  ymax collects the high words; a draw was rejected iff
 * (ymax >> 1) > limit.  muni: the wave's common m (scalar), 0 when its windows differ. */
template <int MT, int MU>
__device__ __forceinline__ void boot_lane(uint64_t y, uint64_t yh, int n, int nlo8, int nhi, int hlen, int hlo8,
                                          int hhi, uint64_t M, int m, int base, uint16_t *rix, uint16_t *rix_half,
                                          bool store_half, uint32_t &ymax, uint32_t &wkey) {
#if FW_KEY16
  const uint64_t MK = (M + 0xFFFFu) >> 16; /* ceil(2^48 / 2n) */
  const uint32_t mlo = (uint32_t)MK, mhi = (uint32_t)(MK >> 32), D7 = 256u * (uint32_t)n;
  const uint64_t add7 = (uint32_t)(D7 - ((uint32_t)base << 24));
#else
  const uint32_t mlo = (uint32_t)M, mhi = (uint32_t)(M >> 32), D7 = 256u * (uint32_t)n;
  const uint64_t add7 = (uint64_t)D7 - ((uint64_t)base << 40);
#endif
  uint32_t ylo = (uint32_t)y, yhi = (uint32_t)(y >> 32);
#pragma unroll 2
  for (int k = 0; k < FW_RPT; ++k) {
    uint32_t K[MT];
    draw_rep<MT>(ylo, yhi, K, n, nlo8, nhi, mlo, mhi, ymax);
    rix[k] = pick_rix<MT, MU>(K, m, D7, add7, wkey);
  }
  ylo = (uint32_t)yh;
  yhi = (uint32_t)(yh >> 32);
  uint32_t K[MT];
  draw_rep<MT>(ylo, yhi, K, hlen, hlo8, hhi, mlo, mhi, ymax);
  uint32_t P[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) P[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)K[i], 0xB1, 0xF, 0xF, false);
#pragma unroll
  for (int i = 0; i < MT; ++i) top_insert_u<MT>(K, P[i]);
  const uint16_t w = pick_rix<MT, MU>(K, m, D7, add7, wkey);
  if (store_half) *rix_half = w;
}

/* Per-n constants of the draw loop, built once per device (k_fet_ntab_build):
 * the rejection limit RAND_MAX - 2^31 mod n (cFisher.c:547-554), Lemire's
 * M = ceil(2^64 / 2n), and the nrand48 jumps to lane q's stream positions as affine
 * maps x -> mul*x + add (mod 2^48): 12qn (its first whole replicate) and
 * fw_half_start (its half replicate). */
__device__ uint32_t g_ntab_limit[FW_NFAST + 1];
__device__ uint64_t g_ntab_M[FW_NFAST + 1];
__device__ uint64_t g_ntab_jmul[FW_NFAST + 1][FW_TPW];
__device__ uint64_t g_ntab_jadd[FW_NFAST + 1][FW_TPW];
__device__ uint64_t g_ntab_hmul[FW_NFAST + 1][FW_TPW];
__device__ uint64_t g_ntab_hadd[FW_NFAST + 1][FW_TPW];

/* stream position and length of lane q's half replicate (replicate 96 + q/2) */
__device__ __forceinline__ int64_t fw_half_start(int q, int n) {
  return (int64_t)(FW_TPW * FW_RPT + (q >> 1)) * n + ((q & 1) ? (n >> 1) : 0);
}
__device__ __forceinline__ int fw_half_len(int q, int n) { return (q & 1) ? n - (n >> 1) : (n >> 1); }

/* Rare second pass for a window whose stream contains rejected draws
 * (random_int_nrand48 redraws while r > limit, cFisher.c:550-552): every draw
 * loops until accepted, starting from the lane's corrected stream position.  One
 * replicate's `len` draws into the index list K (top 8, descending). */
__device__ void draw_rep_rejecting(uint64_t &y, int len, const gd_randint &rd, int (&K)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) K[i] = -1;
  for (int j = 0; j < len; ++j) {
    uint32_t hi;
    do {
      y = y * GD_LCG_A + FW_C16;
      hi = (uint32_t)(y >> 32);
    } while ((hi >> 1) > rd.limit);
    top_insert<8>(K, fmod_n(hi >> 1, rd.magic, rd.shift, rd.n));
  }
}
__device__ __forceinline__ uint16_t pick_rix_idx(const int (&K)[8], int m, int base, int &worst) {
  int a = K[0], b = K[0];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i == m - 1) a = K[i];
    if (i == m - 2) b = K[i];
  }
  worst = min(worst, a);
  return rix_pack(a, b, base);
}

__global__ void k_fet_ntab_build() {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n > FW_NFAST) return;
  const uint32_t nn = n > 0 ? (uint32_t)n : 1u;
  g_ntab_limit[n] = GD_RAND_MAX - (uint32_t)(0x80000000ULL % nn);
  g_ntab_M[n] = ~0ULL / (2ull * nn) + 1;
  for (int q = 0; q < FW_TPW; ++q) {
    const gd_affine f = gd_lcg_jump((uint64_t)q * FW_RPT * nn);
    g_ntab_jmul[n][q] = f.mul;
    g_ntab_jadd[n][q] = f.add;
    const gd_affine h = gd_lcg_jump((uint64_t)fw_half_start(q, (int)nn));
    g_ntab_hmul[n][q] = h.mul;
    g_ntab_hadd[n][q] = h.add;
  }
}

}  // namespace

/* 8-lane DPP max-reduction partners within a lane group: xor 1, xor 2, mirror in 8 */
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = gd_f64_bits(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return gd_f64_from(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
/* the same exchange for patterns whose every lane has a source (quad_perm,
 * row_half_mirror): bound_ctrl DPP movs, so no "old" value is materialised or copied
 * per exchange */
template <int CTRL>
__device__ __forceinline__ double dpp_f64_full(double v) {
  const uint64_t u = gd_f64_bits(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
  return gd_f64_from(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
/* v_max_f64 / v_min_f64 without the canonicalisation fmax/fmin add in front of every
 * operand: a window with a NaN score is handed to the general path anyway */
__device__ __forceinline__ double fw_max(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double fw_min(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ double group8_max(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));  /* quad_perm [1,0,3,2] */
  v = fmax(v, dpp_f64<0x4E>(v));  /* quad_perm [2,3,0,1] */
  v = fmax(v, dpp_f64<0x141>(v)); /* row_half_mirror: lane i <-> 7-i */
  return v;
}

/* Per-SNP scores of chromosome rows [r0, r0 + nrows) (nrows <= FW_SPAN) into
 * dst[0 .. nrows): fetcount (cFisher.c:208-238) as LDS atomics into one word per
 * row holding four byte counters (majA, minA, majB, minB; population sizes < 256),
 * then the score-table lookup (the caller checked that the table holds these sizes).
 * The workgroup's waves stream the rows' A and B values with four 16-byte loads per
 * lane in flight; a value's row is one v_mul_hi_u32 by ceil(2^32 / size), exact for
 * the < 2^18 element offsets of a span. */
__device__ void fw_stage_scores(const gd_chrom_dev &d, int r0, int nrows, const double *avals, const double *bvals,
                                const double *lut, uint32_t *cnt, double *dst) {
  constexpr int NT = FW_WPB * FW_TPW, NW = NT / 64;
  const int asize = d.asize, bsize = d.bsize;
  const int lut_nb = (bsize + 1) * (bsize + 2) / 2;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (nrows <= 0) return; /* workgroup-uniform: no fast window, no span */
  for (int r = threadIdx.x; r < nrows; r += NT) cnt[r] = 0;
  __syncthreads();
#pragma unroll
  for (int pop = 0; pop < 2; ++pop) {
    const int size = pop ? bsize : asize;
    const uint32_t rmul = (uint32_t)((0xFFFFFFFFull + size) / size); /* ceil(2^32 / size) */
    const uint32_t inc3 = 1u << (16 * pop), incm3 = 1u << (16 * pop + 8);
    const double *vals = pop ? bvals : avals;
    const int64_t start = (pop ? d.b_off : d.a_off) + (int64_t)r0 * size;
    const int64_t stop = start + (int64_t)nrows * size;
    const int64_t gb = start & ~(int64_t)1; /* 16-byte aligned element */
    const int rel0 = (int)(gb - start);     /* 0 or -1 */
    const int nel = (int)(stop - start);
    const int nch = (int)((stop - gb + 127) >> 7);
    const int nfull = (int)((stop - gb) >> 7); /* chunks wholly inside [gb, stop) */
    const double2 *v2 = reinterpret_cast<const double2 *>(vals + gb);
    /* full chunks: only x of chunk 0, lane 0 can fall outside (element start - 1 of
     * an odd start); the partial last chunk also masks elements past the span */
    auto count_pair = [&](double x, double y, int k, bool partial) {
      const int rel = rel0 + (k << 7) + 2 * lane; /* element offset of x from start */
      uint32_t ix = x == 3.0 ? inc3 : (x == -3.0 ? incm3 : 0u);
      uint32_t iy = y == 3.0 ? inc3 : (y == -3.0 ? incm3 : 0u);
      int relx = max(rel, 0), rely = rel + 1;
      if (rel < 0) ix = 0;
      if (partial) {
        if (rel + 1 >= nel) iy = 0;
        if (rel >= nel) ix = 0;
        relx = min(relx, nel - 1);
        rely = min(rely, nel - 1);
      }
      atomicAdd(&cnt[__umulhi((uint32_t)relx, rmul)], ix);
      atomicAdd(&cnt[__umulhi((uint32_t)rely, rmul)], iy);
    };
    for (int k0 = wave; k0 < nfull; k0 += FW_STAGE_U * NW) {
      double2 v[FW_STAGE_U];
#pragma unroll
      for (int u = 0; u < FW_STAGE_U; ++u) v[u] = v2[min(k0 + u * NW, nfull - 1) * 64 + lane];
#pragma unroll
      for (int u = 0; u < FW_STAGE_U; ++u)
        if (k0 + u * NW < nfull) count_pair(v[u].x, v[u].y, k0 + u * NW, false);
    }
    if (nfull < nch && wave == NW - 1) { /* the partial last chunk, element by element */
      const int64_t e = gb + ((int64_t)nfull << 7) + 2 * lane;
      count_pair(e < stop ? vals[e] : 0.0, e + 1 < stop ? vals[e + 1] : 0.0, nfull, true);
    }
  }
  __syncthreads();
  for (int r = threadIdx.x; r < nrows; r += NT) {
    const uint32_t c = cnt[r];
    const int f0 = c & 255, f1 = (c >> 8) & 255, f2 = (c >> 16) & 255, f3 = c >> 24;
    dst[r] = lut[(int64_t)gd_pair_index(f0, f1, asize) * lut_nb + gd_pair_index(f2, f3, bsize)];
  }
}

/* Span staging by bit planes (the default wherever the planes fit in LDS).
 *
 * fetcount (cFisher.c:208-238) counts a row's "== 3" and "== -3" values.  Instead of
 * per-value LDS atomics into per-row counters (fw_stage_scores: ~20 lanes of a wave add
 * into one counter word, so every atomic is a ~10-way same-address conflict, and ~13
 * VALU per value), every wave turns 64 consecutive values into two ballots (one
 * v_cmp_eq_f64 each: 64 values per wave-instruction) that one lane stores.  The
 * planes are the span's values in element order, population A then B: bit e of plane
 * word w is value 64 w + e.  A row's counts are then four popcounts over its bit range
 * (one lane per row, v_alignbit + v_bcnt), followed by the score-table lookup.
 *
 * Loads are raw buffer loads against the population's span (num_records = the span's
 * bytes, so the partial last chunk reads zeros past the span, which compare false);
 * per lane one VGPR offset, the 8 chunks of a group at immediate offsets 512 u.  A
 * wave keeps 8 chunks of A and 8 of B in flight (32 VGPRs).
 * Returns false (nothing written) when the planes exceed cap_words u64 words. */
#ifndef FW_PL_U
#define FW_PL_U 8 /* chunks per population in flight per wave */
#endif
__device__ __forceinline__ void *gd_uniform_ptr(const double *p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return (void *)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
/* popcount of plane bits [b, b + s): the planes are uint4 per 64-value chunk
 * {"== 3" lo, hi, "== -3" lo, hi}; kind 0 / 2 selects the plane */
__device__ __forceinline__ int fw_bits(const uint32_t *p32, int b, int s, int kind) {
  int cnt = 0;
  for (int o = 0; o < s; o += 32) {
    const int e = b + o, w = min(s - o, 32);
    const int i0 = ((e >> 6) << 2) + kind + ((e >> 5) & 1);
    const int i1 = (e & 32) ? (((e >> 6) + 1) << 2) + kind : i0 + 1;
    const uint32_t bits = __builtin_amdgcn_alignbit(p32[i1], p32[i0], (uint32_t)(e & 31));
    cnt += __popc(w == 32 ? bits : (bits & ((1u << w) - 1u)));
  }
  return cnt;
}

__device__ bool fw_stage_planes(const gd_chrom_dev &d, int r0, int nrows, const double *avals, const double *bvals,
                                const double *lut, uint4 *planes, int cap_chunks, double *dst) {
  constexpr int NT = FW_WPB * FW_TPW, NW = NT / 64;
  const int asize = d.asize, bsize = d.bsize;
  const int nA = (nrows * asize + 63) >> 6, nB = (nrows * bsize + 63) >> 6, T = nA + nB;
  if (T + 1 > cap_chunks) return false; /* workgroup-uniform */
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  /* the span bases are workgroup-uniform, but the compiler cannot prove it (the
   * descriptor comes from a searched index): scalarise them, or every buffer load
   * becomes a waterfall loop */
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      gd_uniform_ptr(avals + d.a_off + (int64_t)r0 * asize), (short)0,
      __builtin_amdgcn_readfirstlane(nrows * asize * 8), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      gd_uniform_ptr(bvals + d.b_off + (int64_t)r0 * bsize), (short)0,
      __builtin_amdgcn_readfirstlane(nrows * bsize * 8), 0x00020000);
  /* wave w: chunks [a0, a1) of A and [b0, b1) of B */
  const int ca = (nA + NW - 1) / NW, cbk = (nB + NW - 1) / NW;
  const int a0 = min(wave * ca, nA), a1 = min(a0 + ca, nA), b0 = min(wave * cbk, nB), b1 = min(b0 + cbk, nB);
  const int ngrp = max((a1 - a0 + FW_PL_U - 1) / FW_PL_U, (b1 - b0 + FW_PL_U - 1) / FW_PL_U);
  for (int g = 0; g < ngrp; ++g) {
    const int ka = a0 + g * FW_PL_U, kb = b0 + g * FW_PL_U;
    const int va = (ka * 64 + lane) * 8, vb = (kb * 64 + lane) * 8;
    /* unconditional loads: past this wave's range they read the next wave's values
     * (ignored) or zeros past the span (num_records) */
    double xa[FW_PL_U], xb[FW_PL_U];
#pragma unroll
    for (int u = 0; u < FW_PL_U; ++u) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(ra, va + 512 * u, 0, 0);
      xa[u] = gd_f64_from(((uint64_t)v[1] << 32) | v[0]);
      const auto w = __builtin_amdgcn_raw_buffer_load_b64(rb, vb + 512 * u, 0, 0);
      xb[u] = gd_f64_from(((uint64_t)w[1] << 32) | w[0]);
    }
#pragma unroll
    for (int u = 0; u < FW_PL_U; ++u) {
      if (ka + u < a1) { /* wave-uniform */
        const uint64_t m3 = __builtin_amdgcn_ballot_w64(xa[u] == 3.0), mm3 = __builtin_amdgcn_ballot_w64(xa[u] == -3.0);
        if (lane == 0) planes[ka + u] = make_uint4((uint32_t)m3, (uint32_t)(m3 >> 32), (uint32_t)mm3, (uint32_t)(mm3 >> 32));
      }
      if (kb + u < b1) {
        const uint64_t m3 = __builtin_amdgcn_ballot_w64(xb[u] == 3.0), mm3 = __builtin_amdgcn_ballot_w64(xb[u] == -3.0);
        if (lane == 0)
          planes[nA + kb + u] = make_uint4((uint32_t)m3, (uint32_t)(m3 >> 32), (uint32_t)mm3, (uint32_t)(mm3 >> 32));
      }
    }
  }
  if (threadIdx.x == 0) planes[T] = make_uint4(0, 0, 0, 0); /* read by the last rows' alignbit */
  __syncthreads();
  const int lut_nb = (bsize + 1) * (bsize + 2) / 2;
  const uint32_t *p32 = reinterpret_cast<const uint32_t *>(planes);
  for (int r = threadIdx.x; r < nrows; r += NT) {
    const int ea = r * asize, eb = nA * 64 + r * bsize;
    const int f0 = fw_bits(p32, ea, asize, 0), f1 = fw_bits(p32, ea, asize, 2);
    const int f2 = fw_bits(p32, eb, bsize, 0), f3 = fw_bits(p32, eb, bsize, 2);
    dst[r] = lut[(int64_t)gd_pair_index(f0, f1, asize) * lut_nb + gd_pair_index(f2, f3, bsize)];
  }
  return true;
}

/* one compare-exchange step of the lane-group bitonic sort: every register r meets
 * the partner lane's register (MIRROR ? 7 - r : r); the upper lane keeps the larger */
template <int CTRL, bool MIRROR>
__device__ __forceinline__ void fw_cross(double (&v)[8], bool upper) {
  double p[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) p[r] = dpp_f64_full<CTRL>(v[MIRROR ? 7 - r : r]);
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = ((v[r] > p[r]) == upper) ? v[r] : p[r];
}

/* in-lane half-cleaners (register distances 4, 2, 1): a bitonic 8 -> descending */
__device__ __forceinline__ void fw_clean8(double (&v)[8]) {
#define FW_CX2(a, b)                       \
  do {                                     \
    const double hi_ = fw_max(v[a], v[b]); \
    v[b] = fw_min(v[a], v[b]);             \
    v[a] = hi_;                            \
  } while (0)
  FW_CX2(0, 4); FW_CX2(1, 5); FW_CX2(2, 6); FW_CX2(3, 7);
  FW_CX2(0, 2); FW_CX2(1, 3); FW_CX2(4, 6); FW_CX2(5, 7);
  FW_CX2(0, 1); FW_CX2(2, 3); FW_CX2(4, 5); FW_CX2(6, 7);
#undef FW_CX2
}

/* register-allocation target: 7 waves per SIMD (the LDS limit of 7 workgroups per CU); left
 * to itself the allocator takes 76 VGPRs (6 waves) for the FW_LCG_MAD step, and 7 waves ran
 * 0.7-1 % faster (C2: 2.365-2.380 against 2.383-2.385 ms/step; FW_LCG_MAD=0: 2.397-2.412) */
#ifndef FW_WAVES_PER_SIMD
#define FW_WAVES_PER_SIMD 7
#endif
#define FW_WPE __attribute__((amdgpu_waves_per_eu(FW_WAVES_PER_SIMD, 8)))
__global__ void __launch_bounds__(FW_WPB *FW_TPW) FW_WPE
    k_fet_window_fast(const gd_chrom_dev *ch, int nchrom, const int32_t *blk_off, int blk_base,
                      const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b, const double *snp_score,
                      const double *avals, const double *bvals, const uint64_t *binom, const int *lut_hdr,
                      const double *lut, int fused, double perc, double *scores, double *stddev,
                      const unsigned *flags, int32_t *slow_list, unsigned *slow_count) {
  __shared__ double sh_span[FW_SPAN];
  /* the row counters of the span staging (fused mode) share LDS with the ranked top
   * scores and the replicate rank pairs, which are written only after it */
  static_assert(FW_TPW * FW_RPT + FW_HALF == GD_NREP, "8 lanes x 12 whole + 4 halved replicates");
  __shared__ union {
    struct {
      double top[FW_WPB][FW_KTOP];
      uint16_t rix[FW_WPB][GD_NREP]; /* per replicate: rank pair read (rix_pack) */
    } b;
    uint32_t cnt[FW_SPAN]; /* per span row: majA | minA << 8 | majB << 16 | minB << 24 */
  } sh_u; /* fw_stage_planes also takes the whole union for its bit planes */
  double(&sh_top)[FW_WPB][FW_KTOP] = sh_u.b.top;
  uint16_t(&sh_rix)[FW_WPB][GD_NREP] = sh_u.b.rix;
  __shared__ int64_t sh_row[FW_WPB]; /* snp_score index of the window's first row; -1: not fast */
  __shared__ int sh_n[FW_WPB], sh_key[FW_WPB], sh_bad[FW_WPB], sh_slot[FW_WPB], sh_nrej[FW_WPB];
  __shared__ int sh_rej[FW_WPB][FW_MAXREJ];
  __shared__ unsigned long long sh_lo, sh_hi;

  if (*flags & (GD_FLAG_UNSORTED_A | GD_FLAG_UNSORTED_B | GD_FLAG_BAD_SIZE)) return;
  FW_PROF_INIT;
  const int tid = threadIdx.x;
  const int b = blk_base + blockIdx.x;
  /* workgroups never straddle chromosomes: blk_off[c] = first workgroup of chromosome c */
  int cb = 0;
  {
    int lo = 0, hi = nchrom - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (blk_off[mid] <= b)
        lo = mid;
      else
        hi = mid - 1;
    }
    cb = lo;
  }
  const gd_chrom_dev &d = ch[cb];
  const int64_t g0 = d.w_base + (int64_t)(b - blk_off[cb]) * FW_WPB;
  const int64_t wtotal = d.w_base + d.wend; /* end of this chromosome's windows */

  /* ---- A1. window extents (one lane per window), the staged row span, lane-group order ---- */
  if (tid == 0) {
    sh_lo = ~0ull;
    sh_hi = 0;
  }
  __syncthreads();
  if (tid < FW_WPB) {
    const int64_t g = g0 + tid;
    int64_t row = -1;
    int n = 0;
    if (g < wtotal) {
      const int lo = lo_a[g], hi = hi_a[g], lb = lo_b[g];
      n = (hi - lo) / d.asize;
      const bool aligned = n > 0 && (lo % d.asize == 0) && (lb % d.bsize == 0) && (lo / d.asize == lb / d.bsize) &&
                           (lo / d.asize + n <= d.nrows);
      const int m = n - gd_perc_index(n > 0 ? n : 1, perc);
      if (aligned && n >= 2 && n <= FW_NFAST && m <= 8) row = d.a_off + lo / d.asize;
    }
    if (row >= 0) atomicMin(&sh_lo, (unsigned long long)row);
    sh_row[tid] = row;
    sh_n[tid] = n;
    sh_bad[tid] = 0;
  }
  __syncthreads();
  if (tid < FW_WPB) {
    /* rows grow with the window index: windows past FW_SPAN staged rows go to the general path */
    const int64_t row = sh_row[tid];
    const int n = sh_n[tid];
    bool fast = row >= 0 && row + n - (int64_t)sh_lo <= FW_SPAN;
    if (fast) atomicMax(&sh_hi, (unsigned long long)(row + n));
    if (!fast) sh_row[tid] = -1;
    sh_key[tid] = fast ? ((n - gd_perc_index(n, perc)) << 12) + n : -1;
    if (!fast && n > 0 && g0 + tid < wtotal) slow_list[atomicAdd(slow_count, 1u)] = (int32_t)(g0 + tid);
  }
  __syncthreads();
  /* lane groups take windows in order of (m, n), non-fast (idle) windows first: the
   * windows sharing a wave need the same number of order statistics and run draw
   * loops of similar length */
  if (tid < FW_WPB) {
    const int key = sh_key[tid];
    int rank = 0;
    for (int j = 0; j < FW_WPB; ++j) {
      const int kj = sh_key[j];
      rank += (kj < key) || (kj == key && j < tid);
    }
    sh_slot[rank] = tid;
  }
  const int64_t span0 = (int64_t)sh_lo;
  const int spanlen = sh_hi > sh_lo ? (int)(sh_hi - sh_lo) : 0;
#ifdef GD_FET_NOSTAGE
  if (true) { /* diagnostics: span without scores (cost of everything else) */
    for (int i = tid; i < spanlen; i += FW_WPB * FW_TPW) sh_span[i] = (double)(i % 7);
  } else
#endif
  if (spanlen > 0 && fused && gd_lut_holds(lut_hdr, d.asize, d.bsize, binom)) {
    /* fused: the span rows' -log10 p from the genotype values (fetcount + the score
     * table, as k_snp_fet) -- the values are read here, once per workgroup */
#ifndef GD_FET_ATOMIC_STAGE
    if (!fw_stage_planes(d, (int)(span0 - d.a_off), spanlen, avals, bvals, lut, reinterpret_cast<uint4 *>(&sh_u),
                         (int)(sizeof(sh_u) / sizeof(uint4)), sh_span))
#endif
      fw_stage_scores(d, (int)(span0 - d.a_off), spanlen, avals, bvals, lut, sh_u.cnt, sh_span);
  } else {
    /* k_snp_fet scored the rows (unfused mode, or sizes the table does not hold) */
    for (int i = tid; i < spanlen; i += FW_WPB * FW_TPW) sh_span[i] = snp_score[span0 + i];
  }
  __syncthreads();

  FW_PROF(0);
  const int wl = sh_slot[tid / FW_TPW], q = tid % FW_TPW;
  const int64_t g = g0 + wl;
  const bool fast = sh_row[wl] >= 0;
  const int n = sh_n[wl];
  const int ktop = n < FW_KTOP ? n : FW_KTOP;
  const int base = n - ktop;
  const int idx = gd_perc_index(n > 0 ? n : 1, perc);
  const int m = n - idx;

  /* ---- A2. the window's top-KTOP scores in ascending order (sh_top[wl][rank - base]) ---- */
#ifdef GD_FET_NORANK
  if (false) { /* diagnostics: ranking cost */
#else
  if (fast) {
#endif
    const double *S = sh_span + (sh_row[wl] - span0);
    int nan = 0;
    if (n <= FW_TPW * 8) {
      /* each lane sorts its <= 8 scores (S[q], S[q+8], ...) descending in registers
       * (padding -inf), then the 8 lanes merge their runs */
      double v[8];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = q + FW_TPW * u;
        v[u] = (i < n) ? S[i] : -__builtin_inf();
        cnt += (i < n);
        nan |= (i < n) && (v[u] != v[u]);
      }
      /* Batcher odd-even merge sort network for 8 keys, descending */
#define FW_CX(a, b)                         \
  do {                                      \
    const double hi_ = fw_max(v[a], v[b]);  \
    v[b] = fw_min(v[a], v[b]);              \
    v[a] = hi_;                             \
  } while (0)
      FW_CX(0, 1); FW_CX(2, 3); FW_CX(4, 5); FW_CX(6, 7);
      FW_CX(0, 2); FW_CX(1, 3); FW_CX(4, 6); FW_CX(5, 7);
      FW_CX(1, 2); FW_CX(5, 6);
      FW_CX(0, 4); FW_CX(1, 5); FW_CX(2, 6); FW_CX(3, 7);
      FW_CX(2, 4); FW_CX(3, 5);
      FW_CX(1, 2); FW_CX(3, 4); FW_CX(5, 6);
#undef FW_CX
      /* bitonic merges across the 8 lanes (element e = 8q + r, descending): blocks of
       * 8 -> 16 -> 32 -> 64.  Each merge starts with a mirror step (lane q against the
       * block's mirror lane, register r against 7 - r), then half-cleaners at lane
       * distances 2, 1 (DPP) and register distances 4, 2, 1 */
      fw_cross<0xB1, true>(v, (q & 1) == 0);  /* 16: mirror in lane pairs */
      fw_clean8(v);
      fw_cross<0x1B, true>(v, (q & 2) == 0);  /* 32: mirror in quads */
      fw_cross<0xB1, false>(v, (q & 1) == 0); /*     lane distance 1 */
      fw_clean8(v);
      fw_cross<0x141, true>(v, (q & 4) == 0); /* 64: mirror in the 8 lanes */
      fw_cross<0x4E, false>(v, (q & 2) == 0); /*     lane distance 2 */
      fw_cross<0xB1, false>(v, (q & 1) == 0); /*     lane distance 1 */
      fw_clean8(v);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = FW_TPW * q + r; /* ascending rank n - 1 - e */
        if (e < ktop) sh_top[wl][ktop - 1 - e] = v[r];
      }
      (void)cnt;
    } else {
      /* 64 < n <= NFAST: rank by counting (ties by position) */
      for (int i = q; i < n; i += FW_TPW) {
        const double val = S[i];
        nan |= (val != val);
        int rank = 0;
        for (int j = 0; j < i; ++j) rank += (S[j] <= val);
        for (int j = i + 1; j < n; ++j) rank += (S[j] < val);
        if (rank >= base) sh_top[wl][rank - base] = val;
      }
    }
    if (nan) sh_bad[wl] = FW_BAD_GENERAL;
  }
  __syncthreads();

  FW_PROF(1);
  /* ---- B. bootstrap replicates: lane q runs replicates [12q, 12q+12) and half of 96 + q/2 ---- */
  /* wave-uniform loop shape: the largest m (order statistics tracked) and the
   * smallest / largest n and half length among this wave's bootstrapped windows */
  const bool boot = fast && sh_bad[wl] == 0;
  const int hlen = fw_half_len(q, n);
  int mmax = boot ? m : 0, mmin = boot ? m : 1 << 30, nmin = boot ? n : 1 << 30, nmax = boot ? n : 0;
  int hmin = boot ? hlen : 1 << 30, hmax = boot ? hlen : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mmax = max(mmax, __shfl_xor(mmax, o));
    mmin = min(mmin, __shfl_xor(mmin, o));
    nmin = min(nmin, __shfl_xor(nmin, o));
    nmax = max(nmax, __shfl_xor(nmax, o));
    hmin = min(hmin, __shfl_xor(hmin, o));
    hmax = max(hmax, __shfl_xor(hmax, o));
  }
  mmax = __builtin_amdgcn_readfirstlane(mmax);
  const int muni = __builtin_amdgcn_readfirstlane(mmin) == mmax ? mmax : 0;
  const int nlo8 = __builtin_amdgcn_readfirstlane(nmin) & ~7, nhi = __builtin_amdgcn_readfirstlane(nmax);
  const int hlo8 = __builtin_amdgcn_readfirstlane(hmin) & ~7, hhi = __builtin_amdgcn_readfirstlane(hmax);
  const int r0 = q * FW_RPT, hrep = FW_TPW * FW_RPT + (q >> 1);
  const bool hstore = (q & 1) == 0;
  const double delta = gd_perc_delta(n > 0 ? n : 1, perc, idx);
  const int nt = (n > 0 && n <= FW_NFAST) ? n : 1;
  const uint32_t limit = g_ntab_limit[nt];
  uint64_t x0 = 0;
  if (fast) x0 = gd_window_state(d.seed, GD_STREAM_FET, g - d.w_base + d.w_first);
  uint16_t *rix = sh_rix[wl] + r0;
#ifndef GD_FET_NODRAW /* diagnostics: setup cost only */
  if (boot) {
    const gd_affine jump = {g_ntab_jmul[nt][q], g_ntab_jadd[nt][q]};
    const gd_affine hjump = {g_ntab_hmul[nt][q], g_ntab_hadd[nt][q]};
    const uint64_t x = gd_affine_apply(jump, x0), xh = gd_affine_apply(hjump, x0), M = g_ntab_M[nt];
    uint32_t ymax = 0, wkey = ~0u;
#define FW_BOOT(MT, MU)                                                                                          \
  boot_lane<MT, MU>(x << 16, xh << 16, n, nlo8, nhi, hlen, hlo8, hhi, M, m, base, rix, sh_rix[wl] + hrep, hstore, \
                    ymax, wkey)
    if (mmax <= 4) {
      if (muni == 4)
        FW_BOOT(4, 4);
      else if (muni == 3)
        FW_BOOT(4, 3);
      else
        FW_BOOT(4, 0);
    } else if (mmax == 5) {
      if (muni == 5)
        FW_BOOT(5, 5);
      else
        FW_BOOT(5, 0);
    } else {
      FW_BOOT(8, 0);
    }
#undef FW_BOOT
#if FW_KEY16
    if (fw_key16_index(wkey, 2u * (uint32_t)n) < base) atomicOr(&sh_bad[wl], FW_BAD_GENERAL);
#else
    if (fw_key_index(wkey, 2u * (uint32_t)n) < base) atomicOr(&sh_bad[wl], FW_BAD_GENERAL);
#endif
    if ((ymax >> 1) > limit) atomicOr(&sh_bad[wl], FW_BAD_REJECT);
  }
#else
  for (int k = 0; k < FW_RPT; ++k) rix[k] = 0;
  if (hstore) sh_rix[wl][hrep] = 0;
#endif
  __syncthreads();

  FW_PROF(2);
  /* ---- B'. windows whose stream rejected a draw (p ~ n*5000/2^31 per window):
   * lane q locates the rejected positions of its pass-1 ranges [12qn, 12qn + 12n) and
   * its half replicate's, the lanes then restart each range at its corrected position
   * P = start + #(rejections before P) and redraw with the rejection loop.  Taken by
   * ~1 in 300 workgroups. */
  if (fast && sh_bad[wl] == FW_BAD_REJECT && q == 0) sh_nrej[wl] = 0;
  __syncthreads();
  const int64_t hs = fw_half_start(q, n);
  if (fast && sh_bad[wl] == FW_BAD_REJECT) {
    for (int part = 0; part < 2; ++part) {
      const int64_t p0 = part ? hs : (int64_t)r0 * n, len = part ? hlen : (int64_t)FW_RPT * n;
      uint64_t y = gd_affine_apply(gd_lcg_jump((uint64_t)p0), x0) << 16;
      for (int64_t t = 0; t < len; ++t) {
        y = y * GD_LCG_A + FW_C16;
        if (((uint32_t)(y >> 32) >> 1) > limit) {
          const int k = atomicAdd(&sh_nrej[wl], 1);
          if (k < FW_MAXREJ) sh_rej[wl][k] = (int)(p0 + t);
        }
      }
    }
  }
  __syncthreads();
  if (fast && sh_bad[wl] == FW_BAD_REJECT) {
    const int nrej = sh_nrej[wl];
    if (nrej > FW_MAXREJ) {
      if (q == 0) sh_bad[wl] |= FW_BAD_GENERAL;
    } else {
      /* fixed points: P = start + #(rejected positions < P); all such positions lie in [0, 100n) */
      int64_t P[2];
      for (int part = 0; part < 2; ++part) {
        const int64_t s0 = part ? hs : (int64_t)r0 * n;
        int64_t c = 0;
        for (;;) {
          int64_t cnt = 0;
          for (int k = 0; k < nrej; ++k) cnt += (sh_rej[wl][k] < s0 + c);
          if (cnt == c) break;
          c = cnt;
        }
        P[part] = s0 + c;
      }
      int worst = n;
      const gd_randint rd = gd_randint_make((uint32_t)n);
      uint64_t y = gd_affine_apply(gd_lcg_jump((uint64_t)P[0]), x0) << 16;
      int K[8];
      for (int k = 0; k < FW_RPT; ++k) {
        draw_rep_rejecting(y, n, rd, K);
        rix[k] = pick_rix_idx(K, m, base, worst);
      }
      y = gd_affine_apply(gd_lcg_jump((uint64_t)P[1]), x0) << 16;
      draw_rep_rejecting(y, hlen, rd, K);
      int Pk[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) Pk[i] = __builtin_amdgcn_update_dpp(0, K[i], 0xB1, 0xF, 0xF, false);
#pragma unroll
      for (int i = 0; i < 8; ++i) top_insert<8>(K, Pk[i]);
      const uint16_t w = pick_rix_idx(K, m, base, worst);
      if (hstore) sh_rix[wl][hrep] = w;
      if (worst < base) atomicOr(&sh_bad[wl], FW_BAD_GENERAL);
    }
  }
  __syncthreads();

  FW_PROF(3);
  /* ---- C. window score + population std of the 100 replicates (std, cFisher.c:492-518):
   * the sums run over i = 99 .. 0 exactly as the reference's loop: replicates 99 .. 96
   * (held by lanes 6, 4, 2, 0) gathered into lane 7, then one chain that walks down the
   * window's 8 lanes (lane q holds replicates 12q .. 12q + 11), handed from lane to lane
   * with a DPP row shift */
  const bool live = fast && !(sh_bad[wl] & FW_BAD_GENERAL);
  double rep[FW_RPT]; /* this lane's replicates r0 .. r0 + 11, rebuilt from their rank pairs */
#pragma unroll
  for (int k = 0; k < FW_RPT; ++k) {
    rep[k] = 0.0;
    if (live) {
      const unsigned w = rix[k];
      rep[k] = gd_perc_mix(delta, sh_top[wl][w & 255u], sh_top[wl][w >> 8]);
    }
  }
  double rh = 0.0; /* replicate 96 + q/2 (meaningful in even lanes) */
  if (live && hstore) {
    const unsigned w = sh_rix[wl][hrep];
    rh = gd_perc_mix(delta, sh_top[wl][w & 255u], sh_top[wl][w >> 8]);
  }
  const int gl = (int)(threadIdx.x & ~7u); /* the window's lane 0 */
  double h99 = __shfl(rh, gl + 6), h98 = __shfl(rh, gl + 4), h97 = __shfl(rh, gl + 2), h96 = __shfl(rh, gl);
  double sum = (live && q == FW_TPW - 1) ? ((h99 + h98) + h97) + h96 : 0.0;
#pragma unroll
  for (int step = FW_TPW - 1; step >= 0; --step) {
    if (live && q == step) {
#pragma unroll
      for (int k = FW_RPT - 1; k >= 0; --k) sum += rep[k];
    }
    if (step > 0) sum = dpp_f64<0x101>(sum); /* row_shl:1: lane l takes lane l+1's partial */
  }
  const double mu = __shfl(sum, gl) / GD_NREP;
  /* the squared deviations off the chain, all lanes at once (no FMA: the same two
   * roundings as the reference's (x - m) * (x - m)); the chain only adds */
#pragma unroll
  for (int k = 0; k < FW_RPT; ++k) {
    const double dd = rep[k] - mu;
    rep[k] = dd * dd;
  }
  {
    const double d99 = h99 - mu, d98 = h98 - mu, d97 = h97 - mu, d96 = h96 - mu;
    h99 = d99 * d99;
    h98 = d98 * d98;
    h97 = d97 * d97;
    h96 = d96 * d96;
  }
  double ss = (live && q == FW_TPW - 1) ? ((h99 + h98) + h97) + h96 : 0.0;
#pragma unroll
  for (int step = FW_TPW - 1; step >= 0; --step) {
    if (live && q == step) {
#pragma unroll
      for (int k = FW_RPT - 1; k >= 0; --k) ss += rep[k];
    }
    if (step > 0) ss = dpp_f64<0x101>(ss);
  }
  if (q == 0 && fast) {
    if (sh_bad[wl] & FW_BAD_GENERAL) {
      slow_list[atomicAdd(slow_count, 1u)] = (int32_t)g;
    } else {
      const int widx1 = (idx + 1 < n) ? idx + 1 : idx;
      const double ws = gd_perc_mix(delta, sh_top[wl][idx - base], sh_top[wl][widx1 - base]);
      const int64_t w = g - d.w_base;
      scores[d.w_out + w] = ws;
      stddev[d.w_out + w] = sqrt(ss / GD_NREP);
    }
  }
  FW_PROF(4);
}

/* GD_FORCE_GENERAL=1: every window takes the literal path (self-consistency checks) */
__global__ void k_all_windows(int32_t *list, unsigned *count, int64_t wtotal) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < wtotal) list[i] = (int32_t)i;
  if (i == 0) *count = (unsigned)wtotal;
}

int gd_fet_fast_windows_per_block() { return FW_WPB; }

/* per-n draw constants, once per device context */
int gd_fet_fast_init(hipStream_t s) {
  hipLaunchKernelGGL(k_fet_ntab_build, dim3((FW_NFAST + 64) / 64), dim3(64), 0, s);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

/* GD_FORCE_GENERAL=1: fills the slow-path list (zeroed with the scan's flags) with every
 * window and tells the caller to skip the fast kernels. */
int gd_fet_window_prepare(int64_t wtotal, int32_t *slow_list, unsigned *slow_count, hipStream_t s,
                          bool *force_general) {
  const char *force = getenv("GD_FORCE_GENERAL");
  *force_general = force && force[0] == '1';
  if (*force_general)
    hipLaunchKernelGGL(k_all_windows, dim3((unsigned)((wtotal + 255) / 256)), dim3(256), 0, s, slow_list,
                       slow_count, wtotal);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}


/* workgroups [blk_begin, blk_begin + blk_count) of the chromosome-aligned grid */
/* fused: the span scores come from avals/bvals and the score table (snp_score is then
 * read only for chromosomes whose sizes the table does not hold) */
int gd_fet_window_fast_launch(const gd_chrom_dev *ch, int nchrom, const int32_t *blk_off, int blk_begin,
                              int blk_count, const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b,
                              const double *snp_score, const double *avals, const double *bvals,
                              const uint64_t *binom, const int *lut_hdr, const double *lut, int fused, double perc,
                              double *scores, double *stddev, unsigned *flags, int32_t *slow_list,
                              unsigned *slow_count, hipStream_t s) {
  if (blk_count <= 0) return GD_OK;
#ifdef GD_FET_PROFILE
  {
    static int calls = 0;
    unsigned long long h[8];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fet_prof), sizeof h);
    if (++calls % 8 == 0)
      fprintf(stderr, "fet-prof cycles: A1 %llu A2 %llu B %llu Bp %llu C %llu\n", h[0], h[1], h[2], h[3], h[4]);
  }
#endif
  hipLaunchKernelGGL(k_fet_window_fast, dim3((unsigned)blk_count), dim3(FW_WPB * FW_TPW), 0, s, ch, nchrom,
                     blk_off, blk_begin, lo_a, hi_a, lo_b, snp_score, avals, bvals, binom, lut_hdr, lut, fused, perc,
                     scores, stddev, flags, slow_list, slow_count);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

