/*
 * gd_fet_rows.h -- per-SNP-row pieces of the FET scan shared by the pass kernels
 * (gd_fet_kernels.hip) and the fused window kernel (gd_fet_fast.hip): the Zar
 * two-tailed test on a 2x2 table (fet, cFisher.c:405-455, with fet_p / binomial,
 * cFisher.c:245-284, 473-483), fetcount's exact double compares
 * (cFisher.c:208-238), and popcounts over ballot masks of "== 3" / "== -3".
 */
#pragma once
#include "gd_common.h"

namespace {

__device__ __forceinline__ uint64_t binom_at(const uint64_t *tab, int n, int k) {
  if (n >= 0 && k >= 0 && k <= n && n <= GD_BINOM_NMAX) return tab[gd_binom_index(n, k)];
  return gd_binomial_ref((uint64_t)(int64_t)n, (uint64_t)(int64_t)k);
}

/* binomial lookups go through a kernel-local table pointer */
struct BinomTab {
  const uint64_t *t;
  __device__ __forceinline__ uint64_t operator()(int n, int k) const { return binom_at(t, n, k); }
};

/* the table buffer's mode word (reference / exact, gd_common.h) */
__device__ __forceinline__ int fet_mode(const uint64_t *tab) { return (int)tab[GD_FET_MODE_WORD]; }

/* the score table (hdr = {asize, bsize, valid, mode}) holds these sizes in this mode */
__device__ __forceinline__ bool gd_lut_holds(const int *hdr, int asize, int bsize, const uint64_t *binom) {
  return hdr[2] == 1 && hdr[0] == asize && hdr[1] == bsize && hdr[3] == fet_mode(binom);
}

__device__ double fet_p_two_tailed(int a, int b, int c, int d, const uint64_t *tab) {
  BinomTab B{tab};
  const bool exact = fet_mode(tab) != 0;
  const double *lfh = reinterpret_cast<const double *>(tab + GD_FET_LF_OFF), *lfl = lfh + (GD_BINOM_NMAX + 1);
  auto table_p = [&](const int *g) {
    return exact ? gd_fet_table_p_exact(lfh, lfl, g[0], g[1], g[2], g[3]) : GD_FET_TABLE_P(B, g[0], g[1], g[2], g[3]);
  };
  const int tie = (a + b == c + d) || (a + c == b + d);
  int f[4] = {a, b, c, d};
  gd_table_min_to_a(f);
  const double p0 = table_p(f);
  double tot = p0, step = p0;
  while (f[0] > 0) {
    f[1]++;
    f[2]++;
    step = (1.0 * f[0] * f[3]) / (double)(f[1] * f[2]) * step;
    tot += step;
    f[0]--;
    f[3]--;
  }
  if (tie) {
    tot = 2 * tot;
  } else {
    gd_table_opposite_extreme(f);
    gd_table_min_to_a(f);
    double far = table_p(f);
    while (far < (exact ? p0 * (1.0 - GD_FET_EXACT_TIE) : p0)) {
      tot += far;
      if (f[1] == 0 || f[2] == 0) break;
      f[0]++;
      f[3]++;
      far = (1.0 * f[1] * f[2]) / (double)(f[0] * f[3]) * far;
      f[1]--;
      f[2]--;
    }
  }
  if (tot > 1) tot = 1;
  return tot;
}

/* fetcount(): exact double compares against 3 and -3 (cFisher.c:208-238) */
__device__ __forceinline__ double snp_score_raw(const double *a, int asize, const double *b, int bsize,
                                                const uint64_t *tab) {
  int f0 = 0, f1 = 0, f2 = 0, f3 = 0;
  for (int k = 0; k < asize; ++k) {
    const double v = a[k];
    f0 += (v == 3.0);
    f1 += (v == -3.0);
  }
  for (int k = 0; k < bsize; ++k) {
    const double v = b[k];
    f2 += (v == 3.0);
    f3 += (v == -3.0);
  }
  return gd_fet_score_from_p(fet_p_two_tailed(f0, f1, f2, f3, tab));
}

/* the same score through the (asize, bsize) score table (lut_hdr checked by the caller) */
__device__ __forceinline__ double snp_score_table(const double *a, int asize, const double *b, int bsize,
                                                  const double *lut) {
  int f0 = 0, f1 = 0, f2 = 0, f3 = 0;
  for (int k = 0; k < asize; ++k) {
    f0 += (a[k] == 3.0);
    f1 += (a[k] == -3.0);
  }
  for (int k = 0; k < bsize; ++k) {
    f2 += (b[k] == 3.0);
    f3 += (b[k] == -3.0);
  }
  return lut[(int64_t)gd_pair_index(f0, f1, asize) * ((bsize + 1) * (bsize + 2) / 2) + gd_pair_index(f2, f3, bsize)];
}

}  // namespace

/* ------------------------------------------------------------------------ */
/* Row counts from ballot masks.  A wave streams a tile's genotype values with */
/* coalesced 16-byte loads (two values per lane, 128 per wave-instruction) and  */
/* turns them into ballot bit masks of "== 3" and "== -3" (even / odd element   */
/* of each lane separately); a row's four counts are popcounts over its element */
/* range.                                                                       */
/* ------------------------------------------------------------------------ */
#define SF_MAXCH 168 /* 128-element chunks per population per tile */

namespace {

__device__ __forceinline__ uint64_t lane_range(int a, int b) {
  const uint64_t hi = (b >= 64) ? ~0ull : ((1ull << b) - 1);
  const uint64_t lo = (a >= 64) ? ~0ull : ((1ull << a) - 1);
  return hi & ~lo;
}

/* bits set among tile-relative elements [s, e) of one (pop, kind) mask set */
__device__ __forceinline__ int count_range(const uint64_t (*m)[2], int s, int e) {
  int cnt = 0;
  for (int k = s >> 7; k <= (e - 1) >> 7; ++k) {
    const int ls = max(s - (k << 7), 0), le = min(e - (k << 7), 128);
    cnt += __popcll(m[k][0] & lane_range((ls + 1) >> 1, (le + 1) >> 1)) +
           __popcll(m[k][1] & lane_range(ls >> 1, le >> 1));
  }
  return cnt;
}

}  // namespace

