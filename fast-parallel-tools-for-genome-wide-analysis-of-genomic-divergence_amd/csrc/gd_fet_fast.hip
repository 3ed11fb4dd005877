/*
 * gd_fet_fast.hip -- fast window path of the FET scan: window percentile and the
 * 100-replicate bootstrap stddev (cFisher.c:136-144, 547-597) without sorting.
 *
 * Why it is exact.  percentile() sorts the window's SNP scores S ascending and the
 * bootstrap draws indices into that SORTED array (Q6, cFisher.c:188,194,569).  The
 * sorted replicate therefore equals S evaluated at the sorted sampled indices, so
 * its idx-th and (idx+1)-th elements are S[t_{m-1}] and S[t_{m-2}], where t_0 >=
 * t_1 >= ... are the sampled indices in descending order and m = n - idx
 * (m ~ 3-4 at perc 0.95).  Each lane keeps the MTOP largest indices of its
 * replicate in registers (one v_med3 per slot per draw); no sort, no histogram.
 * The window's top-KTOP scores are ranked once into LDS.
 *
 * Parallel RNG.  nrand48 is x -> (a x + c) mod 2^48; lane q of a window starts
 * its replicates at stream position q*13*n via an affine jump (gd_lcg_jump), so
 * the 8 lanes of a window reproduce the reference's single sequential stream.
 * A rejected draw (r > RAND_MAX - 2^31 mod n, probability ~n/2^31) would shift
 * every later draw: such a window is handed to the literal general path, as are
 * windows with NaN scores, n > NFAST, m > MTOP, misaligned A/B rows, or a
 * replicate whose order statistic falls below the ranked top-KTOP.
 *
 * Layout: 256-thread workgroup = 32 consecutive windows x 8 lanes; lanes of a
 * window split its 100 replicates 13/13/.../9.  The SNP scores the 32 windows
 * touch (a contiguous row span of one chromosome) are staged in LDS once.
 */
#include <hip/hip_runtime.h>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_internal.h"

#define FW_WPB 32    /* windows per workgroup */
#define FW_TPW 8     /* lanes per window */
#define FW_RPT 13    /* replicates per lane (8*13 >= 100) */
#define FW_MTOP 8    /* order statistics tracked per replicate */
#define FW_KTOP 32   /* ranked top scores kept per window */
#define FW_NFAST 256 /* largest window handled here */
#define FW_SPAN 2048 /* staged SNP rows per workgroup */

#define FW_BAD 1

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

}  // namespace

__global__ void __launch_bounds__(FW_WPB *FW_TPW)
    k_fet_window_fast(const gd_chrom_dev *ch, int nchrom, int64_t wtotal, const int32_t *lo_a,
                      const int32_t *hi_a, const int32_t *lo_b, const double *snp_score, double perc,
                      double *scores, double *stddev, const unsigned *flags, int32_t *slow_list,
                      unsigned *slow_count) {
  __shared__ double sh_span[FW_SPAN];
  __shared__ double sh_top[FW_WPB][FW_KTOP];
  __shared__ double sh_rep[FW_WPB][GD_NREP];
  __shared__ int64_t sh_row[FW_WPB]; /* global snp_score index of the window's first row, -1 = not fast */
  __shared__ int sh_n[FW_WPB];
  __shared__ int sh_bad[FW_WPB];
  __shared__ int64_t sh_span0;
  __shared__ int sh_spanlen;

  if (*flags & (GD_FLAG_UNSORTED_A | GD_FLAG_UNSORTED_B | GD_FLAG_BAD_SIZE)) return;
  const int tid = threadIdx.x;
  const int wl = tid / FW_TPW, q = tid % FW_TPW;
  const int64_t g = (int64_t)blockIdx.x * FW_WPB + wl;
  const bool live = g < wtotal;

  /* ---- A. window extents; which windows stay on the fast path ---- */
  int c = 0, n = 0;
  int64_t w = 0;
  if (live) {
    c = chrom_of_fast(ch, nchrom, g);
    const gd_chrom_dev &d = ch[c];
    w = g - d.w_base;
    const int lo = lo_a[g], hi = hi_a[g], lb = lo_b[g];
    n = (hi - lo) / d.asize;
    if (q == 0) {
      int64_t row = -1;
      const bool aligned = n > 0 && (lo % d.asize == 0) && (lb % d.bsize == 0) && (lo / d.asize == lb / d.bsize) &&
                           (lo / d.asize + n <= d.nrows);
      const int m = n - gd_perc_index(n > 0 ? n : 1, perc);
      if (aligned && n <= FW_NFAST && m <= FW_MTOP) row = d.a_off + lo / d.asize;
      sh_row[wl] = row;
      sh_n[wl] = n;
      sh_bad[wl] = 0;
    }
  } else if (q == 0) {
    sh_row[wl] = -1;
    sh_n[wl] = 0;
    sh_bad[wl] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    /* one chromosome's contiguous row span: that of the first fast window */
    int64_t s0 = -1, s1 = -1;
    int cref = -1;
    for (int i = 0; i < FW_WPB; ++i) {
      if (sh_row[i] < 0) continue;
      const int64_t gi = (int64_t)blockIdx.x * FW_WPB + i;
      const int ci = chrom_of_fast(ch, nchrom, gi);
      if (cref < 0) cref = ci;
      const int64_t r0 = sh_row[i], r1 = sh_row[i] + sh_n[i];
      const int64_t n0 = (s0 < 0 || r0 < s0) ? r0 : s0;
      const int64_t n1 = (r1 > s1) ? r1 : s1;
      if (ci != cref || n1 - n0 > FW_SPAN) {
        sh_row[i] = -1; /* left to the general path below */
        continue;
      }
      s0 = n0;
      s1 = n1;
    }
    sh_span0 = s0;
    sh_spanlen = (s0 >= 0) ? (int)(s1 - s0) : 0;
  }
  __syncthreads();
  const int64_t span0 = sh_span0;
  for (int i = tid; i < sh_spanlen; i += FW_WPB * FW_TPW) sh_span[i] = snp_score[span0 + i];
  __syncthreads();

  const bool fast = live && sh_row[wl] >= 0;
  const int base = n > FW_KTOP ? n - FW_KTOP : 0;
  if (fast) {
    /* rank the window's scores (ascending, ties by position) into the top-KTOP table */
    const double *S = sh_span + (sh_row[wl] - span0);
    int nan = 0;
    for (int i = q; i < n; i += FW_TPW) {
      const double v = S[i];
      nan |= (v != v);
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        const double u = S[j];
        rank += (u < v) || (u == v && j < i);
      }
      if (rank >= base) sh_top[wl][rank - base] = v;
    }
    if (nan) sh_bad[wl] = FW_BAD;
  } else if (live && q == 0 && n > 0) {
    slow_list[atomicAdd(slow_count, 1u)] = (int32_t)g;
  }
  __syncthreads();

  /* ---- B. bootstrap replicates: lane q runs replicates [13q, 13q+13) ---- */
  if (fast && sh_bad[wl] == 0) {
    const gd_chrom_dev &d = ch[c];
    const int idx = gd_perc_index(n, perc);
    const double delta = gd_perc_delta(n, perc, idx);
    const int m = n - idx;
    const gd_randint rd = gd_randint_make((uint32_t)n);
    const int r0 = q * FW_RPT;
    const int r1 = min(GD_NREP, r0 + FW_RPT);
    uint64_t x = gd_window_state(d.seed, GD_STREAM_FET, w);
    x = gd_affine_apply(gd_lcg_jump((uint64_t)r0 * (uint64_t)n), x);
    uint32_t rmax = 0;
    int worst = n;
    for (int r = r0; r < r1; ++r) {
      int K[FW_MTOP];
#pragma unroll
      for (int i = 0; i < FW_MTOP; ++i) K[i] = -1;
      for (int j = 0; j < n; ++j) {
        x = gd_lcg_next(x);
        const uint32_t rr = gd_lcg_value(x);
        rmax = rmax > rr ? rmax : rr;
        const int v = (int)gd_randint_mod(&rd, rr);
#pragma unroll
        for (int i = FW_MTOP - 1; i > 0; --i) K[i] = med3i(K[i - 1], K[i], v);
        K[0] = max(K[0], v);
      }
      int a = K[0], b = K[0];
#pragma unroll
      for (int i = 0; i < FW_MTOP; ++i) {
        if (i == m - 1) a = K[i];
        if (i == m - 2) b = K[i];
      }
      if (m < 2) b = a;
      worst = min(worst, b < a ? b : a);
      sh_rep[wl][r] = gd_perc_mix(delta, sh_top[wl][max(a - base, 0)], sh_top[wl][max(b - base, 0)]);
    }
    if (rmax > rd.limit || worst < base) atomicOr(&sh_bad[wl], FW_BAD);
  }
  __syncthreads();

  /* ---- C. window score + population std of the 100 replicates ---- */
  if (fast && q == 0) {
    const gd_chrom_dev &d = ch[c];
    if (sh_bad[wl]) {
      slow_list[atomicAdd(slow_count, 1u)] = (int32_t)g;
    } else {
      const int idx = gd_perc_index(n, perc);
      const double delta = gd_perc_delta(n, perc, idx);
      const int idx1 = (idx + 1 < n) ? idx + 1 : idx;
      const double ws = gd_perc_mix(delta, sh_top[wl][idx - base], sh_top[wl][idx1 - base]);
      double sd;
      GD_STD_REVERSE(sd, sh_rep[wl], GD_NREP);
      scores[d.w_out + w] = ws;
      stddev[d.w_out + w] = sd;
    }
  }
}

__global__ void k_zero_count(unsigned *count) { *count = 0; }

/* GD_FORCE_GENERAL=1: every window takes the literal path (self-consistency checks) */
__global__ void k_all_windows(int32_t *list, unsigned *count, int64_t wtotal) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < wtotal) list[i] = (int32_t)i;
  if (i == 0) *count = (unsigned)wtotal;
}

int gd_fet_window_fast_launch(const gd_chrom_dev *ch, int nchrom, int64_t wtotal, const int32_t *lo_a,
                              const int32_t *hi_a, const int32_t *lo_b, const double *snp_score, double perc,
                              double *scores, double *stddev, unsigned *flags, int32_t *slow_list,
                              unsigned *slow_count, hipStream_t s) {
  const char *force = getenv("GD_FORCE_GENERAL");
  if (force && force[0] == '1') {
    hipLaunchKernelGGL(k_all_windows, dim3((unsigned)((wtotal + 255) / 256)), dim3(256), 0, s, slow_list,
                       slow_count, wtotal);
    return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
  }
  hipLaunchKernelGGL(k_zero_count, dim3(1), dim3(1), 0, s, slow_count);
  const unsigned blocks = (unsigned)((wtotal + FW_WPB - 1) / FW_WPB);
  hipLaunchKernelGGL(k_fet_window_fast, dim3(blocks), dim3(FW_WPB * FW_TPW), 0, s, ch, nchrom, wtotal, lo_a, hi_a,
                     lo_b, snp_score, perc, scores, stddev, flags, slow_list, slow_count);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}
