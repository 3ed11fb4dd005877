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
 * The window's top-KTOP scores are ranked once into LDS.
 *
 * Parallel RNG.  nrand48 is x -> (a x + c) mod 2^48; lane q of a window starts
 * its replicates at stream position 13*q*n via an affine jump (gd_lcg_jump), so
 * the 8 lanes of a window reproduce the reference's single sequential stream.
 * A rejected draw (r > RAND_MAX - 2^31 mod n, probability ~n/2^31) would shift
 * every later draw: such a window is handed to the literal general path, as are
 * windows with NaN scores, n < 2, n > NFAST, m > 8, misaligned A/B rows, or a
 * replicate whose order statistic falls below the ranked top-KTOP.
 *
 * Layout: 256-thread workgroup = 32 consecutive windows x 8 lanes; lanes of a
 * window split its 100 replicates 13/13/.../9.  Windows are assigned to lane
 * groups in order of n, so the 8 windows of a wave run loops of similar length.
 * The SNP scores the 32 windows touch (a contiguous row span of one chromosome)
 * are staged in LDS once.  Per draw: 6 VALU for the LCG step, 4 for r mod n,
 * MT (4 or 8, chosen per workgroup) for the order statistics, 1/2 for the
 * rejection maximum.
 */
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_internal.h"

#define FW_WPB 32    /* windows per workgroup */
#define FW_TPW 8     /* lanes per window */
#define FW_RPT 13    /* replicates per lane (8*13 >= 100) */
#define FW_KTOP 32   /* ranked top scores kept per window */
#define FW_NFAST 256 /* largest window handled here */
#define FW_SPAN 2048 /* staged SNP rows per workgroup */

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

/* lane's replicates [r0, r1): stream already positioned at r0*n */
template <int MT>
__device__ __forceinline__ void boot_lane(uint64_t x, int n, const gd_randint &rd, int r0, int r1, int m, int base,
                                          double delta, const double *top, double *rep, uint32_t &rmax,
                                          int &worst) {
  for (int r = r0; r < r1; ++r) {
    int K[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) K[i] = -1;
    int j = n;
    for (; j >= 2; j -= 2) {
      x = gd_lcg_next(x);
      const uint32_t ra = gd_lcg_value(x);
      x = gd_lcg_next(x);
      const uint32_t rb = gd_lcg_value(x);
      rmax = max(rmax, max(ra, rb));
      top_insert<MT>(K, fmod_n(ra, rd.magic, rd.shift, rd.n));
      top_insert<MT>(K, fmod_n(rb, rd.magic, rd.shift, rd.n));
    }
    if (j) {
      x = gd_lcg_next(x);
      const uint32_t ra = gd_lcg_value(x);
      rmax = max(rmax, ra);
      top_insert<MT>(K, fmod_n(ra, rd.magic, rd.shift, rd.n));
    }
    int a = K[0], b = K[0];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (i == m - 1) a = K[i];
      if (i == m - 2) b = K[i];
    }
    worst = min(worst, a); /* a = t_{m-1} <= b = t_{m-2}: the lowest index read */
    rep[r] = gd_perc_mix(delta, top[max(a - base, 0)], top[max(b - base, 0)]);
  }
}

__device__ double std_reverse_lds(const double *a) {
  double sum = 0;
#pragma unroll 4
  for (int i = GD_NREP - 1; i >= 0; --i) sum += a[i];
  const double mu = sum / GD_NREP;
  double ss = 0;
#pragma unroll 4
  for (int i = GD_NREP - 1; i >= 0; --i) {
    const double dd = a[i] - mu;
    ss += dd * dd;
  }
  ss /= GD_NREP;
  return sqrt(ss);
}

}  // namespace

__global__ void __launch_bounds__(FW_WPB *FW_TPW)
    k_fet_window_fast(const gd_chrom_dev *ch, int nchrom, int64_t wtotal, const int32_t *lo_a,
                      const int32_t *hi_a, const int32_t *lo_b, const double *snp_score, double perc,
                      double *scores, double *stddev, const unsigned *flags, int32_t *slow_list,
                      unsigned *slow_count) {
  __shared__ double sh_span[FW_SPAN];
  __shared__ double sh_top[FW_WPB][FW_KTOP];
  __shared__ double sh_rep[FW_WPB][GD_NREP];
  __shared__ int64_t sh_row[FW_WPB]; /* snp_score index of the window's first row; -1: not fast */
  __shared__ int sh_n[FW_WPB], sh_c[FW_WPB], sh_bad[FW_WPB], sh_slot[FW_WPB];
  __shared__ int64_t sh_span0;
  __shared__ int sh_spanlen, sh_mmax;

  if (*flags & (GD_FLAG_UNSORTED_A | GD_FLAG_UNSORTED_B | GD_FLAG_BAD_SIZE)) return;
  const int tid = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * FW_WPB;

  /* ---- A1. window extents (one lane per window) ---- */
  if (tid < FW_WPB) {
    const int64_t g = g0 + tid;
    int64_t row = -1;
    int n = 0, c = 0;
    if (g < wtotal) {
      c = chrom_of_fast(ch, nchrom, g);
      const gd_chrom_dev &d = ch[c];
      const int lo = lo_a[g], hi = hi_a[g], lb = lo_b[g];
      n = (hi - lo) / d.asize;
      const bool aligned = n > 0 && (lo % d.asize == 0) && (lb % d.bsize == 0) && (lo / d.asize == lb / d.bsize) &&
                           (lo / d.asize + n <= d.nrows);
      const int m = n - gd_perc_index(n > 0 ? n : 1, perc);
      if (aligned && n >= 2 && n <= FW_NFAST && m <= 8) row = d.a_off + lo / d.asize;
    }
    sh_row[tid] = row;
    sh_n[tid] = n;
    sh_c[tid] = c;
    sh_bad[tid] = 0;
  }
  if (tid == 0) sh_mmax = 0;
  __syncthreads();
  if (tid == 0) {
    /* one chromosome's contiguous row span: that of the first fast window */
    int64_t s0 = -1, s1 = -1;
    int cref = -1;
    for (int i = 0; i < FW_WPB; ++i) {
      if (sh_row[i] < 0) continue;
      if (cref < 0) cref = sh_c[i];
      const int64_t r0 = sh_row[i], r1 = sh_row[i] + sh_n[i];
      const int64_t n0 = (s0 < 0 || r0 < s0) ? r0 : s0;
      const int64_t n1 = (r1 > s1) ? r1 : s1;
      if (sh_c[i] != cref || n1 - n0 > FW_SPAN) {
        sh_row[i] = -1; /* left to the general path */
        continue;
      }
      s0 = n0;
      s1 = n1;
    }
    sh_span0 = s0;
    sh_spanlen = (s0 >= 0) ? (int)(s1 - s0) : 0;
  }
  __syncthreads();
  /* lane groups take windows in order of n (non-fast windows first, they are idle) */
  if (tid < FW_WPB) {
    const int key = sh_row[tid] >= 0 ? sh_n[tid] : -1;
    int rank = 0;
    for (int j = 0; j < FW_WPB; ++j) {
      const int kj = sh_row[j] >= 0 ? sh_n[j] : -1;
      rank += (kj < key) || (kj == key && j < tid);
    }
    sh_slot[rank] = tid;
    if (sh_row[tid] < 0 && sh_n[tid] > 0 && g0 + tid < wtotal) slow_list[atomicAdd(slow_count, 1u)] = (int32_t)(g0 + tid);
  }
  const int64_t span0 = sh_span0;
  for (int i = tid; i < sh_spanlen; i += FW_WPB * FW_TPW) sh_span[i] = snp_score[span0 + i];
  __syncthreads();

  const int wl = sh_slot[tid / FW_TPW], q = tid % FW_TPW;
  const int64_t g = g0 + wl;
  const bool fast = sh_row[wl] >= 0;
  const int n = sh_n[wl];
  const int base = n > FW_KTOP ? n - FW_KTOP : 0;
  const int idx = gd_perc_index(n > 0 ? n : 1, perc);
  const int m = n - idx;

  /* ---- A2. rank the window's scores (ascending, ties by position) into the top-KTOP table ---- */
  if (fast) {
    const double *S = sh_span + (sh_row[wl] - span0);
    int nan = 0;
    for (int i = q; i < n; i += FW_TPW) {
      const double v = S[i];
      nan |= (v != v);
      int rank = 0;
      for (int j = 0; j < i; ++j) rank += (S[j] <= v);
      for (int j = i + 1; j < n; ++j) rank += (S[j] < v);
      if (rank >= base) sh_top[wl][rank - base] = v;
    }
    if (nan) sh_bad[wl] = 1;
    if (q == 0) atomicMax(&sh_mmax, m);
  }
  __syncthreads();

  /* ---- B. bootstrap replicates: lane q runs replicates [13q, 13q+13) ---- */
  const int mmax = sh_mmax;
  if (fast && sh_bad[wl] == 0) {
    const gd_chrom_dev &d = ch[sh_c[wl]];
    const double delta = gd_perc_delta(n, perc, idx);
    const gd_randint rd = gd_randint_make((uint32_t)n);
    const int r0 = q * FW_RPT;
    const int r1 = min(GD_NREP, r0 + FW_RPT);
    uint64_t x = gd_window_state(d.seed, GD_STREAM_FET, g - d.w_base);
    x = gd_affine_apply(gd_lcg_jump((uint64_t)r0 * (uint64_t)n), x);
    uint32_t rmax = 0;
    int worst = n;
    if (mmax <= 4)
      boot_lane<4>(x, n, rd, r0, r1, m, base, delta, sh_top[wl], sh_rep[wl], rmax, worst);
    else
      boot_lane<8>(x, n, rd, r0, r1, m, base, delta, sh_top[wl], sh_rep[wl], rmax, worst);
    if (rmax > rd.limit || worst < base) atomicOr(&sh_bad[wl], 1);
  }
  __syncthreads();

  /* ---- C. window score + population std of the 100 replicates ---- */
  if (fast && q == 0) {
    const gd_chrom_dev &d = ch[sh_c[wl]];
    if (sh_bad[wl]) {
      slow_list[atomicAdd(slow_count, 1u)] = (int32_t)g;
    } else {
      const double delta = gd_perc_delta(n, perc, idx);
      const int idx1 = (idx + 1 < n) ? idx + 1 : idx;
      const double ws = gd_perc_mix(delta, sh_top[wl][idx - base], sh_top[wl][idx1 - base]);
      const int64_t w = g - d.w_base;
      scores[d.w_out + w] = ws;
      stddev[d.w_out + w] = std_reverse_lds(sh_rep[wl]);
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
