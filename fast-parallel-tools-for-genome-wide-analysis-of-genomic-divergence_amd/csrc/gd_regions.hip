/*
 * gd_regions.hip -- the step after the scan: turning a score track into divergent
 * regions, on the device.
 *
 *   FilterFisherScores.py:83-93    limit = cmedian(score) + qnorm * scoreatpercentile(stddev, perc)
 *   SignificantCSSRegions.py:102-123  Benjamini-Hochberg step-up p threshold
 *   SignificantCSSRegions.py:124-127  score of the num_top-th best window
 *   FilterFisherScores.py:97-114 / SignificantCSSRegions.py:129-150  select + merge into segments
 *
 * A "track" is the list of windows the tools' tabular file holds (windows with a
 * non-zero score, file order): value columns plus, for the merge, a sequence index
 * and the window start.  10M windows are 80 MB per column, so the whole track stays
 * in HBM: order statistics come from one 64-bit radix sort of order-preserving keys,
 * the BH scan is one pass over the sorted keys, the cmedian histogram is an LDS
 * histogram, and the merge is two stream compactions.  Host code here only does the
 * O(1000) arithmetic on the histogram and the scalar formulas.
 *
 * Ordering follows numpy: NaN sorts last (np.sort / np.argsort), -0.0 == +0.0.
 */
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "../../include/gdscan.h"

void gd_set_error(const char *msg);

#define RG_TRY(expr)                                                                                  \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess) {                                                                           \
      gd_set_error((std::string(#expr ": ") + hipGetErrorString(e_)).c_str());                        \
      return GD_ERR_HIP;                                                                              \
    }                                                                                                 \
  } while (0)

static int rg_fail(int code, const char *msg) {
  gd_set_error(msg);
  return code;
}

#define RG_CMEDIAN_BINS 1000 /* scipy.stats.cmedian(a, numbins=1000) */
#define RG_BLOCK 256

/* ------------------------------------------------------------- order keys */
/* monotone map double -> u64 under numpy's order: NaN above +inf, -0.0 == +0.0 */
__host__ __device__ static inline uint64_t okey(double x) {
  if (x != x) return ~0ull;
  if (x == 0.0) x = 0.0;
  uint64_t b;
  memcpy(&b, &x, 8);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
static inline double okey_value(uint64_t k) {
  if (k == ~0ull) return std::nan("");
  uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  double x;
  memcpy(&x, &b, 8);
  return x;
}

__global__ void k_rg_keys(const double *__restrict__ v, int64_t n, uint64_t *__restrict__ keys) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys[i] = okey(v[i]);
}

/* min / max keys and a non-finite flag (numpy.histogram refuses a non-finite range) */
__global__ void k_rg_minmax(const double *__restrict__ v, int64_t n, unsigned long long *mm) {
  uint64_t lo = ~0ull, hi = 0;
  unsigned bad = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double x = v[i];
    bad |= !isfinite(x);
    const uint64_t k = okey(x);
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
  }
  for (int o = 32; o; o >>= 1) {
    const uint64_t l2 = __shfl_xor(lo, o), h2 = __shfl_xor(hi, o);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
    bad |= __shfl_xor(bad, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], (unsigned long long)lo);
    atomicMax(&mm[1], (unsigned long long)hi);
    if (bad) atomicOr(&mm[2], 1ull);
  }
}

/* numpy.histogram's uniform-bin assignment (numpy/lib/_histograms_impl.py): estimate the
 * bin from the range, then correct by one against the linspace edges, so that bin i holds
 * edges[i] <= x < edges[i+1] (the last bin is closed). */
__global__ void k_rg_hist(const double *__restrict__ v, int64_t n, const double *__restrict__ edges,
                          unsigned long long *__restrict__ counts) {
  __shared__ unsigned h[RG_CMEDIAN_BINS];
  for (int b = threadIdx.x; b < RG_CMEDIAN_BINS; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const double first = edges[0], last = edges[RG_CMEDIAN_BINS];
  const double denom = last - first;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double x = v[i];
    int b = (int)(((x - first) / denom) * (double)RG_CMEDIAN_BINS);
    if (b >= RG_CMEDIAN_BINS) b = RG_CMEDIAN_BINS - 1;
    if (b < 0) b = 0;
    if (x < edges[b]) --b;
    if (b != RG_CMEDIAN_BINS - 1 && x >= edges[b + 1]) ++b;
    atomicAdd(&h[b], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < RG_CMEDIAN_BINS; b += blockDim.x)
    if (h[b]) atomicAdd(&counts[b], (unsigned long long)h[b]);
}

/* Benjamini-Hochberg (SignificantCSSRegions.py:104-114): the loop walks p from the
 * largest down with k = n, n-1, ... and stops at the first p <= k/n * FDR, i.e. at the
 * largest rank k (1-based, ascending) with sorted[k-1] <= (k/n) * FDR.  NaN never passes. */
__global__ void k_rg_bh(const uint64_t *__restrict__ sorted, int64_t n, double fdr, unsigned long long *best) {
  unsigned long long mine = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = sorted[i];
    if (k == ~0ull) continue;
    const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    const double p = __longlong_as_double((long long)b);
    if (p <= (double)(i + 1) / (double)n * fdr) mine = (unsigned long long)(i + 1);
  }
  for (int o = 32; o; o >>= 1) {
    const unsigned long long t = __shfl_xor(mine, o);
    mine = t > mine ? t : mine;
  }
  if ((threadIdx.x & 63) == 0 && mine) atomicMax(best, mine);
}

/* selection flags; a sequence index outside [0, nseq) is reported instead of read */
__global__ void k_rg_select_flags(const double *__restrict__ v, const int32_t *__restrict__ seq, int64_t n,
                                  int nseq, int cmp, double thr, uint8_t *__restrict__ f, int64_t *bad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double x = v[i];
    f[i] = cmp == GD_SELECT_GE ? (x >= thr) : (x <= thr);
    if ((unsigned)seq[i] >= (unsigned)nseq) *bad = 1;
  }
}

/* region starts among the selected windows (FilterFisherScores.py:103): a new region
 * begins at a sequence change or when start - gap > the previous selected start */
__global__ void k_rg_region_flags(const int64_t *__restrict__ sel, int64_t ns, const int32_t *__restrict__ seq,
                                  const int64_t *__restrict__ start, int64_t gap, uint8_t *__restrict__ f) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < ns; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = sel[j];
    uint8_t s = 1;
    if (j > 0) {
      const int64_t p = sel[j - 1];
      s = seq[i] != seq[p] || start[i] - gap > start[p];
    }
    f[j] = s;
  }
}

/* region r spans selected windows [rs[r], rs[r+1]); it is written as
 * (first window, min(last start + gap, seq_end))  (FilterFisherScores.py:104-106) */
__global__ void k_rg_region_out(const int64_t *__restrict__ rs, int64_t nr, const int64_t *__restrict__ sel,
                                int64_t ns, const int32_t *__restrict__ seq, const int64_t *__restrict__ start,
                                int64_t gap, const int64_t *__restrict__ seq_end, int64_t *__restrict__ first,
                                int64_t *__restrict__ end) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nr; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t jl = (r + 1 < nr ? rs[r + 1] : ns) - 1;
    const int64_t il = sel[jl];
    const int64_t e = start[il] + gap, lim = seq_end[seq[il]];
    first[r] = sel[rs[r]];
    end[r] = e < lim ? e : lim;
  }
}

/* ------------------------------------------------------------ host helpers */
static unsigned grid_for(int64_t n) {
  int64_t g = (n + RG_BLOCK - 1) / RG_BLOCK;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

/* arguments may live in host or device memory (unified addressing): host arrays are
 * staged into stream-ordered device buffers, and every buffer taken here is released
 * on the stream when the call returns */
struct Pool {
  hipStream_t s;
  std::vector<void *> held;
  explicit Pool(hipStream_t st) : s(st) {}
  ~Pool() {
    for (void *p : held) (void)hipFreeAsync(p, s);
  }
  template <class T>
  int take(T **out, size_t n) {
    void *p = nullptr;
    RG_TRY(hipMallocAsync(&p, sizeof(T) * (n ? n : 1), s));
    held.push_back(p);
    *out = (T *)p;
    return GD_OK;
  }
};

static bool on_device(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.type == hipMemoryTypeArray;
}

template <class T>
static int stage_in(Pool &pl, const T *p, size_t n, const T **out) {
  if (!n || on_device(p)) {
    *out = p;
    return GD_OK;
  }
  T *d;
  int st = pl.take(&d, n);
  if (st) return st;
  RG_TRY(hipMemcpyAsync(d, p, sizeof(T) * n, hipMemcpyHostToDevice, pl.s));
  *out = d;
  return GD_OK;
}

/* ascending numpy-order keys of v[0..n) */
static int sorted_keys(Pool &pl, const double *v, int64_t n, uint64_t **out) {
  uint64_t *k, *o;
  int st;
  if ((st = pl.take(&k, n)) || (st = pl.take(&o, n))) return st;
  hipLaunchKernelGGL(k_rg_keys, dim3(grid_for(n)), dim3(RG_BLOCK), 0, pl.s, v, n, k);
  RG_TRY(hipGetLastError());
  size_t bytes = 0;
  RG_TRY(rocprim::radix_sort_keys(nullptr, bytes, k, o, (size_t)n, 0, 64, pl.s));
  void *tmp;
  if ((st = pl.take((char **)&tmp, bytes))) return st;
  RG_TRY(rocprim::radix_sort_keys(tmp, bytes, k, o, (size_t)n, 0, 64, pl.s));
  *out = o;
  return GD_OK;
}

static int key_at(Pool &pl, const uint64_t *keys, int64_t i, double *x) {
  uint64_t k;
  RG_TRY(hipMemcpyAsync(&k, keys + i, 8, hipMemcpyDeviceToHost, pl.s));
  RG_TRY(hipStreamSynchronize(pl.s));
  *x = okey_value(k);
  return GD_OK;
}

/* Python's float % 1.0 for the non-negative index of scoreatpercentile */
static double frac1(double x) { return std::fmod(x, 1.0); }

/* scipy.stats.scoreatpercentile as of the tool's scipy (0.x, which still had cmedian):
 * idx = per/100. * (n-1); values[idx] if integral, else a + (b - a) * (idx % 1) */
static int score_at_percentile(Pool &pl, const double *v, int64_t n, double per, double *out) {
  uint64_t *keys;
  int st = sorted_keys(pl, v, n, &keys);
  if (st) return st;
  const double idx = per / 100. * (double)(n - 1);
  const int64_t i = (int64_t)idx;
  double a, b;
  if ((st = key_at(pl, keys, i, &a))) return st;
  if (frac1(idx) == 0) {
    *out = a;
    return GD_OK;
  }
  if (i + 1 >= n) return rg_fail(GD_ERR_ARG, "percentile index past the last window (IndexError)");
  if ((st = key_at(pl, keys, i + 1, &b))) return st;
  *out = a + (b - a) * frac1(idx);
  return GD_OK;
}

/* scipy.stats.cmedian(a, numbins=1000) (scipy 0.9-0.11, restated with its floating-point
 * steps): scipy.stats.histogram over its default limits (smallest = min - s,
 * max + s), s = (max - min) / (2 (numbins - 1)), binsize = bin_edges[1] - bin_edges[0];
 * cfbin = searchsorted(cumhist, n/2.0); LRL = smallest + binsize * cfbin; median = LRL +
 * ((n/2.0 - cumhist[cfbin-1]) / hist[cfbin]) * binsize, with Python's cumhist[-1] at
 * cfbin == 0 */
static int cmedian(Pool &pl, const double *v, int64_t n, double *out) {
  unsigned long long *mm;
  int st;
  if ((st = pl.take(&mm, 3))) return st;
  const unsigned long long init[3] = {~0ull, 0ull, 0ull};
  RG_TRY(hipMemcpyAsync(mm, init, sizeof init, hipMemcpyHostToDevice, pl.s));
  hipLaunchKernelGGL(k_rg_minmax, dim3(grid_for(n)), dim3(RG_BLOCK), 0, pl.s, v, n, mm);
  RG_TRY(hipGetLastError());
  unsigned long long h_mm[3];
  RG_TRY(hipMemcpyAsync(h_mm, mm, sizeof h_mm, hipMemcpyDeviceToHost, pl.s));
  RG_TRY(hipStreamSynchronize(pl.s));
  if (h_mm[2]) return rg_fail(GD_ERR_ARG, "cmedian: non-finite score (numpy.histogram range is not finite)");
  const double dmin = okey_value(h_mm[0]), dmax = okey_value(h_mm[1]);
  const int nb = RG_CMEDIAN_BINS;
  const double s = (dmax - dmin) / (2. * (nb - 1.));
  const double smallest = dmin - s;
  double first = smallest, last = dmax + s;
  if (first == last) { /* numpy.histogram widens an empty range by 0.5 each side */
    first -= 0.5;
    last += 0.5;
  }
  std::vector<double> edges(nb + 1); /* numpy.linspace(first, last, nb + 1) */
  const double delta = last - first, step = delta / nb;
  for (int i = 0; i <= nb; ++i) edges[i] = (step == 0 ? (double)i / nb * delta : (double)i * step) + first;
  edges[nb] = last;
  double *d_edges;
  unsigned long long *d_cnt;
  if ((st = pl.take(&d_edges, nb + 1)) || (st = pl.take(&d_cnt, nb))) return st;
  RG_TRY(hipMemcpyAsync(d_edges, edges.data(), sizeof(double) * (nb + 1), hipMemcpyHostToDevice, pl.s));
  RG_TRY(hipMemsetAsync(d_cnt, 0, sizeof(unsigned long long) * nb, pl.s));
  hipLaunchKernelGGL(k_rg_hist, dim3(grid_for(n)), dim3(RG_BLOCK), 0, pl.s, v, n, d_edges, d_cnt);
  RG_TRY(hipGetLastError());
  std::vector<unsigned long long> hist(nb);
  RG_TRY(hipMemcpyAsync(hist.data(), d_cnt, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost, pl.s));
  RG_TRY(hipStreamSynchronize(pl.s));
  std::vector<long long> cum(nb);
  long long acc = 0;
  for (int i = 0; i < nb; ++i) cum[i] = acc += (long long)hist[i];
  const double half = (double)n / 2.0;
  int cfbin = 0;
  while (cfbin < nb && (double)cum[cfbin] < half) ++cfbin;
  if (cfbin == nb) return rg_fail(GD_ERR_ARG, "cmedian: histogram lost values"); /* cannot happen */
  const double binsize = edges[1] - edges[0];
  const double lrl = smallest + binsize * (double)cfbin;
  const double cfbelow = (double)cum[cfbin == 0 ? nb - 1 : cfbin - 1];
  const double freq = (double)hist[cfbin];
  *out = lrl + ((half - cfbelow) / freq) * binsize;
  return GD_OK;
}

/* ----------------------------------------------------------- entry points */
int gd_rg_fet_limit(const double *scores, const double *stddev, int64_t n, double qnorm, double percentile,
                    double *out, hipStream_t s) {
  if (n <= 0) return rg_fail(GD_ERR_SIZE, "empty score track (numpy min of an empty array)");
  if (!scores || !stddev || !out) return rg_fail(GD_ERR_ARG, "null pointer");
  if (!(percentile >= 0 && percentile <= 100)) return rg_fail(GD_ERR_ARG, "percentile must lie in [0, 100]");
  Pool pl(s);
  const double *d_sc, *d_sd;
  int st;
  if ((st = stage_in(pl, scores, (size_t)n, &d_sc)) || (st = stage_in(pl, stddev, (size_t)n, &d_sd))) return st;
  double med, upq;
  if ((st = cmedian(pl, d_sc, n, &med))) return st;
  if ((st = score_at_percentile(pl, d_sd, n, percentile, &upq))) return st;
  out[0] = med + qnorm * upq;
  out[1] = med;
  out[2] = upq;
  RG_TRY(hipStreamSynchronize(s));
  return GD_OK;
}

int gd_rg_fdr_threshold(const double *p, int64_t n, double fdr, double *testp, int64_t *k_out, hipStream_t s) {
  if (!testp || !k_out || n < 0 || (n > 0 && !p)) return rg_fail(GD_ERR_ARG, "bad arguments");
  *testp = 0;
  *k_out = 0;
  if (n == 0) return GD_OK;
  Pool pl(s);
  const double *d_p;
  uint64_t *keys;
  unsigned long long *best;
  int st;
  if ((st = stage_in(pl, p, (size_t)n, &d_p)) || (st = sorted_keys(pl, d_p, n, &keys)) ||
      (st = pl.take(&best, 1)))
    return st;
  RG_TRY(hipMemsetAsync(best, 0, 8, pl.s));
  hipLaunchKernelGGL(k_rg_bh, dim3(grid_for(n)), dim3(RG_BLOCK), 0, pl.s, keys, n, fdr, best);
  RG_TRY(hipGetLastError());
  unsigned long long k;
  RG_TRY(hipMemcpyAsync(&k, best, 8, hipMemcpyDeviceToHost, pl.s));
  RG_TRY(hipStreamSynchronize(pl.s));
  if (k) {
    if ((st = key_at(pl, keys, (int64_t)k - 1, testp))) return st;
    *k_out = (int64_t)k;
  }
  RG_TRY(hipStreamSynchronize(s));
  return GD_OK;
}

int gd_rg_top_limit(const double *scores, int64_t n, int64_t num_top, double *limit, hipStream_t s) {
  if (!limit || n < 0 || (n > 0 && !scores)) return rg_fail(GD_ERR_ARG, "bad arguments");
  /* scores[argsort(scores)[::-1][num_top - 1]] with Python indexing */
  int64_t d = num_top - 1;
  if (d < 0) d += n;
  if (d < 0 || d >= n) return rg_fail(GD_ERR_ARG, "num_top outside the track (IndexError)");
  Pool pl(s);
  const double *d_sc;
  uint64_t *keys;
  int st;
  if ((st = stage_in(pl, scores, (size_t)n, &d_sc)) || (st = sorted_keys(pl, d_sc, n, &keys))) return st;
  if ((st = key_at(pl, keys, n - 1 - d, limit))) return st;
  RG_TRY(hipStreamSynchronize(s));
  return GD_OK;
}

int gd_rg_merge(const double *vals, const int32_t *seq, const int64_t *start, int64_t n, int cmp, double thr,
                int64_t gap, const int64_t *seq_end, int nseq, int64_t *region_first, int64_t *region_end,
                int64_t *nregions, int64_t *nselected, hipStream_t s) {
  if (!nregions || n < 0 || (n > 0 && (!vals || !seq || !start || !seq_end || nseq <= 0)) ||
      (cmp != GD_SELECT_GE && cmp != GD_SELECT_LE))
    return rg_fail(GD_ERR_ARG, "bad arguments");
  *nregions = 0;
  if (nselected) *nselected = 0;
  if (n == 0) return GD_OK;
  Pool pl(s);
  const double *d_v;
  const int32_t *d_seq;
  const int64_t *d_start, *d_end;
  int st;
  if ((st = stage_in(pl, vals, (size_t)n, &d_v)) || (st = stage_in(pl, seq, (size_t)n, &d_seq)) ||
      (st = stage_in(pl, start, (size_t)n, &d_start)) || (st = stage_in(pl, seq_end, (size_t)nseq, &d_end)))
    return st;
  uint8_t *flag;
  int64_t *sel, *rs, *cnt;
  if ((st = pl.take(&flag, n)) || (st = pl.take(&sel, n)) || (st = pl.take(&rs, n)) || (st = pl.take(&cnt, 3)))
    return st;
  RG_TRY(hipMemsetAsync(cnt, 0, 3 * sizeof(int64_t), pl.s));
  hipLaunchKernelGGL(k_rg_select_flags, dim3(grid_for(n)), dim3(RG_BLOCK), 0, pl.s, d_v, d_seq, n, nseq, cmp, thr,
                     flag, cnt + 2);
  RG_TRY(hipGetLastError());
  rocprim::counting_iterator<int64_t> idx(0);
  size_t bytes = 0;
  RG_TRY(rocprim::select(nullptr, bytes, idx, flag, sel, cnt, (size_t)n, pl.s));
  char *tmp;
  if ((st = pl.take(&tmp, bytes))) return st;
  RG_TRY(rocprim::select(tmp, bytes, idx, flag, sel, cnt, (size_t)n, pl.s));
  int64_t h_cnt[3];
  RG_TRY(hipMemcpyAsync(h_cnt, cnt, sizeof h_cnt, hipMemcpyDeviceToHost, pl.s));
  RG_TRY(hipStreamSynchronize(pl.s));
  if (h_cnt[2]) return rg_fail(GD_ERR_ARG, "sequence index outside [0, nseq)");
  const int64_t ns = h_cnt[0];
  if (nselected) *nselected = ns;
  if (ns == 0) return GD_OK;
  if (!region_first || !region_end) return rg_fail(GD_ERR_ARG, "null region outputs");
  hipLaunchKernelGGL(k_rg_region_flags, dim3(grid_for(ns)), dim3(RG_BLOCK), 0, pl.s, sel, ns, d_seq, d_start, gap,
                     flag);
  RG_TRY(hipGetLastError());
  size_t bytes2 = 0;
  RG_TRY(rocprim::select(nullptr, bytes2, idx, flag, rs, cnt + 1, (size_t)ns, pl.s));
  char *tmp2;
  if ((st = pl.take(&tmp2, bytes2))) return st;
  RG_TRY(rocprim::select(tmp2, bytes2, idx, flag, rs, cnt + 1, (size_t)ns, pl.s));
  int64_t nr;
  RG_TRY(hipMemcpyAsync(&nr, cnt + 1, 8, hipMemcpyDeviceToHost, pl.s));
  RG_TRY(hipStreamSynchronize(pl.s));
  const bool dev_out = on_device(region_first) && on_device(region_end);
  int64_t *o_first = region_first, *o_end = region_end;
  if (!dev_out && ((st = pl.take(&o_first, nr)) || (st = pl.take(&o_end, nr)))) return st;
  hipLaunchKernelGGL(k_rg_region_out, dim3(grid_for(nr)), dim3(RG_BLOCK), 0, pl.s, rs, nr, sel, ns, d_seq, d_start,
                     gap, d_end, o_first, o_end);
  RG_TRY(hipGetLastError());
  if (!dev_out) {
    RG_TRY(hipMemcpyAsync(region_first, o_first, 8 * nr, hipMemcpyDeviceToHost, pl.s));
    RG_TRY(hipMemcpyAsync(region_end, o_end, 8 * nr, hipMemcpyDeviceToHost, pl.s));
  }
  RG_TRY(hipStreamSynchronize(pl.s));
  *nregions = nr;
  return GD_OK;
}
