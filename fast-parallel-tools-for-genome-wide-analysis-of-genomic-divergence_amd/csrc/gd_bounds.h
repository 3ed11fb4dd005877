/*
 * gd_bounds.h -- slide_right() (comparative.c:49-71) for every window of one population of
 * one chromosome, one wave-segment at a time.  Shared by the stand-alone pass k_bounds
 * (gd_fet_kernels.hip), which every FET and CSS scan runs once per chromosome group before
 * its window kernels.
 *
 * lo = first idx with pos >= start, hi = first idx with pos > start + wsize (inclusive
 * end).  Element i owns the windows whose start lies in (pos[i-1], pos[i]] (lo) and whose
 * inclusive stop lies in [pos[i-1], pos[i]) (hi); i == len is the +inf sentinel.  Within a
 * SNP's run of identical positions nothing is owned, so the common case is one compare.
 */
#pragma once
#include "gd_internal.h"

/* floor(a / b) for b > 0, |a| < 2^40: double-reciprocal estimate, one fix-up step */
__device__ __forceinline__ int64_t gd_fdiv_fast(int64_t a, int32_t b, double inv) {
  int64_t q = (int64_t)floor((double)a * inv);
  const int64_t r = a - q * (int64_t)b;
  q += (r >= b) - (r < 0);
  return q;
}

/* one (chromosome, population) pass: its positions, outputs and the window-index division */
struct gd_bounds_job {
  const int32_t *pos;
  int32_t *lo, *hi; /* hi: A only */
  int64_t len, wend, wf; /* wf: the chromosome index of local window 0 (window-range shards) */
  int wsize, wstep, pop;
  double inv;
  int kl;
  uint32_t kmag, ksh;
  bool aligned16; /* int4 loads stay 16-byte aligned */

  gd_bounds_job() = default;
  __device__ __forceinline__ gd_bounds_job(const gd_chrom_dev &d, int pop_, const int32_t *apos, const int32_t *bpos,
                                           int wsize_, int wstep_, int32_t *lo_a, int32_t *hi_a, int32_t *lo_b) {
    init(d, pop_, apos, bpos, wsize_, wstep_, lo_a, hi_a, lo_b);
  }
  __device__ __forceinline__ void init(const gd_chrom_dev &d, int pop_, const int32_t *apos, const int32_t *bpos,
                                       int wsize_, int wstep_, int32_t *lo_a, int32_t *hi_a, int32_t *lo_b) {
    pop = pop_;
    wend = d.wend;
    wf = d.w_first;
    len = pop ? d.blen : d.alen;
    pos = pop ? bpos + d.b_off : apos + d.a_off;
    lo = (pop ? lo_b : lo_a) + d.w_base;
    hi = hi_a + d.w_base;
    wsize = wsize_;
    wstep = wstep_;
    inv = 1.0 / (double)wstep;
    /* floor(a / wstep) for 0 <= a < 2^31 as a multiply-high (Granlund-Montgomery, N = 31:
     * mag = ceil(2^(31+l) / wstep), l = ceil(log2 wstep)); other a (negative near the
     * chromosome start, wstep == 1) take gd_fdiv_fast */
    kl = 0;
    while ((1ll << kl) < wstep) ++kl;
    kmag = kl > 0 ? (uint32_t)(((1ull << (31 + kl)) + (uint64_t)wstep - 1) / (uint64_t)wstep) : 0u;
    ksh = kl > 0 ? (uint32_t)(kl - 1) : 0u;
    aligned16 = ((pop ? d.b_off : d.a_off) & 3) == 0;
  }

  __device__ __forceinline__ int64_t fl(int64_t a) const {
    if (kl > 0 && a >= 0 && a < 0x80000000ll) return (int64_t)(__umulhi((uint32_t)a, kmag) >> ksh);
    return gd_fdiv_fast(a, wstep, inv);
  }

  /* element i (a boundary: i == 0, i == len or pos[i] != pos[i-1]) with p = pos[i] (i < len)
   * and pp = pos[i-1] (i > 0) */
  __device__ __forceinline__ void own(int64_t i, int64_t p, int64_t pp) const {
    const bool first = (i == 0), last = (i == len);
    int64_t f = first ? 0 : fl(pp) + 1 - wf;
    int64_t l = last ? wend - 1 : fl(p) - wf;
    if (f < 0) f = 0;
    if (l > wend - 1) l = wend - 1;
    for (int64_t w = f; w <= l; ++w) lo[w] = (int32_t)i;
    if (pop == 0) {
      /* -floor((wsize - x) / wstep) = ceil((x - wsize) / wstep) = floor((x - wsize + wstep - 1) / wstep) */
      f = first ? 0 : fl(pp - wsize + wstep - 1) - wf;
      l = last ? wend - 1 : fl(p - wsize + wstep - 1) - 1 - wf;
      if (f < 0) f = 0;
      if (l > wend - 1) l = wend - 1;
      for (int64_t w = f; w <= l; ++w) hi[w] = (int32_t)i;
    }
  }

  /* One wave's segment of 256 CH elements starting at seg (seg <= len).  Full aligned
   * segments (full()): lane l's chunk k holds elements seg + 256 k + 4 l .. + 3 (one
   * coalesced int4 per chunk, load()); process() marks boundaries in a bit mask (three VALU
   * per element: unsigned difference, min with 1, shift-or), then the lane walks just those
   * bits, reading pos[i] and pos[i-1] from the wave's LDS copy sg of the segment (256 CH
   * ints; nullptr: from memory).  The partial last segment goes element by element (4 CH
   * consecutive elements per lane, partial()).  Each returns true when a decrease was seen
   * (unsorted positions). */
  template <int CH>
  __device__ __forceinline__ bool full(int64_t seg) const {
    return aligned16 && seg + 256 * CH <= len;
  }
  template <int CH>
  __device__ __forceinline__ void load(int64_t seg, int4 (&v)[CH], int32_t &before) const {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < CH; ++k) v[k] = *reinterpret_cast<const int4 *>(pos + seg + 256 * k + 4 * lane);
    before = seg > 0 ? pos[seg - 1] : 0; /* element 0 has no predecessor (process: v[0].x) */
  }
  template <int CH>
  __device__ __forceinline__ bool process(int64_t seg, const int4 (&v)[CH], int32_t before, int32_t *sg) const {
    static_assert(CH >= 1 && 4 * CH <= 32, "the boundary mask holds 4 CH bits in a uint32_t");
    const int lane = threadIdx.x & 63;
    if (seg == 0) before = v[0].x;
    uint32_t bits = 0;
    bool dec = false;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int32_t up = __shfl_up(v[k].w, 1);
      const int32_t wrap = __shfl(v[k > 0 ? k - 1 : 0].w, 63);
      const int32_t prev = lane > 0 ? up : (k > 0 ? wrap : before);
      const int32_t e[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
      int32_t pv = prev;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bits |= min((uint32_t)e[j] - (uint32_t)pv, 1u) << (4 * k + j);
        dec |= e[j] < pv;
        pv = e[j];
      }
    }
    if (seg == 0 && lane == 0) bits |= 1u; /* element 0 opens the first run */
    if (sg) {
#pragma unroll
      for (int k = 0; k < CH; ++k) *reinterpret_cast<int4 *>(sg + 256 * k + 4 * lane) = v[k];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      while (bits) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1;
        const int r = 256 * (b >> 2) + 4 * lane + (b & 3);
        own(seg + r, sg[r], r > 0 ? sg[r - 1] : before);
      }
      __builtin_amdgcn_wave_barrier(); /* the slice is rewritten by the next segment */
    } else {
      while (bits) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1;
        const int64_t i = seg + 256 * (b >> 2) + 4 * lane + (b & 3);
        own(i, pos[i], i > 0 ? pos[i - 1] : 0);
      }
    }
    return dec;
  }
  template <int CH>
  __device__ __forceinline__ bool partial(int64_t seg) const {
    constexpr int SEG = 256 * CH;
    const int lane = threadIdx.x & 63;
    bool unsorted = false;
    for (int64_t i0 = seg + 4 * CH * lane; i0 < seg + SEG && i0 <= len; i0 += SEG) {
      int32_t prev = (i0 > 0) ? pos[i0 - 1] : 0;
      for (int k = 0; k < 4 * CH && i0 + k <= len; ++k) {
        const int64_t i = i0 + k;
        const int32_t v = (i < len) ? pos[i] : 0;
        const bool bnd = (i == 0) || (i == len) || (v != prev);
        if (i > 0 && i < len) unsorted |= (v < prev);
        if (bnd) own(i, v, prev);
        prev = v;
      }
    }
    return unsorted;
  }
  template <int CH>
  __device__ __forceinline__ bool segment(int64_t seg, int32_t *sg) const {
    if (!full<CH>(seg)) return partial<CH>(seg);
    int4 v[CH];
    int32_t before;
    load<CH>(seg, v, before);
    return process<CH>(seg, v, before, sg);
  }
};

/* get_population_size() (comparative.c:25-34) of one population by one wave: the leading
 * run of pos[0], bounded by the array length */
__device__ __forceinline__ int gd_popsize_wave(const int32_t *p, int len) {
  const int lane = threadIdx.x & 63;
  int size = len;
  if (len > 0) {
    const int32_t p0 = p[0];
    for (int base = 0; base < len; base += 64) {
      const int i = base + lane;
      const unsigned long long m = __ballot(i < len && p[i] != p0);
      if (m) {
        size = base + __ffsll((long long)m) - 1;
        break;
      }
    }
  }
  return size;
}
