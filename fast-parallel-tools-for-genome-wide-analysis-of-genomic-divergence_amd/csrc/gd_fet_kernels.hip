/*
 * gd_fet_kernels.hip -- HIP/CDNA4 kernels of the Fisher-exact-test window scan.
 *
 * Pipeline (one stream, no host round trip):
 *   k_popsize        get_population_size() per chromosome      comparative.c:25-34
 *   k_bounds         slide_right() for every window at once:    comparative.c:49-71
 *                    one coalesced pass over the positions; element i owns the
 *                    windows whose start (or inclusive stop) falls between
 *                    pos[i-1] and pos[i]
 *   k_snp_fet        fetcount() + fet() + -log10 once per SNP    cFisher.c:180-184
 *                    (the reference recomputes each SNP in every one of the
 *                    ~wsize/wstep windows covering it; the value depends only on
 *                    the SNP's four counts, so computing it once is exact)
 *   k_fet_window_*   percentile + 100-replicate bootstrap std   cFisher.c:136-144, 547-597
 * All FP arithmetic is compiled with -ffp-contract=off (the reference build has no FMA).
 */
#include "gd_common.h"
#include "gd_bounds.h"
#include "gd_fet_rows.h"
#include "gd_internal.h"

namespace {

__device__ __forceinline__ int64_t fdiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
__device__ __forceinline__ int64_t cdiv(int64_t a, int64_t b) { return -fdiv(-a, b); }

__device__ __forceinline__ int chrom_of(const gd_chrom_dev *ch, int nchrom, int64_t g) {
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

}  // namespace

/* ------------------------------------------------------------------------ */
__global__ void k_binom_table(uint64_t *tab) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= GD_BINOM_ENTRIES) return;
  int n = 0;
  while ((n + 1) * (n + 2) / 2 <= e) ++n;
  const int k = e - n * (n + 1) / 2;
  tab[e] = gd_binomial_ref((uint64_t)n, (uint64_t)k);
}

/* get_population_size(): leading run of pos[0], bounded by the array length */
__device__ __forceinline__ void popsize_store(gd_chrom_dev &d, const int32_t *apos, const int32_t *bpos,
                                              unsigned *flags) {
  const int sa = gd_popsize_wave(apos + d.a_off, d.alen), sb = gd_popsize_wave(bpos + d.b_off, d.blen);
  if ((threadIdx.x & 63) == 0) {
    d.asize = sa;
    d.bsize = sb;
    d.nrows = 0;
    if (d.wend > 0 && (sa <= 0 || sb <= 0)) atomicOr(flags, GD_FLAG_BAD_SIZE);
    if (sa > 0 && sb > 0) {
      const int ra = d.alen / sa, rb = d.blen / sb;
      d.nrows = ra < rb ? ra : rb;
    }
  }
}

__global__ void __launch_bounds__(64) k_popsize(gd_chrom_dev *ch, const int32_t *apos, const int32_t *bpos,
                                                unsigned *flags) {
  popsize_store(ch[blockIdx.x], apos, bpos, flags);
}

/* slide_right() for all windows (gd_bounds.h).  Grid (x, chrom, pop); a wave scans
 * KB_SEG-element segments grid-strided, reading each segment with KB_CH coalesced int4
 * loads per lane. */
#ifndef KB_CH
#define KB_CH 4 /* int4 chunks per lane and segment (loads in flight; 4: 0.326 ms per C2 bounds pass, 8: 0.312 (parity not yet run on the GPU), 2: 0.366) */
#endif
__global__ void __launch_bounds__(256) k_bounds(const gd_chrom_dev *ch, const int32_t *apos, const int32_t *bpos,
                                                int wsize, int wstep, int32_t *lo_a, int32_t *hi_a,
                                                int32_t *lo_b, unsigned *flags) {
  constexpr int KB_SEG = 256 * KB_CH;
  __shared__ __attribute__((aligned(16))) int32_t kb_sh[4][KB_SEG];
  const gd_chrom_dev &d = ch[blockIdx.y];
  if (d.wend <= 0) return;
  const gd_bounds_job job(d, blockIdx.z, apos, bpos, wsize, wstep, lo_a, hi_a, lo_b);
  const int64_t wave0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  bool unsorted = false;
  for (int64_t seg = wave0 * KB_SEG; seg <= job.len; seg += nwaves * KB_SEG)
    unsorted |= job.segment<KB_CH>(seg, kb_sh[threadIdx.x >> 6]);
  if (unsorted) atomicOr(flags, job.pop ? GD_FLAG_UNSORTED_B : GD_FLAG_UNSORTED_A);
}

/* ------------------------------------------------------------------------ */
/* Per-SNP FET.  A workgroup takes a tile of R SNP rows.  Its four waves stream   */
/* the tile's genotype values with coalesced 16-byte loads (two values per lane,  */
/* 128 per wave-instruction) and turn them into ballot bit masks of "== 3" and     */
/* "== -3" (even / odd element of each lane separately), kept in LDS.  Thread r   */
/* then counts its row's bits with popcounts, runs the Zar two-tailed test and     */
/* -log10.  Values are read once from HBM at full width; the FP compare is the     */
/* reference's exact double compare (fetcount, cFisher.c:216-233).               */
/* ------------------------------------------------------------------------ */
/* skip_table_held: fused scans score rows inside the window kernel whenever the
 * score table holds the chromosome's sizes; only the other chromosomes run here */
__global__ void __launch_bounds__(256) k_snp_fet(const gd_chrom_dev *ch, const double *avals, const double *bvals,
                                                 const uint64_t *binom, const int *lut_hdr, const double *lut,
                                                 double *snp_score, int skip_table_held) {
  __shared__ uint64_t sh_m[2][2][SF_MAXCH][2]; /* [pop][maj/min][chunk][even/odd] */
  const gd_chrom_dev &d = ch[blockIdx.y];
  if (d.wend <= 0) return;
  const int nrows = d.nrows, asize = d.asize, bsize = d.bsize;
  const bool use_lut = gd_lut_holds(lut_hdr, asize, bsize, binom);
  if (use_lut && skip_table_held) return;
  const int lut_nb = (bsize + 1) * (bsize + 2) / 2;
  const int big = max(asize, bsize);
  const int R = min(256, ((SF_MAXCH - 2) * 128) / max(big, 1));
  if (R <= 0 || nrows <= 0) return;
  const int ntiles = (nrows + R - 1) / R;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int s0 = tile * R;
    const int rows = min(R, nrows - s0);
    int rel0[2];
    for (int pop = 0; pop < 2; ++pop) {
      const int size = pop ? bsize : asize;
      const double *vals = pop ? bvals : avals;
      const int64_t start = (pop ? d.b_off : d.a_off) + (int64_t)s0 * size;
      const int64_t stop = start + (int64_t)rows * size;
      const int64_t gb = start & ~(int64_t)1; /* 16-byte aligned element */
      rel0[pop] = (int)(start - gb);
      const int nch = (int)((stop - gb + 127) >> 7);
      for (int k = wave; k < nch; k += 4) {
        const int64_t e = gb + ((int64_t)k << 7) + 2 * lane;
        double v0 = 0.0, v1 = 0.0;
        if (e + 1 < stop) {
          const double2 t = *reinterpret_cast<const double2 *>(vals + e);
          v0 = t.x;
          v1 = t.y;
        } else if (e < stop) {
          v0 = vals[e];
        }
        const uint64_t ja = __ballot(v0 == 3.0), jb = __ballot(v1 == 3.0);
        const uint64_t na = __ballot(v0 == -3.0), nb = __ballot(v1 == -3.0);
        if (lane == 0) {
          sh_m[pop][0][k][0] = ja;
          sh_m[pop][0][k][1] = jb;
          sh_m[pop][1][k][0] = na;
          sh_m[pop][1][k][1] = nb;
        }
      }
    }
    __syncthreads();
    const int r = threadIdx.x;
    if (r < rows) {
      const int sa = rel0[0] + r * asize, sb = rel0[1] + r * bsize;
      const int f0 = count_range(sh_m[0][0], sa, sa + asize);
      const int f1 = count_range(sh_m[0][1], sa, sa + asize);
      const int f2 = count_range(sh_m[1][0], sb, sb + bsize);
      const int f3 = count_range(sh_m[1][1], sb, sb + bsize);
      snp_score[d.a_off + s0 + r] =
          use_lut ? lut[(int64_t)gd_pair_index(f0, f1, asize) * lut_nb + gd_pair_index(f2, f3, bsize)]
                  : gd_fet_score_from_p(fet_p_two_tailed(f0, f1, f2, f3, binom));
    }
    __syncthreads();
  }
}

/* ------------------------------------------------------------------------ */
/* Score table: -log10 p of every 2x2 table (majA, minA, majB, minB) with      */
/* majA + minA <= asize and majB + minB <= bsize, computed by the same device */
/* code as above (so a lookup is bit-identical to a direct evaluation).  Built */
/* once per (asize, bsize) and kept in the context; k_snp_fet then only counts */
/* and gathers.  20+20 individuals: 231 x 231 = 53,361 tables (427 KB, L2).    */
/* hdr = {asize, bsize, valid, mode}.                                               */
/* ------------------------------------------------------------------------ */
__global__ void __launch_bounds__(256) k_fet_lut_build(const gd_chrom_dev *ch, const uint64_t *binom,
                                                       const int *hdr, double *lut, int64_t cap) {
  const int asize = ch[0].asize, bsize = ch[0].bsize;
  if (asize <= 0 || bsize <= 0) return;
  if (hdr[2] == 1 && hdr[0] == asize && hdr[1] == bsize && hdr[3] == fet_mode(binom)) return; /* cached */
  const int64_t na = (int64_t)(asize + 1) * (asize + 2) / 2, nb = (int64_t)(bsize + 1) * (bsize + 2) / 2;
  if (na * nb > cap) return;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < na * nb; e += (int64_t)gridDim.x * blockDim.x) {
    int ia = (int)(e / nb), ib = (int)(e - (int64_t)ia * nb);
    int a = 0, c = 0;
    while (ia >= asize + 1 - a) {
      ia -= asize + 1 - a;
      ++a;
    }
    while (ib >= bsize + 1 - c) {
      ib -= bsize + 1 - c;
      ++c;
    }
    lut[e] = gd_fet_score_from_p(fet_p_two_tailed(a, ia, c, ib, binom));
  }
}

__global__ void k_fet_lut_publish(const gd_chrom_dev *ch, const uint64_t *binom, int *hdr, int64_t cap) {
  const int asize = ch[0].asize, bsize = ch[0].bsize;
  const int64_t na = (int64_t)(asize + 1) * (asize + 2) / 2, nb = (int64_t)(bsize + 1) * (bsize + 2) / 2;
  const bool ok = asize > 0 && bsize > 0 && na * nb <= cap;
  hdr[0] = asize;
  hdr[1] = bsize;
  hdr[2] = ok ? 1 : 0;
  hdr[3] = fet_mode(binom);
}

/* The prologue of a grouped FET scan in one launch (gd_api.hip): every chromosome's
 * population sizes (one wave each, as k_popsize), the score table for chromosome 0's sizes
 * when the context does not hold it yet (as k_fet_lut_build; every workgroup derives the
 * sizes itself from the positions, so nothing waits for the size pass), and the header,
 * written by the last workgroup to finish (done: a zeroed counter).  With the table
 * cached the launch only reads a few positions per chromosome. */
__global__ void __launch_bounds__(256) k_fet_setup(gd_chrom_dev *ch, int nchrom, const int32_t *apos,
                                                   const int32_t *bpos, unsigned *flags, const uint64_t *binom,
                                                   int *hdr, double *lut, int64_t cap, unsigned *done) {
  __shared__ int sh_sz[2];
  const int wave = threadIdx.x >> 6;
  if (wave == 0) {
    const gd_chrom_dev &d0 = ch[0];
    const int sa = gd_popsize_wave(apos + d0.a_off, d0.alen), sb = gd_popsize_wave(bpos + d0.b_off, d0.blen);
    if (threadIdx.x == 0) {
      sh_sz[0] = sa;
      sh_sz[1] = sb;
    }
  }
  for (int c = blockIdx.x * 4 + wave; c < nchrom; c += gridDim.x * 4) popsize_store(ch[c], apos, bpos, flags);
  __syncthreads();
  const int asize = sh_sz[0], bsize = sh_sz[1];
  const int64_t na = (int64_t)(asize + 1) * (asize + 2) / 2, nb = (int64_t)(bsize + 1) * (bsize + 2) / 2;
  const bool ok = asize > 0 && bsize > 0 && na * nb <= cap;
  const bool cached = hdr[2] == 1 && hdr[0] == asize && hdr[1] == bsize && hdr[3] == fet_mode(binom);
  if (ok && !cached) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < na * nb;
         e += (int64_t)gridDim.x * blockDim.x) {
      int ia = (int)(e / nb), ib = (int)(e - (int64_t)ia * nb);
      int a = 0, c = 0;
      while (ia >= asize + 1 - a) {
        ia -= asize + 1 - a;
        ++a;
      }
      while (ib >= bsize + 1 - c) {
        ib -= bsize + 1 - c;
        ++c;
      }
      lut[e] = gd_fet_score_from_p(fet_p_two_tailed(a, ia, c, ib, binom));
    }
  }
  /* the table and the header are read by later kernels only (kernel-boundary ordering): the
   * counter just picks the workgroup that writes the header after every slice is built */
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(done, 1u) == gridDim.x - 1) {
    hdr[0] = asize;
    hdr[1] = bsize;
    hdr[2] = ok ? 1 : 0;
    hdr[3] = fet_mode(binom);
  }
}

/* ------------------------------------------------------------------------ */
/* General window path: one workgroup per window, literal semantics.         */
/*   - scores gathered from snp_score when the window's A and B slices start  */
/*     on the same SNP row, else recomputed from the raw slices              */
/*   - ascending sort: bitonic (no NaN) or glibc-2.35 msort order (NaN)      */
/*   - bootstrap: the nrand48 stream is consumed in order, BLOCK positions   */
/*     per step, rejections compacted with a block scan                      */
/* ------------------------------------------------------------------------ */
namespace {

template <int BLOCK>
__device__ int block_incl_scan(int v, int *sh, int *total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int off = 1; off < BLOCK; off <<= 1) {
    const int add = (t >= off) ? sh[t - off] : 0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  const int r = sh[t];
  *total = sh[BLOCK - 1];
  __syncthreads();
  return r;
}

/* glibc 2.35 qsort == top-down merge sort, left run wins ties (cmp <= 0) */
__device__ void msort_glibc(double *a, double *tmp, int n) {
  struct Frame {
    int off, n, stage;
  };
  Frame st[64];
  int sp = 0;
  st[sp++] = {0, n, 0};
  while (sp) {
    Frame &fr = st[sp - 1];
    if (fr.n <= 1) {
      --sp;
      continue;
    }
    const int n1 = fr.n / 2;
    if (fr.stage == 0) {
      fr.stage = 1;
      st[sp++] = {fr.off, n1, 0};
    } else if (fr.stage == 1) {
      fr.stage = 2;
      st[sp++] = {fr.off + n1, fr.n - n1, 0};
    } else {
      double *b1 = a + fr.off, *b2 = a + fr.off + n1;
      int c1 = n1, c2 = fr.n - n1, o = 0;
      while (c1 > 0 && c2 > 0) {
        const double x = *b1, y = *b2;
        const int cmp = (x > y) - (x < y);
        if (cmp <= 0) {
          tmp[o++] = x;
          ++b1;
          --c1;
        } else {
          tmp[o++] = y;
          ++b2;
          --c2;
        }
      }
      while (c1 > 0) {
        tmp[o++] = *b1++;
        --c1;
      }
      for (int i = 0; i < o; ++i) a[fr.off + i] = tmp[i];
      --sp;
    }
  }
}

template <int BLOCK>
__device__ void bitonic_sort_pad(double *s, int n, int np2) {
  for (int i = n + threadIdx.x; i < np2; i += BLOCK) s[i] = __builtin_inf();
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np2; i += BLOCK) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const double x = s[i], y = s[ixj];
          const bool up = (i & k) == 0;
          if (up ? (x > y) : (x < y)) {
            s[i] = y;
            s[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace

template <int BLOCK, bool GLOBAL_SCRATCH>
__global__ void __launch_bounds__(BLOCK)
    k_fet_window_general(const gd_chrom_dev *ch, int nchrom, const int32_t *wlist, const unsigned *wlist_count,
                         int64_t wtotal, const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b,
                         const double *avals, const double *bvals, const double *snp_score,
                         const uint64_t *binom, const int *lut_hdr, const double *lut, double perc, double *scores,
                         double *stddev, unsigned *flags, int32_t *huge_list, unsigned *huge_count,
                         double *gscratch, int64_t gscratch_n) {
  __shared__ double sh_rep[GD_NREP];
  __shared__ int sh_scan[BLOCK];
  __shared__ uint64_t sh_x;
  __shared__ int sh_pick[2];
  __shared__ int sh_nan;
  constexpr int LDS_N = GLOBAL_SCRATCH ? 1 : GD_GEN_LDS_N;
  __shared__ double sh_s[LDS_N], sh_smp[LDS_N], sh_tmp[LDS_N];
  __shared__ uint32_t sh_hist[LDS_N];

  if (*flags & (GD_FLAG_UNSORTED_A | GD_FLAG_UNSORTED_B | GD_FLAG_BAD_SIZE)) return;
  const int tid = threadIdx.x;
  const int64_t count = wlist ? (int64_t)*wlist_count : wtotal;
  /* per-thread jump map: position P -> P + tid + 1 */
  const gd_affine jmp = gd_lcg_jump((uint64_t)tid + 1);

  for (int64_t it = blockIdx.x; it < count; it += gridDim.x) {
    const int64_t g = wlist ? (int64_t)wlist[it] : it;
    const int c = chrom_of(ch, nchrom, g);
    const gd_chrom_dev &d = ch[c];
    const int64_t w = g - d.w_base;
    const int asize = d.asize, bsize = d.bsize;
    const int lo = lo_a[g], hi = hi_a[g], lb = lo_b[g];
    const int n = (hi - lo) / asize;
    if (n <= 0) continue;
    if ((int64_t)lb + (int64_t)n * bsize > d.blen) {
      if (tid == 0) atomicOr(flags, GD_FLAG_B_BOUNDS);
      continue;
    }
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    double *S, *smp, *tmp;
    uint32_t *hist;
    if (GLOBAL_SCRATCH) {
      if ((int64_t)np2 + 2 * (int64_t)n + (n + 1) / 2 + 1 > gscratch_n) {
        if (tid == 0) atomicOr(flags, GD_FLAG_BAD_SIZE);
        continue;
      }
      double *base = gscratch + (int64_t)blockIdx.x * gscratch_n;
      S = base;
      smp = base + np2;
      tmp = smp + n;
      hist = (uint32_t *)(tmp + n);
    } else {
      if (np2 > LDS_N) {
        if (tid == 0) huge_list[atomicAdd(huge_count, 1u)] = (int32_t)g;
        continue;
      }
      S = sh_s;
      smp = sh_smp;
      tmp = sh_tmp;
      hist = sh_hist;
    }

    /* 1. per-SNP scores of the window, in window order */
    const bool aligned = (lo % asize == 0) && (lb % bsize == 0) && (lo / asize == lb / bsize) &&
                         (lo / asize + n <= d.nrows);
    if (tid == 0) sh_nan = 0;
    __syncthreads();
    int has_nan = 0;
    const bool held = lut_hdr && gd_lut_holds(lut_hdr, asize, bsize, binom);
    for (int i = tid; i < n; i += BLOCK) {
      double v;
      if (held) /* fused scans keep per-SNP scores only where the table misses */
        v = snp_score_table(avals + d.a_off + lo + (int64_t)i * asize, asize,
                            bvals + d.b_off + lb + (int64_t)i * bsize, bsize, lut);
      else if (aligned)
        v = snp_score[d.a_off + lo / asize + i];
      else
        v = snp_score_raw(avals + d.a_off + lo + (int64_t)i * asize, asize,
                          bvals + d.b_off + lb + (int64_t)i * bsize, bsize, binom);
      S[i] = v;
      has_nan |= (v != v);
    }
    if (has_nan) sh_nan = 1;
    __syncthreads();
    const bool nan_mode = sh_nan != 0;

    /* 2. ascending sort (qsort in percentile(), cFisher.c:140) */
    if (nan_mode) {
      if (tid == 0) msort_glibc(S, tmp, n);
      __syncthreads();
    } else {
      bitonic_sort_pad<BLOCK>(S, n, np2);
    }

    const int idx = gd_perc_index(n, perc);
    const double delta = gd_perc_delta(n, perc, idx);
    const int idx1 = (idx + 1 < n) ? idx + 1 : idx;
    const double wscore = gd_perc_mix(delta, S[idx], S[idx1]);

    /* 3. bootstrap: 100 replicates of n draws from the sorted scores */
    const gd_randint rd = gd_randint_make((uint32_t)n);
    uint64_t xP = gd_window_state(d.seed, GD_STREAM_FET, w + d.w_first);
    for (int i = tid; i < n; i += BLOCK) hist[i] = 0;
    __syncthreads();
    for (int rep = 0; rep < GD_NREP; ++rep) {
      int got = 0;
      while (got < n) {
        const uint64_t xt = gd_affine_apply(jmp, xP);
        const uint32_t r = gd_lcg_value(xt);
        const int ok = r <= rd.limit;
        int total;
        const int incl = block_incl_scan<BLOCK>(ok, sh_scan, &total);
        const int need = n - got;
        const int rank = incl - 1;
        if (ok && rank < need) {
          const int j = got + rank;
          const uint32_t v = gd_randint_mod(&rd, r);
          if (nan_mode)
            smp[n - 1 - j] = S[v];
          else
            atomicAdd(&hist[v], 1u);
        }
        if (total >= need) {
          if (ok && rank == need - 1) sh_x = xt;
          got = n;
        } else {
          if (tid == BLOCK - 1) sh_x = xt;
          got += total;
        }
        __syncthreads();
        xP = sh_x;
        __syncthreads();
      }
      /* percentile of the replicate */
      if (nan_mode) {
        if (tid == 0) {
          msort_glibc(smp, tmp, n);
          sh_rep[rep] = gd_perc_mix(delta, smp[idx], smp[idx1]);
        }
        __syncthreads();
      } else {
        const int per = (n + BLOCK - 1) / BLOCK;
        const int b0 = tid * per;
        int local = 0;
        for (int b = b0; b < b0 + per && b < n; ++b) local += (int)hist[b];
        int total;
        const int incl = block_incl_scan<BLOCK>(local, sh_scan, &total);
        int cum = incl - local;
        for (int b = b0; b < b0 + per && b < n; ++b) {
          const int h = (int)hist[b];
          if (cum <= idx && idx < cum + h) sh_pick[0] = b;
          if (cum <= idx1 && idx1 < cum + h) sh_pick[1] = b;
          cum += h;
        }
        __syncthreads();
        for (int b = b0; b < b0 + per && b < n; ++b) hist[b] = 0;
        if (tid == 0) sh_rep[rep] = gd_perc_mix(delta, S[sh_pick[0]], S[sh_pick[1]]);
        __syncthreads();
      }
    }
    if (tid == 0) {
      double sd;
      GD_STD_REVERSE(sd, sh_rep, GD_NREP);
      scores[d.w_out + w] = wscore;
      stddev[d.w_out + w] = sd;
    }
    __syncthreads();
  }
}

template __global__ void k_fet_window_general<64, false>(const gd_chrom_dev *, int, const int32_t *,
                                                         const unsigned *, int64_t, const int32_t *,
                                                         const int32_t *, const int32_t *, const double *,
                                                         const double *, const double *, const uint64_t *,
                                                         const int *, const double *, double, double *, double *,
                                                         unsigned *, int32_t *, unsigned *, double *, int64_t);
template __global__ void k_fet_window_general<256, true>(const gd_chrom_dev *, int, const int32_t *,
                                                         const unsigned *, int64_t, const int32_t *,
                                                         const int32_t *, const int32_t *, const double *,
                                                         const double *, const double *, const uint64_t *,
                                                         const int *, const double *, double, double *, double *,
                                                         unsigned *, int32_t *, unsigned *, double *, int64_t);

/* elements of one population's positions a k_bounds workgroup (4 waves) scans per pass:
 * the launch sizes its grid from this, so it follows the KB_CH build switch */
int gd_bounds_elems_per_block() { return 4 * 256 * KB_CH; }
