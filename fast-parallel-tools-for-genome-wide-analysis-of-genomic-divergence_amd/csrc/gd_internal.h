/*
 * gd_internal.h -- device-side descriptors shared by the kernels and the C-ABI glue.
 *
 * HBM layout of one scan (batch of chromosomes, all device-resident):
 *   avals/bvals  f64  [sum alen] / [sum blen]   genotype values, SNP-major (as the
 *   apos/bpos    i32  [sum alen] / [sum blen]   reference receives them), positions
 *                                               repeated once per individual
 *   lo_a/hi_a/lo_b i32 [sum wend]               window -> element index range
 *   snp_score    f64  [sum alen]                per-SNP -log10 p, row s of chromosome
 *                                               c at a_off(c) + s (rows <= alen)
 *   scores/stddev f64 [sum regend/wstep]        caller-owned outputs
 */
#pragma once
#include <stdint.h>

typedef struct gd_chrom_dev {
  int64_t a_off, b_off; /* element offsets into avals/apos and bvals/bpos */
  int64_t w_base;       /* first global window index of this chromosome */
  int64_t w_out;        /* output index of window 0 (scores/stddev/p) */
  int32_t alen, blen;
  int32_t regend, wend; /* windows [0, wend) are computed */
  int32_t asize, bsize; /* get_population_size(), filled on the device */
  int32_t nrows;        /* min(alen/asize, blen/bsize), filled on the device */
  int32_t w_first;      /* chromosome index of this descriptor's window 0 (window-range shards) */
  uint64_t seed;
} gd_chrom_dev;

/* status bits raised by kernels into one device word */
#define GD_FLAG_UNSORTED_A 1u
#define GD_FLAG_UNSORTED_B 2u
#define GD_FLAG_B_BOUNDS 4u
#define GD_FLAG_BAD_SIZE 8u

/* general-path window capacity held in LDS; larger windows use global scratch */
#define GD_GEN_LDS_N 1024
#define GD_MAX_GROUPS 32 /* chromosome groups pipelined across the scan's streams (capacity) */
#define GD_LUT_CAP (1 << 22) /* FET score-table entries (32 MB): up to ~62+62 individuals */
#define GD_NREP 100 /* bootstrap replicates (cFisher.c:62) */

/* CSS cohort sizes (m = asize + bsize): register tiers up to GD_CSS_TIER_MAX; the general
 * path (k_css_mds_big, k_css_perm_big, k_css_smacof_big) above, up to GD_CSS_BIG_MAX (SMACOF,
 * mds 1 / 2: up to GD_CSS_SMACOF_MAX, two individuals per thread above 1024), with each
 * workgroup's matrices in a global-memory slab of its own */
#define GD_CSS_TIER_MAX 128
#define GD_CSS_BIG_MAX 2048
#define GD_CSS_SMACOF_MAX 2048
/* doubles at the end of a 1024-tier slab for the inverse-iteration factors (LDS budget) */
#define GD_CSS_BIG_LU_DOUBLES (6 * 1024 + 2 * 1024 / 8 + 8)
/* the 2048 tier's: the factors, then its vectors that leave LDS (the 64-SNP compare masks,
 * the two eigenvector iterates and the multipliers / coordinates, 2 m each) */
#define GD_CSS_BIG_LU_DOUBLES_2K (6 * 2048 + 2 * 2048 / 8 + 8)
#define GD_CSS_BIG_GX_DOUBLES_2K (6 * 2048)
static inline int64_t gd_css_big_tail_doubles(int m) {
  return m > 1024 ? GD_CSS_BIG_LU_DOUBLES_2K + GD_CSS_BIG_GX_DOUBLES_2K : m > 512 ? GD_CSS_BIG_LU_DOUBLES : 0;
}
/* leading dimension (doubles) of a general-path matrix: m rounded up to 128-byte columns */
static inline int gd_css_big_ld(int m) { return (m + 15) & ~15; }
/* doubles of one workgroup's slab: the m x ld matrix of the MDS / permutation kernels or
 * SMACOF's 16-bit counts + packed stress triangle, whichever is larger, and the tier's tail */
static inline int64_t gd_css_big_slab_per_wg(int m) {
  const int64_t mds = (int64_t)gd_css_big_ld(m) * m;
  const int64_t sm = (int64_t)m * (m - 1) / 2 + 8 + ((int64_t)gd_css_big_ld(m) * m + 3) / 4 + 8;
  return (mds > sm ? mds : sm) + 32 + gd_css_big_tail_doubles(m);
}
/* Workgroups (= slabs) of the general-path kernels for a batch of wtotal windows and tier
 * mp: the device's resident capacity -- CUs x 4 workgroups of the 256-thread tier, x 2 of
 * the 512-thread tiers (512 and 1024 individuals) -- so every slab belongs to a running workgroup and the workgroups
 * loop over windows (gd_api.hip).  GD_CSS_BIG_GRID=<n> overrides it (diagnostics: the
 * tests force several windows per workgroup with it). */
int64_t gd_css_big_grid(int64_t wtotal, int mp);

/* CSS bit planes of one chromosome (word offsets into the plane buffer).  Pop A:
 * individual i's "== 3" plane at pa + 2i*wa, its "== -3" plane at pa + (2i+1)*wa,
 * the per-row "irregular value" plane at pa + 2*asize*wa; pop B likewise.  A plane
 * holds one bit per SNP row plus 3 zero words of padding. */
typedef struct gd_css_planes {
  int64_t pa, pb;
  int32_t wa, wb;
} gd_css_planes;
