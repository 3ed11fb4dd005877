/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin driver linked against the reference's own, unmodified FET sources
 * (/root/reference/statistics/fisher/{cFisher.c,comparative.c,threadfisher.c},
 * compiled in place by oracle/Makefile into oracle/_ref/libref_fisher.so).
 * The reference's threadcompute()/compute()/fet()/binomial()... are exported
 * by that library as-is; this file only adds a seeded scan so that the
 * bootstrap stddev becomes reproducible: it walks the windows of the threaded
 * driver (threadfisher.c:191-239) and calls the reference's
 * fisher_exact_test() (cFisher.c:170-195) with a per-window nrand48 state.
 */
#include <stdint.h>
#include <math.h>
#include <stdlib.h>

#include "cFisher.h"
#include "comparative.h"

static uint64_t h_mix(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return z;
}

static int h_window_end(int regend, int wsize, int wstep, int serial) {
  int end = 0;
  long w;
  if (serial) {
    for (w = 0; w + wsize <= (long)regend + wstep; w += wstep) end++;
  } else {
    int num_tasks = (regend / wstep - 3) / 100, t;
    if (num_tasks <= 0) return 0;
    for (t = 0; t <= num_tasks; t++) {
      long stop = (long)(t + 1) * 100 * wstep + (wsize - wstep);
      if (stop >= regend) stop = (long)regend + wstep;
      for (w = (long)t * 100 * wstep; w + wsize <= stop; w += wstep)
        if (w / wstep + 1 > end) end = (int)(w / wstep) + 1;
    }
  }
  if (end > regend / wstep) end = regend / wstep;
  return end;
}

int ref_fet_scan_seeded(double *avals, double *bvals, int *apos, int *bpos, int regend, int wsize, int wstep,
                        int alen, int blen, double perc, uint64_t seed, int serial, double *scores,
                        double *stddev) {
  int asize = get_population_size(apos), bsize = get_population_size(bpos);
  int wend = h_window_end(regend, wsize, wstep, serial), w, cap = 0;
  int aidx[2] = {0, 0}, bidx[2] = {0, 0}, f[4], tmp[4];
  double res[2], stds[100], *fs = NULL, *sm = NULL;
  for (w = 0; w < wend; w++) {
    int npos;
    slide_right(aidx, apos, w * wstep, w * wstep + wsize, alen);
    slide_right(bidx, bpos, w * wstep, w * wstep + wsize, blen);
    npos = (aidx[1] - aidx[0]) / asize;
    if (npos <= 0) continue;
    if (npos > cap) {
      cap = npos;
      /* one spare slot: percentile() reads s[idx+1] when idx == n-1 */
      fs = (double *)realloc(fs, (cap + 1) * sizeof(double));
      sm = (double *)realloc(sm, (cap + 1) * sizeof(double));
    }
    fs[npos] = 0.0;
    sm[npos] = 0.0;
    {
      uint64_t x = h_mix(seed ^ h_mix(0 + 0x9E3779B97F4A7C15ULL * (uint64_t)(w + 1))) & 0xFFFFFFFFFFFFULL;
      unsigned short st[3] = {(unsigned short)(x & 0xFFFF), (unsigned short)((x >> 16) & 0xFFFF),
                              (unsigned short)(x >> 32)};
      fisher_exact_test(res, avals + aidx[0], bvals + bidx[0], asize, bsize, npos, f, tmp, sm, stds, 100, fs, st,
                        perc);
    }
    scores[w] = res[0];
    stddev[w] = res[1];
  }
  free(fs);
  free(sm);
  return 0;
}

/* -1.0 * log10(fet(table)) exactly as fisher_exact_test() computes a SNP's score (cFisher.c:182-183) */
double ref_fet_score(int a, int b, int c, int d) {
  int f[4] = {a, b, c, d}, tmp[4];
  return -1.0 * log10(fet(f, tmp));
}
