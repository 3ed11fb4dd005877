/*
 * libgdscan_css.so -- the reference's CSS symbols with their exact C signatures
 * (statistics/css/threadcss.h:36-37, css.h:10-11) for the unmodified
 * css_cython_parallel.pyx / css_cython.pyx.  Failures go to stderr.
 */
#include <stdio.h>
#include "../../include/gdscan.h"

void threadcompute(double *avals, double *bvals, int *apos, int *bpos, int regstart, int regend, int wsize,
                   int wstep, int alen, int blen, int treshold, int runs, int drosophila, int mds, double *scores,
                   double *p) {
  int st = gd_css_threadcompute(avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, treshold,
                                runs, drosophila, mds, scores, p);
  if (st != GD_OK) fprintf(stderr, "gdscan: threadcompute (CSS) failed (%d): %s\n", st, gd_last_error());
}

void compute(double *avals, double *bvals, int *apos, int *bpos, int regstart, int regend, int wsize, int wstep,
             int alen, int blen, int treshold, int runs, int drosophila, int mds, double *scores, double *p) {
  int st = gd_css_compute(avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, treshold, runs,
                          drosophila, mds, scores, p);
  if (st != GD_OK) fprintf(stderr, "gdscan: compute (CSS) failed (%d): %s\n", st, gd_last_error());
}
