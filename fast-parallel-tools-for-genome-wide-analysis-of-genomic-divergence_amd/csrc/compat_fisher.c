/*
 * libgdscan_fisher.so -- the reference's FET symbols with their exact C
 * signatures (statistics/fisher/threadfisher.h:33-34, cFisher.h:11-12), so the
 * unmodified fisher_cython_parallel.pyx / fisher_cython.pyx link against the
 * MI355X implementation.  The reference returns void and exit()s on failure;
 * here a failure is reported on stderr and the outputs are left untouched.
 */
#include <stdio.h>
#include "../../include/gdscan.h"

void threadcompute(double *avals, double *bvals, int *apos, int *bpos, int regstart, int regend, int wsize,
                   int wstep, int alen, int blen, double perc, double *scores, double *stddev) {
  int st = gd_fet_threadcompute(avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, perc, scores,
                                stddev);
  if (st != GD_OK) fprintf(stderr, "gdscan: threadcompute (FET) failed (%d): %s\n", st, gd_last_error());
}

void compute(double *avals, double *bvals, int *apos, int *bpos, int regstart, int regend, int wsize, int wstep,
             int alen, int blen, double perc, double *scores, double *stddev) {
  int st = gd_fet_compute(avals, bvals, apos, bpos, regstart, regend, wsize, wstep, alen, blen, perc, scores,
                          stddev);
  if (st != GD_OK) fprintf(stderr, "gdscan: compute (FET) failed (%d): %s\n", st, gd_last_error());
}
