/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference's Cluster Separation Score window
 * scan (statistics/css/), the checker for the HIP CSS path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Restated literally, in the reference's evaluation order:
 *   compare_all (count metric) ..... css.c:277-327  ((int)x_i * x_j == -9)
 *   fill_averages .................. css.c:337-366
 *   cmds ........................... css.c:505-560  (Z B Z by two naive GEMMs)
 *   calc_dist ...................... css.c:573-587
 *   css ............................ css.c:608-647
 *   random_int_nrand48 / shuffle ... css.c:675-706
 *   significance_treshold .......... css.c:727-752
 *   window drivers ................. css.c:49-156, threadcss.c:52-293
 * Differences, all documented in DESIGN.md:
 *   - The eigen-decomposition (GSL 1.16 gsl_eigen_symmv, css.c:533-541) is
 *     replaced by a cyclic Jacobi solver: GSL is neither vendored nor installed,
 *     so the reference CSS C cannot be compiled here.  CSS depends only on the
 *     distances in X, which are invariant to eigenvector sign and to rotations
 *     within a degenerate top pair; solver differences are O(1e-14).
 *   - The permutation RNG state and the shuffled track array are reset per
 *     window ((seed, window) stream 1, identity tracks) instead of chaining
 *     across windows from a time() seed (threadcss.c:197-223, Q9).
 * Pinned by the known answers of testcss.c (test_compare_all, test_fill_averages,
 * test_calc_dist, test_cmds, test_css) in tests/test_oracle_css.py.
 */
#define _DEFAULT_SOURCE
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

void orc_css_compare_all(const double *av, const double *bv, int asize, int bsize, int npos, double *D) {
  int i, j, k, m = asize + bsize;
  for (i = 0; i < m; i++) D[i * m + i] = 0;
  for (i = asize; i--;)
    for (j = i; j--;) {
      double cnt = 0;
      for (k = npos; k--;)
        if (((int)av[k * asize + i] * av[k * asize + j]) == -9) cnt++;
      D[i * m + j] = cnt;
      D[j * m + i] = cnt;
    }
  for (i = bsize; i--;)
    for (j = i; j--;) {
      double cnt = 0;
      for (k = npos; k--;)
        if (((int)bv[k * bsize + i] * bv[k * bsize + j]) == -9) cnt++;
      D[(i + asize) * m + j + asize] = cnt;
      D[(j + asize) * m + i + asize] = cnt;
    }
  for (i = asize; i--;)
    for (j = bsize; j--;) {
      double cnt = 0;
      for (k = npos; k--;)
        if (((int)av[k * asize + i] * bv[k * bsize + j]) == -9) cnt++;
      D[i * m + j + asize] = cnt;
      D[(j + asize) * m + i] = cnt;
    }
}

int orc_css_fill_averages(double *D, int m) {
  int i, j, unval = 0, tot = m * m;
  double avg = 0;
  for (i = m; i--;)
    for (j = m; j--;) {
      if (D[i * m + j] < 0.00001)
        unval++;
      else
        avg += D[i * m + j];
    }
  avg = avg / tot;
  if (unval > tot / 2) return 0;
  for (i = m; i--;)
    for (j = m; j--;)
      if (D[i * m + j] < 0.00001) D[i * m + j] = avg;
  return 1;
}

/* cyclic Jacobi (the Numerical Recipes "jacobi" thresholds): A (m*m, destroyed)
 * -> eigenvalues w, eigenvectors in the columns of V.  Off-diagonal entries that
 * no longer change the diagonal in floating point are zeroed, so the sweep loop
 * ends with an exactly diagonal A (typically 6-10 sweeps). */
static void orc_jacobi(double *A, int m, double *w, double *V) {
  int i, j, k, p, sweep;
  for (i = 0; i < m; i++)
    for (j = 0; j < m; j++) V[i * m + j] = (i == j);
  for (sweep = 0; sweep < 100; sweep++) {
    double off = 0, thresh;
    for (p = 0; p < m - 1; p++)
      for (k = p + 1; k < m; k++) off += fabs(A[p * m + k]);
    if (off == 0.0) break;
    thresh = sweep < 3 ? 0.2 * off / (m * m) : 0.0;
    for (p = 0; p < m - 1; p++)
      for (k = p + 1; k < m; k++) {
        double apq = A[p * m + k], app, aqq, theta, t, c, s, g = 100.0 * fabs(apq);
        app = A[p * m + p];
        aqq = A[k * m + k];
        if (sweep > 3 && fabs(app) + g == fabs(app) && fabs(aqq) + g == fabs(aqq)) {
          A[p * m + k] = 0.0;
          A[k * m + p] = 0.0;
          continue;
        }
        if (fabs(apq) <= thresh || apq == 0.0) continue;
        theta = (aqq - app) / (2 * apq);
        t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
        c = 1 / sqrt(t * t + 1);
        s = t * c;
        for (i = 0; i < m; i++) {
          double aip = A[i * m + p], aiq = A[i * m + k];
          A[i * m + p] = c * aip - s * aiq;
          A[i * m + k] = s * aip + c * aiq;
        }
        for (i = 0; i < m; i++) {
          double api = A[p * m + i], aqi = A[k * m + i];
          A[p * m + i] = c * api - s * aqi;
          A[k * m + i] = s * api + c * aqi;
        }
        A[p * m + k] = 0.0;
        A[k * m + p] = 0.0;
        for (i = 0; i < m; i++) {
          double vip = V[i * m + p], viq = V[i * m + k];
          V[i * m + p] = c * vip - s * viq;
          V[i * m + k] = s * vip + c * viq;
        }
      }
  }
  for (i = 0; i < m; i++) w[i] = A[i * m + i];
}

/* classical MDS to 2 dimensions: D (m*m, read) -> X (m*2); eig2 (optional) gets the top-2 eigenvalues */
void orc_css_cmds(const double *D, int m, double *X, double *eig2) {
  double *B = malloc(sizeof(double) * m * m), *Z = malloc(sizeof(double) * m * m);
  double *T = malloc(sizeof(double) * m * m), *V = malloc(sizeof(double) * m * m), *w = malloc(sizeof(double) * m);
  int i, j, k, i0 = 0, i1 = 1;
  double L0, L1, zero_tol;
  for (i = 0; i < m * m; i++) B[i] = D[i] * D[i];
  for (i = m; i--;)
    for (j = m; j--;) Z[i * m + j] = (i != j) ? -1.0 / m : (m - 1) / (m * 1.0);
  for (i = 0; i < m; i++)
    for (j = 0; j < m; j++) {
      double acc = 0;
      for (k = 0; k < m; k++) acc += Z[i * m + k] * B[k * m + j];
      T[i * m + j] = acc;
    }
  for (i = 0; i < m; i++)
    for (j = 0; j < m; j++) {
      double acc = 0;
      for (k = 0; k < m; k++) acc += T[i * m + k] * Z[k * m + j];
      B[i * m + j] = acc;
    }
  for (i = m; i--;)
    for (j = m; j--;) B[i * m + j] *= -0.5;
  {
    /* eigenvalues within rounding of 0 are 0 (see below) */
    double fro = 0;
    for (i = 0; i < m * m; i++) fro += B[i] * B[i];
    zero_tol = 64.0 * m * DBL_EPSILON * sqrt(fro);
  }
  orc_jacobi(B, m, w, V);
  /* Documented deviation: B = -1/2 Z D2 Z always has the eigenvalue 0 (eigenvector
   * 1), so a window of rank <= 1 has lambda_2 = 0 exactly and the reference's
   * sqrt(lambda_2) is NaN or finite depending on the solver's rounding (GSL is not
   * available to pin it).  Both the oracle and the HIP kernel treat |lambda| <=
   * 64 m eps ||B||_F as 0, i.e. the finite outcome. */
  for (i = 0; i < m; i++)
    if (fabs(w[i]) <= zero_tol) w[i] = 0.0;
  /* the two largest eigenvalues, first occurrence on ties (a stable descending sort) */
  for (i = 0; i < m; i++)
    if (w[i] > w[i0]) i0 = i;
  i1 = (i0 == 0) ? 1 : 0;
  for (i = 0; i < m; i++)
    if (i != i0 && w[i] > w[i1]) i1 = i;
  if (eig2) {
    eig2[0] = w[i0];
    eig2[1] = w[i1];
  }
  L0 = sqrt(w[i0]);
  L1 = sqrt(w[i1]);
  for (i = 0; i < m; i++) {
    X[i * 2 + 0] = V[i * m + i0] * L0 + V[i * m + i1] * 0.0;
    X[i * 2 + 1] = V[i * m + i0] * 0.0 + V[i * m + i1] * L1;
  }
  free(B);
  free(Z);
  free(T);
  free(V);
  free(w);
}

void orc_css_dist(const double *X, int m, double *S) {
  int i, j;
  for (i = m; i--;) {
    S[i * m + i] = 0;
    for (j = i; j--;) {
      double ans = sqrt((X[i * 2] - X[j * 2]) * (X[i * 2] - X[j * 2]) +
                        (X[i * 2 + 1] - X[j * 2 + 1]) * (X[i * 2 + 1] - X[j * 2 + 1]));
      S[i * m + j] = ans;
      S[j * m + i] = ans;
    }
  }
}

double orc_css_score(const double *S, int m, const int *atr, const int *btr, int asize, int bsize) {
  int i, j;
  double bet = 0, ad = 0, bd = 0;
  for (i = asize; i--;)
    for (j = bsize; j--;) bet += S[atr[i] * m + btr[j]];
  bet = bet / (asize * bsize);
  if (asize > 1) {
    for (i = asize - 1; i--;) ad += S[atr[i] * m + atr[i + 1]];
    ad = ad / (asize * asize * (asize - 1));
  }
  if (bsize > 1) {
    for (i = bsize - 1; i--;) bd += S[btr[i] * m + btr[i + 1]];
    bd = bd / (bsize * bsize * (bsize - 1));
  }
  return bet - (asize + bsize) * (ad + bd);
}

static long orc_randint_css(long n, unsigned short st[3]) {
  long lim = 2147483647L - (2147483647L + 1) % n;
  long r = nrand48(st);
  while (r > lim) r = nrand48(st);
  return r % n;
}

double orc_css_significance(const double *S, int m, int *tracks, int asize, int bsize, double score, int treshold,
                            int runs, unsigned short st[3], int *nperm) {
  int hits = 0, nscores = 0;
  while (hits < treshold && nscores < runs) {
    int i;
    for (i = m - 1; i > 0; i--) {
      int r = (int)orc_randint_css(i + 1, st), t = tracks[i];
      tracks[i] = tracks[r];
      tracks[r] = t;
    }
    if (orc_css_score(S, m, tracks, tracks + asize, asize, bsize) >= score) hits++;
    nscores++;
  }
  if (nperm) *nperm = nscores;
  return (hits + 1) * 1.0 / (nscores + 1);
}

/* significance_treshold (css.c:727-752) of one window on given coordinates X (m x 2):
 * S = calc_dist(X), the observed score css() of the identity tracks, then the literal
 * shuffle / css() / hits loop with identity start tracks and the window's nrand48 state.
 * For the isolated permutation test (tests/test_css_perm_isolated.py), which feeds it the
 * device's own X: a permuted score within tie_rel * (|observed| + the observed score's
 * term magnitudes) of the observed one is a near tie, whose hit decision depends on the
 * summation order.  p_lo / p_hi resolve every near tie as a miss / as a hit (p is
 * monotone in the set of hits, so any consistent resolution lies in [p_lo, p_hi]);
 * *p is the literal `new >= score` decision; *nties counts the near ties seen before both
 * resolutions stopped. */
void orc_css_perm_from_x(const double *X, int asize, int bsize, int treshold, int runs, uint64_t state48,
                         double tie_rel, double *score, double *p, double *p_lo, double *p_hi, int *nties) {
  int m = asize + bsize, i, n;
  double *S = malloc(sizeof(double) * m * m);
  int *tracks = malloc(sizeof(int) * m), *atr = malloc(sizeof(int) * asize), *btr = malloc(sizeof(int) * bsize);
  int h_ex = 0, n_ex = 0, h_lo = 0, n_lo = 0, h_hi = 0, n_hi = 0, d_ex, d_lo, d_hi, ties = 0;
  unsigned short st[3];
  double sc, tol, bet = 0, ad = 0, bd = 0;
  orc_css_dist(X, m, S);
  for (i = 0; i < asize; i++) atr[i] = i;
  for (i = 0; i < bsize; i++) btr[i] = asize + i;
  sc = orc_css_score(S, m, atr, btr, asize, bsize);
  /* the magnitudes of the observed score's terms (every S entry is >= 0) */
  for (i = 0; i < asize; i++)
    for (n = 0; n < bsize; n++) bet += S[i * m + asize + n];
  for (i = 0; i + 1 < asize; i++) ad += S[i * m + i + 1];
  for (i = 0; i + 1 < bsize; i++) bd += S[(asize + i) * m + asize + i + 1];
  tol = tie_rel * (fabs(sc) + bet / (asize * bsize) +
                   (asize + bsize) * (asize > 1 ? ad / (asize * asize * (asize - 1.0)) : 0.0) +
                   (asize + bsize) * (bsize > 1 ? bd / (bsize * bsize * (bsize - 1.0)) : 0.0));
  for (i = 0; i < m; i++) tracks[i] = i;
  orc_state_words(state48, st);
  d_ex = d_lo = d_hi = !(treshold > 0 && runs > 0);
  for (n = 0; n < runs && !(d_ex && d_lo && d_hi); n++) {
    double v, diff;
    for (i = m - 1; i > 0; i--) {
      int r = (int)orc_randint_css(i + 1, st), t = tracks[i];
      tracks[i] = tracks[r];
      tracks[r] = t;
    }
    v = orc_css_score(S, m, tracks, tracks + asize, asize, bsize);
    diff = v - sc;
    if (fabs(diff) <= tol && !(d_lo && d_hi)) ties++;
    if (!d_ex) {
      h_ex += v >= sc;
      n_ex++;
      d_ex = h_ex >= treshold || n_ex >= runs;
    }
    if (!d_lo) {
      h_lo += diff > tol;
      n_lo++;
      d_lo = h_lo >= treshold || n_lo >= runs;
    }
    if (!d_hi) {
      h_hi += diff >= -tol;
      n_hi++;
      d_hi = h_hi >= treshold || n_hi >= runs;
    }
  }
  *score = sc;
  *p = (h_ex + 1) * 1.0 / (n_ex + 1);
  *p_lo = (h_lo + 1) * 1.0 / (n_lo + 1);
  *p_hi = (h_hi + 1) * 1.0 / (n_hi + 1);
  *nties = ties;
  free(S);
  free(tracks);
  free(atr);
  free(btr);
}

/* one window: returns 1 and fills score/p, or 0 when fill_averages discards it */
int orc_css_window(const double *av, const double *bv, int asize, int bsize, int npos, int treshold, int runs,
                   uint64_t state48, double *score, double *p, int *nperm) {
  int m = asize + bsize, i, ok;
  double *D = malloc(sizeof(double) * m * m), *S = malloc(sizeof(double) * m * m), *X = malloc(sizeof(double) * m * 2);
  int *tracks = malloc(sizeof(int) * m), *atr = malloc(sizeof(int) * asize), *btr = malloc(sizeof(int) * bsize);
  orc_css_compare_all(av, bv, asize, bsize, npos, D);
  ok = orc_css_fill_averages(D, m);
  if (ok) {
    double sc;
    unsigned short st[3];
    orc_css_cmds(D, m, X, NULL);
    orc_css_dist(X, m, S);
    for (i = 0; i < asize; i++) atr[i] = i;
    for (i = 0; i < bsize; i++) btr[i] = asize + i;
    sc = orc_css_score(S, m, atr, btr, asize, bsize);
    if (sc == -1) {
      ok = 0; /* the reference treats a score of exactly -1 as "discarded" (css.c:127) */
    } else {
      for (i = 0; i < m; i++) tracks[i] = i;
      orc_state_words(state48, st);
      *score = sc;
      *p = orc_css_significance(S, m, tracks, asize, bsize, sc, treshold, runs, st, nperm);
    }
  }
  free(D);
  free(S);
  free(X);
  free(tracks);
  free(atr);
  free(btr);
  return ok;
}

int orc_css_scan(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend, int wsize,
                 int wstep, int alen, int blen, int treshold, int runs, uint64_t seed, int serial, double *scores,
                 double *p) {
  int asize = orc_population_size(apos, alen), bsize = orc_population_size(bpos, blen);
  int wend = serial ? orc_serial_window_end(regend, wsize, wstep) : orc_threaded_window_end(regend, wsize, wstep);
  int w, la[2] = {0, 0}, lb[2] = {0, 0};
  if (alen <= 0 || blen <= 0) return 0;
  for (w = 0; w < wend; w++) {
    int start = w * wstep, stop = start + wsize, npos, l, r;
    l = la[0];
    r = la[1];
    while (l < alen && apos[l] < start) l++;
    while (r < alen && apos[r] <= stop) r++;
    la[0] = l;
    la[1] = r;
    l = lb[0];
    r = lb[1];
    while (l < blen && bpos[l] < start) l++;
    while (r < blen && bpos[r] <= stop) r++;
    lb[0] = l;
    lb[1] = r;
    npos = (la[1] - la[0]) / asize;
    if (npos <= 0) continue;
    if ((long)lb[0] + (long)npos * bsize > blen) return ORC_ERR_BOUNDS;
    {
      double sc, pv;
      if (orc_css_window(avals + la[0], bvals + lb[0], asize, bsize, npos, treshold, runs,
                         orc_window_state(seed, 1, w), &sc, &pv, NULL)) {
        scores[w] = sc;
        p[w] = pv;
      }
    }
  }
  return 0;
}

/* The reference's own permutation convention (Q9), for the statistical check of
 * deviation 1: css.c compute() (css.c:49-156) keeps ONE nrand48 state for the whole scan
 * (seeded from time(NULL) at css.c:111-114; here from state48) and ONE `signtracks`
 * array that every window's significance_treshold keeps shuffling (css.c:739), so each
 * window's permutations start from the previous window's last shuffle.  Window set and
 * scores as orc_css_scan (serial = compute(), else threadcompute()'s windows visited in
 * order, as one thread would). */
int orc_css_scan_chained(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                         int wsize, int wstep, int alen, int blen, int treshold, int runs, uint64_t state48,
                         int serial, double *scores, double *p) {
  int asize = orc_population_size(apos, alen), bsize = orc_population_size(bpos, blen);
  int wend = serial ? orc_serial_window_end(regend, wsize, wstep) : orc_threaded_window_end(regend, wsize, wstep);
  int w, i, m = asize + bsize, la[2] = {0, 0}, lb[2] = {0, 0};
  int *signtracks, *atr, *btr;
  double *D, *S, *X;
  unsigned short st[3];
  if (alen <= 0 || blen <= 0) return 0;
  signtracks = malloc(sizeof(int) * m);
  atr = malloc(sizeof(int) * asize);
  btr = malloc(sizeof(int) * bsize);
  D = malloc(sizeof(double) * m * m);
  S = malloc(sizeof(double) * m * m);
  X = malloc(sizeof(double) * m * 2);
  for (i = 0; i < m; i++) signtracks[i] = i;
  for (i = 0; i < asize; i++) atr[i] = i;
  for (i = 0; i < bsize; i++) btr[i] = asize + i;
  orc_state_words(state48, st);
  for (w = 0; w < wend; w++) {
    int start = w * wstep, stop = start + wsize, npos, l, r;
    l = la[0];
    r = la[1];
    while (l < alen && apos[l] < start) l++;
    while (r < alen && apos[r] <= stop) r++;
    la[0] = l;
    la[1] = r;
    l = lb[0];
    r = lb[1];
    while (l < blen && bpos[l] < start) l++;
    while (r < blen && bpos[r] <= stop) r++;
    lb[0] = l;
    lb[1] = r;
    npos = (la[1] - la[0]) / asize;
    if (npos <= 0) continue;
    if ((long)lb[0] + (long)npos * bsize > blen) {
      w = -1;
      break;
    }
    orc_css_compare_all(avals + la[0], bvals + lb[0], asize, bsize, npos, D);
    if (!orc_css_fill_averages(D, m)) continue;
    orc_css_cmds(D, m, X, NULL);
    orc_css_dist(X, m, S);
    {
      double sc = orc_css_score(S, m, atr, btr, asize, bsize);
      if (sc == -1) continue;
      scores[w] = sc;
      p[w] = orc_css_significance(S, m, signtracks, asize, bsize, sc, treshold, runs, st, NULL);
    }
  }
  free(signtracks);
  free(atr);
  free(btr);
  free(D);
  free(S);
  free(X);
  return w < 0 ? ORC_ERR_BOUNDS : 0;
}
