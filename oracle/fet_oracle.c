/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference's Fisher-exact-test window scan
 * (tuvakt/Fast-Parallel-Tools..., statistics/fisher/).  It is the checker for
 * the HIP product path: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product never links or calls it.
 *
 * Pinning: tests/test_oracle_fet.py checks every function here against the
 * reference's own C (compiled from /root/reference into oracle/_ref/ by
 * oracle/Makefile) and against the known answers of testFisher.c; the
 * committed fixtures in tests/golden/ were produced by the reference itself.
 *
 * The algorithm is restated literally, in the reference's own evaluation order,
 * so that results are bit-identical:
 *   get_population_size ......... comparative.c:25-34
 *   slide_right .................. comparative.c:49-71
 *   threaded window set .......... threadfisher.c:55-58, 106-116, 191-239
 *   serial window set ............ cFisher.c:59-99
 *   fisher_exact_test ............ cFisher.c:170-195
 *   fetcount ..................... cFisher.c:208-238
 *   binomial / gcd_ui ............ cFisher.c:245-284
 *   min_idx / shift_table ........ cFisher.c:292-346
 *   create_table ................. cFisher.c:357-390
 *   fet / fet_p .................. cFisher.c:405-483
 *   percentile (qsort) ........... cFisher.c:124-144
 *   bootstrap / calc_std / std ... cFisher.c:492-597
 * One deliberate difference: the bootstrap RNG state is re-seeded per window
 * from (seed, window index) -- see orc_window_state() -- instead of from
 * time(NULL) (cFisher.c:77-79, threadfisher.c:186-188).
 */
#define _DEFAULT_SOURCE
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---------------------------------------------------------------- windows */

int orc_population_size(const int *pos, int len) {
  int n = 1;
  if (len <= 0) return 0;
  while (n < len && pos[n] == pos[0]) n++;
  return n;
}

static void orc_slide(int *lr, const int *pos, int start, int stop, int len) {
  int l = lr[0], r = lr[1];
  while (l < len && pos[l] < start) l++;
  while (r < len && pos[r] <= stop) r++;
  lr[0] = l;
  lr[1] = r;
}

/* Windows computed by the reference's threaded driver: [0, *end).  Tasks of
 * 100 windows, num_tasks = (regend/wstep - 3)/100, tasks 0..num_tasks, the
 * task stop clamped to regend + wstep once it reaches regend; nothing at all
 * when num_tasks == 0.  Windows whose index falls outside regend/wstep (only
 * possible when wsize <= wstep, an out-of-bounds write in the reference) are
 * dropped. */
int orc_threaded_window_end(int regend, int wsize, int wstep) {
  int num_windows = regend / wstep - 3;
  int num_tasks = num_windows / 100;
  int end = 0, t;
  if (num_tasks <= 0) return 0;
  for (t = 0; t <= num_tasks; t++) {
    long start = (long)t * 100 * wstep;
    long stop = (long)(t + 1) * 100 * wstep + (wsize - wstep);
    long w;
    if (stop >= regend) stop = (long)regend + wstep;
    for (w = start; w + wsize <= stop; w += wstep) {
      int idx = (int)(w / wstep);
      if (idx + 1 > end) end = idx + 1;
    }
  }
  if (end > regend / wstep) end = regend / wstep;
  return end;
}

/* Windows computed by the serial compute(): start = 0, 1, 2 ... * wstep while
 * start + wsize <= regend + wstep (cFisher.c:81). */
int orc_serial_window_end(int regend, int wsize, int wstep) {
  long start = 0;
  int end = 0;
  while (start + wsize <= (long)regend + wstep) {
    end++;
    start += wstep;
  }
  if (end > regend / wstep) end = regend / wstep;
  return end;
}

uint64_t orc_window_state(uint64_t seed, uint64_t stream, long w) {
  uint64_t z = stream + 0x9E3779B97F4A7C15ULL * (uint64_t)(w + 1);
  uint64_t y;
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  y = seed ^ z;
  y ^= y >> 30;
  y *= 0xBF58476D1CE4E5B9ULL;
  y ^= y >> 27;
  y *= 0x94D049BB133111EBULL;
  y ^= y >> 31;
  return y & 0xFFFFFFFFFFFFULL;
}

void orc_state_words(uint64_t x, unsigned short st[3]) {
  st[0] = (unsigned short)(x & 0xFFFF);
  st[1] = (unsigned short)((x >> 16) & 0xFFFF);
  st[2] = (unsigned short)((x >> 32) & 0xFFFF);
}

/* --------------------------------------------------------------- FET math */

static unsigned long orc_gcd(unsigned long x, unsigned long y) {
  unsigned long t;
  if (y < x) {
    t = x;
    x = y;
    y = t;
  }
  while (y > 0) {
    t = y;
    y = x % y;
    x = t;
  }
  return x;
}

unsigned long orc_binomial(unsigned long n, unsigned long k) {
  unsigned long i, acc, g;
  if (k == 0 || k == n) return 1;
  if (k == 1) return n;
  if (k > n) return 0;
  if (k > n / 2) k = n - k;
  acc = 1;
  for (i = 1; i <= k; i++) {
    if (acc >= ULONG_MAX / n) {
      unsigned long nr, ir;
      g = orc_gcd(n, i);
      nr = n / g;
      ir = i / g;
      g = orc_gcd(acc, ir);
      acc = acc / g;
      ir = ir / g;
      if (acc >= ULONG_MAX / nr) return 0;
      acc *= nr;
      acc /= ir;
    } else {
      acc *= n;
      acc /= i;
    }
    n--;
  }
  return acc;
}

/* exact mode (not in the reference), the checker for
 * gd_fet_table_p_exact: the hypergeometric probability from ln k! in long double */
static int orc_fet_mode = 0;
int orc_set_fet_mode(int mode) {
  int old = orc_fet_mode;
  orc_fet_mode = mode;
  return old;
}

double orc_fet_p(int a, int b, int c, int d) {
  if (orc_fet_mode) {
    long double s = lgammal(a + b + 1.0L) + lgammal(c + d + 1.0L) + lgammal(a + c + 1.0L) + lgammal(b + d + 1.0L) -
                    lgammal(a + 1.0L) - lgammal(b + 1.0L) - lgammal(c + 1.0L) - lgammal(d + 1.0L) -
                    lgammal(a + b + c + d + 1.0L);
    return (double)expl(s);
  }
  double nom = orc_binomial(a + b, a) * orc_binomial(c + d, c);
  double den = orc_binomial(a + b + c + d, a + c);
  return nom / den;
}

static int orc_min_idx(const int *v, int n) {
  int i, m = 0;
  for (i = 1; i < n; i++)
    if (v[i] < v[m]) m = i;
  return m;
}

/* rotate the 2x2 table so the smallest cell lands in position a */
static void orc_shift(int *f) {
  int ring[4], out[4], i, s, t;
  ring[0] = f[0];
  ring[1] = f[1];
  ring[2] = f[3];
  ring[3] = f[2];
  s = orc_min_idx(ring, 4);
  for (i = 0; i < 4; i++) out[i] = ring[(s + i) % 4];
  t = out[2];
  out[2] = out[3];
  out[3] = t;
  memcpy(f, out, sizeof out);
}

static void orc_extreme(int *f) {
  int R1 = f[0] + f[1], R2 = f[2] + f[3], C1 = f[0] + f[2], C2 = f[1] + f[3];
  int m[4] = {R1, R2, C1, C2};
  int mn = m[orc_min_idx(m, 4)];
  if (R1 <= R2 && C1 <= C2) {
    f[0] = mn - f[0];
    f[1] = R1 - f[0];
    f[2] = C1 - f[0];
    f[3] = C2 - f[1];
  } else if (R1 <= R2 && C2 <= C1) {
    f[1] = mn - f[1];
    f[0] = R1 - f[1];
    f[3] = C2 - f[1];
    f[2] = C1 - f[0];
  } else if (R1 >= R2 && C1 <= C2) {
    f[2] = mn - f[2];
    f[0] = C1 - f[2];
    f[3] = R2 - f[2];
    f[1] = R1 - f[0];
  } else {
    f[3] = mn - f[3];
    f[1] = C2 - f[3];
    f[2] = R2 - f[3];
    f[0] = R1 - f[1];
  }
}

double orc_fet(int a, int b, int c, int d) {
  int f[4] = {a, b, c, d};
  int equal_margin = (a + b == c + d) || (a + c == b + d);
  double P, P0, P1, P2;
  orc_shift(f);
  P0 = orc_fet_p(f[0], f[1], f[2], f[3]);
  P = P1 = P0;
  while (f[0] > 0) {
    f[1]++;
    f[2]++;
    P1 = (1.0 * f[0] * f[3]) / (f[1] * f[2]) * P1;
    P += P1;
    f[0]--;
    f[3]--;
  }
  if (equal_margin) {
    P = 2 * P;
  } else {
    orc_extreme(f);
    orc_shift(f);
    P2 = orc_fet_p(f[0], f[1], f[2], f[3]);
    while (P2 < (orc_fet_mode ? P0 * (1.0 - 1e-9) : P0)) { /* exact mode: ties within 1e-9 */
      P += P2;
      if (f[1] == 0 || f[2] == 0) break;
      f[0]++;
      f[3]++;
      P2 = (1.0 * f[1] * f[2]) / (f[0] * f[3]) * P2;
      f[1]--;
      f[2]--;
    }
  }
  if (P > 1) P = 1;
  return P;
}

double orc_fet_score(int a, int b, int c, int d) { return -1.0 * log10(orc_fet(a, b, c, d)); }

/* counts of exact 3 / -3 for SNP i of a window slice */
void orc_fet_counts(const double *av, const double *bv, int i, int asize, int bsize, int *f) {
  int k;
  f[0] = f[1] = f[2] = f[3] = 0;
  for (k = i * asize; k < i * asize + asize; k++) {
    if (av[k] == 3)
      f[0]++;
    else if (av[k] == -3)
      f[1]++;
  }
  for (k = i * bsize; k < i * bsize + bsize; k++) {
    if (bv[k] == 3)
      f[2]++;
    else if (bv[k] == -3)
      f[3]++;
  }
}

static int orc_cmp(const void *x, const void *y) {
  double a = *(const double *)x, b = *(const double *)y;
  return (a > b) - (a < b);
}

/* sorts s in place; reads s[idx+1] only when it exists (see gd_common.h) */
double orc_percentile(double *s, int n, double perc) {
  int idx;
  double delta, hi;
  qsort(s, n, sizeof(double), orc_cmp);
  idx = (n - 1) * perc;
  delta = (n - 1) * perc - idx;
  hi = (idx + 1 < n) ? s[idx + 1] : s[idx];
  return (1 - delta) * s[idx] + delta * hi;
}

static long orc_randint(long n, unsigned short st[3]) {
  long lim = 2147483647L - (2147483647L + 1) % n;
  long r = nrand48(st);
  while (r > lim) r = nrand48(st);
  return r % n;
}

static double orc_std(const double *a, int n) {
  int i;
  double mu = 0, s = 0;
  for (i = n; i--;) mu += a[i];
  mu = mu / n;
  for (i = n; i--;) s += (a[i] - mu) * (a[i] - mu);
  s /= n;
  return sqrt(s);
}

/* one window: fetscores[npos] scratch, samples[npos] scratch */
void orc_fet_window(const double *av, const double *bv, int asize, int bsize, int npos, double perc,
                    unsigned short st[3], double *fetscores, double *samples, double *out2) {
  int i, r;
  double reps[ORC_NSAMPLES];
  for (i = npos; i--;) {
    int f[4];
    orc_fet_counts(av, bv, i, asize, bsize, f);
    fetscores[i] = -1.0 * log10(orc_fet(f[0], f[1], f[2], f[3]));
  }
  out2[0] = orc_percentile(fetscores, npos, perc);
  for (r = 0; r < ORC_NSAMPLES; r++) {
    for (i = npos; i--;) samples[i] = fetscores[orc_randint(npos, st)];
    reps[r] = orc_percentile(samples, npos, perc);
  }
  out2[1] = orc_std(reps, ORC_NSAMPLES);
}

int orc_fet_scan(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                 int wsize, int wstep, int alen, int blen, double perc, uint64_t seed, int serial,
                 double *scores, double *stddev) {
  int asize = orc_population_size(apos, alen), bsize = orc_population_size(bpos, blen);
  int wend = serial ? orc_serial_window_end(regend, wsize, wstep) : orc_threaded_window_end(regend, wsize, wstep);
  int w, cap = 0;
  double *fs = NULL, *sm = NULL;
  if (alen <= 0 || blen <= 0) return 0;
  int la[2] = {0, 0}, lb[2] = {0, 0};
  for (w = 0; w < wend; w++) {
    int npos;
    int start = w * wstep, stop = start + wsize;
    orc_slide(la, apos, start, stop, alen);
    orc_slide(lb, bpos, start, stop, blen);
    npos = (la[1] - la[0]) / asize;
    if (npos <= 0) continue;
    if ((long)lb[0] + (long)npos * bsize > blen) return ORC_ERR_BOUNDS;
    if (npos > cap) {
      cap = npos;
      fs = (double *)realloc(fs, cap * sizeof(double));
      sm = (double *)realloc(sm, cap * sizeof(double));
    }
    {
      unsigned short st[3];
      double out2[2];
      orc_state_words(orc_window_state(seed, 0, w), st);
      orc_fet_window(avals + la[0], bvals + lb[0], asize, bsize, npos, perc, st, fs, sm, out2);
      scores[w] = out2[0];
      stddev[w] = out2[1];
    }
  }
  free(fs);
  free(sm);
  return 0;
}

/* libc nrand48 stream, for checking the product's LCG */
void orc_nrand48_stream(uint64_t x0, int n, long *out) {
  unsigned short st[3];
  int i;
  orc_state_words(x0, st);
  for (i = 0; i < n; i++) out[i] = nrand48(st);
}
