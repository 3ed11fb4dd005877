/*
 * gd_common.h -- scalar building blocks of the genomic-divergence window scan,
 * shared by the HIP kernels (device) and the host-side unit tests (gcc build).
 *
 * Everything here is pure integer or IEEE-754 basic arithmetic (+ - * / sqrt),
 * compiled with -ffp-contract=off, so a value computed on the GPU is bit-identical
 * to the same expression on the host.  The one transcendental, log10, is rebuilt
 * from glibc's published formula (see gd_log10_glibc) over a correctly rounded
 * natural log, because the reference links glibc's log10 (cFisher.c:183).
 *
 * Reference semantics restated here (file:line in /root/reference):
 *   nrand48 LCG + rejection sampling ... statistics/fisher/cFisher.c:547-554,
 *                                        statistics/css/css.c:675-690
 *   binomial() with its overflow guard  statistics/fisher/cFisher.c:245-284
 *   fet_p()                              statistics/fisher/cFisher.c:473-483
 *   shift_table()/min_idx()/swap()       statistics/fisher/cFisher.c:292-346
 *   create_table()                       statistics/fisher/cFisher.c:357-390
 *   fet() (Feldman-Klinger / Zar tails)  statistics/fisher/cFisher.c:405-455
 *   percentile() index/interpolation     statistics/fisher/cFisher.c:136-144
 *   std()/mean() summation order         statistics/fisher/cFisher.c:492-518
 */
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GD_HD __host__ __device__ __forceinline__
#define GD_DEV __device__ __forceinline__
#define GD_CTABLE __device__ __constant__
#else
#include <math.h>
#define GD_HD static inline
#define GD_DEV static inline
#define GD_CTABLE static const
#endif

#include "gd_logtab.h"

/* ------------------------------------------------------------------------- */
/* glibc nrand48: x' = (a x + c) mod 2^48, value = x' >> 17 (31 bits)         */
/* ------------------------------------------------------------------------- */
#define GD_LCG_A 0x5DEECE66DULL
#define GD_LCG_C 0xBULL
#define GD_MASK48 0xFFFFFFFFFFFFULL
#define GD_RAND_MAX 0x7FFFFFFFU

GD_HD uint64_t gd_lcg_next(uint64_t x) { return (x * GD_LCG_A + GD_LCG_C) & GD_MASK48; }
GD_HD uint32_t gd_lcg_value(uint64_t x) { return (uint32_t)(x >> 17); }

/* An affine map x -> (mul * x + add) mod 2^48; k LCG steps are one such map. */
typedef struct { uint64_t mul, add; } gd_affine;

/* outer o applied after inner i */
GD_HD gd_affine gd_affine_then(gd_affine i, gd_affine o) {
  gd_affine r;
  r.mul = (o.mul * i.mul) & GD_MASK48;
  r.add = (o.mul * i.add + o.add) & GD_MASK48;
  return r;
}

/* map of k consecutive LCG steps (binary powering) */
GD_HD gd_affine gd_lcg_jump(uint64_t k) {
  gd_affine acc = {1, 0};
  gd_affine sq = {GD_LCG_A, GD_LCG_C};
  while (k) {
    if (k & 1) acc = gd_affine_then(acc, sq);
    sq = gd_affine_then(sq, sq);
    k >>= 1;
  }
  return acc;
}

GD_HD uint64_t gd_affine_apply(gd_affine f, uint64_t x) { return (f.mul * x + f.add) & GD_MASK48; }

/* ------------------------------------------------------------------------- */
/* Seeding convention (ours; the reference seeds from time(), cFisher.c:77-79, */
/* threadfisher.c:186-188, threadcss.c:221-223, so its stddev/p are not        */
/* reproducible).  Every window gets its own 48-bit nrand48 state:             */
/*   x0(seed, stream, w) = mix64(seed ^ mix64(stream + PHI*(w+1))) mod 2^48     */
/* stream 0 = FET bootstrap, stream 1 = CSS permutations, stream 2 = SMACOF   */
/* starts.  The state words an nrand48 caller would hold are                  */
/* {x0 & 0xffff, (x0>>16) & 0xffff, x0 >> 32}.                                */
/* ------------------------------------------------------------------------- */
#define GD_STREAM_FET 0ULL
#define GD_STREAM_CSS 1ULL
#define GD_STREAM_SMACOF 2ULL /* drand48 starts of smacof_runs (css.c:818-821) */

GD_HD uint64_t gd_mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return z;
}

GD_HD uint64_t gd_window_state(uint64_t seed, uint64_t stream, int64_t w) {
  return gd_mix64(seed ^ gd_mix64(stream + 0x9E3779B97F4A7C15ULL * (uint64_t)(w + 1))) & GD_MASK48;
}

/* random_int_nrand48(n): draws r until r <= limit, returns r % n.             */
/* The modulo is done by a multiply-high with a per-n magic number:            */
/* for r < 2^31 and l = ceil(log2 n), m = ceil(2^(31+l) / n) < 2^32 gives       */
/* floor(r / n) = (r * m) >> (31 + l) exactly (Granlund-Montgomery, N = 31).   */
typedef struct {
  uint32_t n;      /* divisor, >= 1 */
  uint32_t limit;  /* largest accepted raw value */
  uint32_t magic;
  uint32_t shift;  /* = 31 + l - 32 = l - 1 applied after the high word; n==1 special */
} gd_randint;

GD_HD gd_randint gd_randint_make(uint32_t n) {
  gd_randint d;
  d.n = n;
  d.limit = GD_RAND_MAX - (uint32_t)((0x80000000ULL) % n);
  uint32_t l = 0;
  while ((1ULL << l) < n) ++l;
  if (l == 0) {
    d.magic = 0;
    d.shift = 0;
  } else {
    uint64_t p = 1ULL << (31 + l);
    d.magic = (uint32_t)((p + n - 1) / n);
    d.shift = l - 1;
  }
  return d;
}

/* branch-free: for n == 1 the magic is 0 (q = 0) and the result is masked to 0 */
GD_HD uint32_t gd_randint_mod(const gd_randint *d, uint32_t r) {
  const uint32_t q = (uint32_t)(((uint64_t)r * d->magic) >> 32) >> d->shift;
  return (r - q * d->n) & (d->n == 1 ? 0u : 0xFFFFFFFFu);
}

/* ------------------------------------------------------------------------- */
/* binomial(n, k) exactly as the reference computes it: u64 multiplicative    */
/* formula with a gcd reduction, returning 0 on "unavoidable overflow".       */
/* The first such 0 is C(68, 31).                                              */
/* ------------------------------------------------------------------------- */
GD_HD uint64_t gd_gcd_u64(uint64_t x, uint64_t y) {
  if (y < x) {
    uint64_t t = x;
    x = y;
    y = t;
  }
  while (y > 0) {
    uint64_t t = y;
    y = x % y;
    x = t;
  }
  return x;
}

GD_HD uint64_t gd_binomial_ref(uint64_t n, uint64_t k) {
  if (k == 0 || k == n) return 1;
  if (k == 1) return n;
  if (k > n) return 0;
  if (k > n / 2) k = n - k;
  uint64_t acc = 1;
  for (uint64_t i = 1; i <= k; ++i, --n) {
    if (acc >= UINT64_MAX / n) {
      uint64_t g = gd_gcd_u64(n, i);
      uint64_t num = n / g, den = i / g;
      g = gd_gcd_u64(acc, den);
      acc /= g;
      den /= g;
      if (acc >= UINT64_MAX / num) return 0;
      acc = acc * num / den;
    } else {
      acc = acc * n / i;
    }
  }
  return acc;
}

/* index of the count pair (maj, min), maj + min <= size, in row-major triangular order */
GD_HD int gd_pair_index(int maj, int mnr, int size) { return maj * (size + 1) - maj * (maj - 1) / 2 + mnr; }

/* Triangular table of gd_binomial_ref(n, k) for 0 <= k <= n <= GD_BINOM_NMAX. */
#define GD_BINOM_NMAX 255
GD_HD int gd_binom_index(int n, int k) { return n * (n + 1) / 2 + k; }
#define GD_BINOM_ENTRIES ((GD_BINOM_NMAX + 1) * (GD_BINOM_NMAX + 2) / 2)

/* ------------------------------------------------------------------------- */
/* Two-tailed Fisher exact test, Feldman-Klinger / Zar shortcut (NOT the      */
/* textbook two-sided sum; differs from scipy on ~4-5% of tables).            */
/* Table layout f = {a, b, c, d} = {majA, minA, majB, minB}.                   */
/* ------------------------------------------------------------------------- */

/* Re-orient the table so that its smallest cell is a: walk the cells         */
/* clockwise (a, b, d, c) from the first minimum, then write back row-major.  */
GD_HD void gd_table_min_to_a(int *f) {
  const int ring[4] = {f[0], f[1], f[3], f[2]};
  int s = 0;
  for (int i = 1; i < 4; ++i)
    if (ring[i] < ring[s]) s = i;
  const int r0 = ring[s], r1 = ring[(s + 1) & 3], r2 = ring[(s + 2) & 3], r3 = ring[(s + 3) & 3];
  f[0] = r0;
  f[1] = r1;
  f[2] = r3;
  f[3] = r2;
}

/* Jump to the most extreme table of the opposite tail (same margins). */
GD_HD void gd_table_opposite_extreme(int *f) {
  const int R1 = f[0] + f[1], R2 = f[2] + f[3], C1 = f[0] + f[2], C2 = f[1] + f[3];
  int m = R1;
  if (R2 < m) m = R2;
  if (C1 < m) m = C1;
  if (C2 < m) m = C2;
  if (R1 <= R2 && C1 <= C2) {
    f[0] = m - f[0];
    f[1] = R1 - f[0];
    f[2] = C1 - f[0];
    f[3] = C2 - f[1];
  } else if (R1 <= R2 && C2 <= C1) {
    f[1] = m - f[1];
    f[0] = R1 - f[1];
    f[3] = C2 - f[1];
    f[2] = C1 - f[0];
  } else if (R1 >= R2 && C1 <= C2) {
    f[2] = m - f[2];
    f[0] = C1 - f[2];
    f[3] = R2 - f[2];
    f[1] = R1 - f[0];
  } else {
    f[3] = m - f[3];
    f[1] = C2 - f[3];
    f[2] = R2 - f[3];
    f[0] = R1 - f[1];
  }
}

/* Hypergeometric probability of one table: C(a+b,a) C(c+d,c) / C(n,a+c).   */
/* The numerator product wraps mod 2^64 exactly like the reference's          */
/* unsigned long arithmetic.  BINOM(n,k) is a callable returning uint64_t.    */
#define GD_FET_TABLE_P(BINOM, a, b, c, d)                                        \
  ((double)((uint64_t)BINOM((a) + (b), (a)) * (uint64_t)BINOM((c) + (d), (c))) / \
   (double)BINOM((a) + (b) + (c) + (d), (a) + (c)))

#define GD_DEFINE_FET(NAME, QUAL, BINOM) GD_DEFINE_FET_P(NAME, QUAL, BINOM, GD_FET_TABLE_P, 0.0)
/* TABLEP(BINOM, a, b, c, d): probability of one table (GD_FET_TABLE_P or an exact form);
 * TIE: relative tie tolerance of the far tail (0 reproduces the reference) */
#define GD_DEFINE_FET_P(NAME, QUAL, BINOM, TABLEP, TIE)                                     \
  QUAL double NAME(int a, int b, int c, int d) {                             \
    const int tie = (a + b == c + d) || (a + c == b + d);                    \
    int f[4] = {a, b, c, d};                                                 \
    gd_table_min_to_a(f);                                                    \
    const double p0 = TABLEP(BINOM, f[0], f[1], f[2], f[3]);                  \
    double tot = p0, step = p0;                                              \
    while (f[0] > 0) {                                                       \
      f[1]++;                                                                \
      f[2]++;                                                                \
      step = (1.0 * f[0] * f[3]) / (double)(f[1] * f[2]) * step;             \
      tot += step;                                                           \
      f[0]--;                                                                \
      f[3]--;                                                                \
    }                                                                        \
    if (tie) {                                                               \
      tot = 2 * tot;                                                         \
    } else {                                                                 \
      gd_table_opposite_extreme(f);                                          \
      gd_table_min_to_a(f);                                                  \
      double far = TABLEP(BINOM, f[0], f[1], f[2], f[3]);                     \
      while (far < p0 * (1.0 - (TIE))) {                                                     \
        tot += far;                                                          \
        if (f[1] == 0 || f[2] == 0) break;                                   \
        f[0]++;                                                              \
        f[3]++;                                                              \
        far = (1.0 * f[1] * f[2]) / (double)(f[0] * f[3]) * far;             \
        f[1]--;                                                              \
        f[2]--;                                                              \
      }                                                                      \
    }                                                                        \
    if (tot > 1) tot = 1;                                                    \
    return tot;                                                              \
  }

/* ------------------------------------------------------------------------- */
/* log10 as glibc 2.35 computes it (fdlibm e_log10.c formula):               */
/*   x = 2^k * m, i = (k < 0), y = k + i, m scaled into [1,2) or [0.5,1)      */
/*   log10(x) = (y*log10_2lo + ivln10*log(m)) + y*log10_2hi                   */
/* with log(m) correctly rounded (glibc's own log is within 0.52 ulp, so the  */
/* two agree on all but ~0.1% of arguments, by at most one ulp).              */
/* ------------------------------------------------------------------------- */
GD_HD uint64_t gd_f64_bits(double x) {
  union { double d; uint64_t u; } v;
  v.d = x;
  return v.u;
}
GD_HD double gd_f64_from(uint64_t u) {
  union { double d; uint64_t u; } v;
  v.u = u;
  return v.d;
}

typedef struct { double hi, lo; } gd_dd;

GD_HD gd_dd gd_dd_add(gd_dd a, gd_dd b) {
  double s = a.hi + b.hi;
  double v = s - a.hi;
  double e = (a.hi - (s - v)) + (b.hi - v);
  e += a.lo + b.lo;
  gd_dd r;
  r.hi = s + e;
  r.lo = e - (r.hi - s);
  return r;
}

/* natural log, correctly rounded in all but ~2^-15 of cases, for m in [0.5, 2) */
GD_DEV double gd_log_reduced(double m) {
  double e = 0.0;
  if (m < 1.0) {
    m = m * 2.0;
    e = -1.0;
  }
  const int j = (int)((m - 1.0) * 128.0 + 0.5);
  const double c = 1.0 + (double)j * (1.0 / 128.0);
  const double d = m - c; /* exact: same binade, |d| <= 2^-8 */
  const double rh = d / c;
  const double rl = fma(-rh, c, d) / c;
  /* r^2 / 2 as a double-double */
  const double sq = rh * rh;
  const double sqe = fma(rh, rh, -sq) + 2.0 * rh * rl;
  /* r^3 (1/3 - r/4 + r^2/5 - ...) in plain double: |r| <= 2^-8 */
  double t = 1.0 / 11.0;
  t = 1.0 / 10.0 - rh * t;
  t = 1.0 / 9.0 - rh * t;
  t = 1.0 / 8.0 - rh * t;
  t = 1.0 / 7.0 - rh * t;
  t = 1.0 / 6.0 - rh * t;
  t = 1.0 / 5.0 - rh * t;
  t = 1.0 / 4.0 - rh * t;
  t = 1.0 / 3.0 - rh * t;
  const double tail = sq * rh * t;
  gd_dd base = {e * GD_LN2_HI, e * GD_LN2_LO};
  gd_dd lc = {GD_LOGTAB[j][0], GD_LOGTAB[j][1]};
  gd_dd acc = gd_dd_add(base, lc);
  gd_dd r = {rh, rl};
  gd_dd hs = {-0.5 * sq, -0.5 * sqe};
  gd_dd poly = gd_dd_add(r, hs);
  poly.lo += tail;
  acc = gd_dd_add(acc, poly);
  return acc.hi + acc.lo;
}

GD_DEV double gd_log10_glibc(double x) {
  const double two54 = 1.80143985094819840000e+16;
  const double ivln10 = 4.34294481903251816668e-01;
  const double log10_2hi = 3.01029995663611771306e-01;
  const double log10_2lo = 3.69423907715893078616e-13;
  uint64_t u = gd_f64_bits(x);
  int32_t hx = (int32_t)(u >> 32);
  uint32_t lx = (uint32_t)u;
  int32_t k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | lx) == 0) return -__builtin_inf(); /* log(+-0) = -inf */
    if (hx < 0) return __builtin_nan("");                       /* log(-x) = NaN */
    k -= 54;
    x *= two54;
    u = gd_f64_bits(x);
    hx = (int32_t)(u >> 32);
    lx = (uint32_t)u;
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  const int32_t i = (int32_t)(((uint32_t)k & 0x80000000U) >> 31);
  hx = (hx & 0x000fffff) | ((0x3ff - i) << 20);
  const double y = (double)(k + i);
  x = gd_f64_from(((uint64_t)(uint32_t)hx << 32) | lx);
  const double z = y * log10_2lo + ivln10 * gd_log_reduced(x);
  return z + y * log10_2hi;
}

/* ------------------------------------------------------------------------- */
/* FET table-probability modes.  The kernels receive one table buffer:        */
/*   [0, GD_BINOM_ENTRIES)        binomial(n, k) as the reference computes it   */
/*   [GD_FET_MODE_WORD]           0 = reference, 1 = exact                      */
/*   [GD_FET_LF_OFF, +2*256)      ln k!, k <= 255, as double-double (hi, lo)    */
/* Reference mode: fet_p = C(a+b,a) C(c+d,c) / C(n,a+c) in u64 (cFisher.c:     */
/* 473-483), wrapping / 0 where the reference's unsigned long overflows (first */
/* at C(68,31)).  Exact mode: the same tail algorithm  */
/* over P = exp(sum of +-ln k!) with the sum in double-double: finite and      */
/* accurate to ~1e-13 relative for every table the u64 path overflows on.      */
/* ------------------------------------------------------------------------- */
#define GD_FET_MODE_WORD GD_BINOM_ENTRIES
#define GD_FET_LF_OFF (GD_BINOM_ENTRIES + 1)
#define GD_FET_TAB_WORDS (GD_BINOM_ENTRIES + 1 + 2 * (GD_BINOM_NMAX + 1))
/* Exact mode counts a far-tail table whose probability lies within this relative distance
 * of the observed table's as a tie and stops there, as the reference's `far < p0` does on
 * its exactly rounded u64 quotients; otherwise the rounding of the ln k! sums would decide
 * ties (e.g. table (1, 6, 8, 6)). */
#define GD_FET_EXACT_TIE 1e-9

GD_HD gd_dd gd_dd_neg(gd_dd a) {
  gd_dd r;
  r.hi = -a.hi;
  r.lo = -a.lo;
  return r;
}

/* C(a+b, a) C(c+d, c) / C(n, a+c) from the ln k! table (lf_hi / lf_lo, k <= 255) */
GD_DEV double gd_fet_table_p_exact(const double *lf_hi, const double *lf_lo, int a, int b, int c, int d) {
  const int n = a + b + c + d;
  gd_dd s = {0.0, 0.0};
  if (n <= GD_BINOM_NMAX) {
    const int pos[4] = {a + b, c + d, a + c, b + d};
    const int neg[5] = {a, b, c, d, n};
    for (int k = 0; k < 4; ++k) {
      const gd_dd t = {lf_hi[pos[k]], lf_lo[pos[k]]};
      s = gd_dd_add(s, t);
    }
    for (int k = 0; k < 5; ++k) {
      const gd_dd t = {lf_hi[neg[k]], lf_lo[neg[k]]};
      s = gd_dd_add(s, gd_dd_neg(t));
    }
  } else {
    s.hi = lgamma(a + b + 1.0) + lgamma(c + d + 1.0) + lgamma(a + c + 1.0) + lgamma(b + d + 1.0) -
           lgamma(a + 1.0) - lgamma(b + 1.0) - lgamma(c + 1.0) - lgamma(d + 1.0) - lgamma(n + 1.0);
  }
  return exp(s.hi) * (1.0 + s.lo);
}

/* per-SNP score: -1.0 * log10(p)  (cFisher.c:183) */
GD_DEV double gd_fet_score_from_p(double p) { return -1.0 * gd_log10_glibc(p); }

/* ------------------------------------------------------------------------- */
/* percentile(): idx = (int)((n-1)*perc), delta = (n-1)*perc - idx,          */
/* value = (1-delta)*s[idx] + delta*s[idx+1] over the ascending sort.          */
/* When idx == n-1 the reference reads s[n] (out of bounds) times delta == 0; */
/* we substitute s[n-1] for that operand.                                     */
/* ------------------------------------------------------------------------- */
GD_HD int gd_perc_index(int n, double perc) { return (int)((n - 1) * perc); }
GD_HD double gd_perc_delta(int n, double perc, int idx) { return (n - 1) * perc - idx; }
GD_HD double gd_perc_mix(double delta, double lo, double hi) { return (1 - delta) * lo + delta * hi; }

/* population std of n values, summed from the last element down (cFisher.c:492-518) */
#define GD_STD_REVERSE(OUT, ARR, N)                  \
  do {                                               \
    double gd_sum_ = 0;                              \
    for (int gd_i_ = (N); gd_i_--;) gd_sum_ += (ARR)[gd_i_]; \
    const double gd_mu_ = gd_sum_ / (N);             \
    double gd_ss_ = 0;                               \
    for (int gd_i_ = (N); gd_i_--;) {                \
      const double gd_d_ = (ARR)[gd_i_] - gd_mu_;    \
      gd_ss_ += gd_d_ * gd_d_;                       \
    }                                                \
    gd_ss_ /= (N);                                   \
    (OUT) = sqrt(gd_ss_);                            \
  } while (0)
