/* Host build of csrc/gd_common.h (the device kernels' scalar code) for CPU unit
 * tests: the same source, compiled by gcc with -ffp-contract=off. */
#include "gd_common.h"

static uint64_t shim_binom(int n, int k) { return gd_binomial_ref((uint64_t)(int64_t)n, (uint64_t)(int64_t)k); }
#define SHIM_BINOM(n, k) shim_binom((n), (k))
GD_DEFINE_FET(shim_fet_static, static, SHIM_BINOM)

double shim_fet(int a, int b, int c, int d) { return shim_fet_static(a, b, c, d); }
double shim_log10(double x) { return gd_log10_glibc(x); }
double shim_score(int a, int b, int c, int d) { return gd_fet_score_from_p(shim_fet_static(a, b, c, d)); }
uint64_t shim_binomial(uint64_t n, uint64_t k) { return gd_binomial_ref(n, k); }
uint64_t shim_window_state(uint64_t seed, uint64_t stream, int64_t w) { return gd_window_state(seed, stream, w); }
uint64_t shim_jump(uint64_t x, uint64_t k) { return gd_affine_apply(gd_lcg_jump(k), x); }
void shim_stream(uint64_t x, int n, uint32_t *out) {
  for (int i = 0; i < n; ++i) {
    x = gd_lcg_next(x);
    out[i] = gd_lcg_value(x);
  }
}
uint32_t shim_limit(uint32_t n) { return gd_randint_make(n).limit; }
/* r mod n through the magic-number path for every r in rs */
void shim_mod(uint32_t n, const uint32_t *rs, int cnt, uint32_t *out) {
  const gd_randint d = gd_randint_make(n);
  for (int i = 0; i < cnt; ++i) out[i] = gd_randint_mod(&d, rs[i]);
}
int shim_pair_index(int maj, int mnr, int size) { return gd_pair_index(maj, mnr, size); }

/* exact mode: gd_fet_table_p_exact over a host ln k! table */
static double shim_lf[2][GD_BINOM_NMAX + 1];
static int shim_lf_ready;
static void shim_lf_init(void) {
  if (shim_lf_ready) return;
  for (int k = 0; k <= GD_BINOM_NMAX; ++k) {
    const long double L = lgammal((long double)k + 1.0L);
    shim_lf[0][k] = (double)L;
    shim_lf[1][k] = (double)(L - (long double)shim_lf[0][k]);
  }
  shim_lf_ready = 1;
}
#define SHIM_EXACT_P(B, a, b, c, d) gd_fet_table_p_exact(shim_lf[0], shim_lf[1], (a), (b), (c), (d))
GD_DEFINE_FET_P(shim_fet_exact_static, static, 0, SHIM_EXACT_P, GD_FET_EXACT_TIE)
double shim_fet_p_exact(int a, int b, int c, int d) {
  shim_lf_init();
  return gd_fet_table_p_exact(shim_lf[0], shim_lf[1], a, b, c, d);
}
double shim_fet_exact(int a, int b, int c, int d) {
  shim_lf_init();
  return shim_fet_exact_static(a, b, c, d);
}
double shim_score_exact(int a, int b, int c, int d) {
  shim_lf_init();
  return gd_fet_score_from_p(shim_fet_exact_static(a, b, c, d));
}
