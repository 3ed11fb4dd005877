/* ORACLE -- TEST INFRASTRUCTURE ONLY (see fet_oracle.c / css_oracle.c headers). */
#ifndef GD_ORACLE_H
#define GD_ORACLE_H
#include <stdint.h>

#define ORC_NSAMPLES 100 /* bootstrap replicates, cFisher.c:62 / threadfisher.c:171 */
#define ORC_ERR_BOUNDS (-5)

int orc_population_size(const int *pos, int len);
int orc_threaded_window_end(int regend, int wsize, int wstep);
int orc_serial_window_end(int regend, int wsize, int wstep);
uint64_t orc_window_state(uint64_t seed, uint64_t stream, long w);
void orc_state_words(uint64_t x, unsigned short st[3]);

unsigned long orc_binomial(unsigned long n, unsigned long k);
double orc_fet_p(int a, int b, int c, int d);
int orc_set_fet_mode(int mode); /* 1: exact table probabilities (not in the reference) */
double orc_fet(int a, int b, int c, int d);
double orc_fet_score(int a, int b, int c, int d);
void orc_fet_counts(const double *av, const double *bv, int i, int asize, int bsize, int *f);
double orc_percentile(double *s, int n, double perc);
void orc_fet_window(const double *av, const double *bv, int asize, int bsize, int npos, double perc,
                    unsigned short st[3], double *fetscores, double *samples, double *out2);
int orc_fet_scan(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                 int wsize, int wstep, int alen, int blen, double perc, uint64_t seed, int serial,
                 double *scores, double *stddev);
void orc_nrand48_stream(uint64_t x0, int n, long *out);

/* CSS (css_oracle.c); matrices are dense row-major m*m */
void orc_css_compare_all(const double *av, const double *bv, int asize, int bsize, int npos, double *D);
int orc_css_fill_averages(double *D, int m);
void orc_css_cmds(const double *D, int m, double *X, double *eig2);
void orc_css_dist(const double *X, int m, double *S);
double orc_css_score(const double *S, int m, const int *atr, const int *btr, int asize, int bsize);
double orc_css_significance(const double *S, int m, int *tracks, int asize, int bsize, double score, int treshold,
                            int runs, unsigned short st[3], int *nperm);
void orc_css_perm_from_x(const double *X, int asize, int bsize, int treshold, int runs, uint64_t state48,
                         double tie_rel, double *score, double *p, double *p_lo, double *p_hi, int *nties);
int orc_css_window(const double *av, const double *bv, int asize, int bsize, int npos, int treshold, int runs,
                   uint64_t state48, double *score, double *p, int *nperm);
int orc_css_scan(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend, int wsize,
                 int wstep, int alen, int blen, int treshold, int runs, uint64_t seed, int serial, double *scores,
                 double *p);

int orc_css_scan_chained(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                         int wsize, int wstep, int alen, int blen, int treshold, int runs, uint64_t state48,
                         int serial, double *scores, double *p);

/* CSS options (css_options_oracle.c) */
void orc_css_compare_freq(const double *av, const double *bv, int npos, double *D);
double orc_css_stress(const double *delta, const double *D, int m);
double orc_css_smacof(const double *delta, int m, double *X, int max_iters, double epsilon, int *iters);
double orc_css_smacof_runs(const double *delta, int m, double *X, uint64_t state48);
int orc_css_window_ex(const double *av, const double *bv, int asize, int bsize, int npos, int treshold, int runs,
                      int drosophila, int mds, uint64_t perm48, uint64_t smacof48, double *score, double *p,
                      int *nperm);
int orc_css_scan_ex(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                    int wsize, int wstep, int alen, int blen, int treshold, int runs, int drosophila, int mds,
                    uint64_t seed, int serial, double *scores, double *p);

#endif
