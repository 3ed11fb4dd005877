/*
 * gdscan.h -- C ABI of the MI355X genomic-divergence window scanner (libgdscan.so).
 *
 * Drop-in boundary for the reference's hot path.  Each entry point names the
 * reference interface it replaces (paths relative to the reference tree):
 *
 *   gd_fet_threadcompute  <- threadcompute()   statistics/fisher/threadfisher.h:33-34
 *                            (bound by fisher_exact_tester, fisher_cython_parallel.pyx:14-15)
 *   gd_fet_compute        <- compute()         statistics/fisher/cFisher.h:11-12
 *                            (bound by fisher_exact_tester, fisher_cython.pyx:11-12)
 *   gd_css_threadcompute  <- threadcompute()   statistics/css/threadcss.h:36-37
 *                            (bound by cluster_separation_scorer, css_cython_parallel.pyx:14-15)
 *   gd_css_compute        <- compute()         statistics/css/css.h:10-11
 *
 * The reference symbols are void and exit() on failure; ours return a status
 * (GD_OK or a negative GD_ERR_*).  Buffers are caller-owned, plain host pointers,
 * read-only except the outputs, which are written ONLY at the indices of windows
 * the reference would compute (other entries keep the caller's values).  Calls are
 * reentrant and thread-safe (a mutex per device context).
 *
 * Reproducibility: the reference seeds its bootstrap / permutation RNG from
 * time(NULL); here every window w draws from its own nrand48 stream seeded by
 * (seed, w) (gd_set_seed, default GD_DEFAULT_SEED; the seed is per calling
 * thread, so concurrent callers do not share it), so stddev and p are
 * deterministic.  Scores do not depend on the seed.
 *
 * libgdscan_fisher.so / libgdscan_css.so additionally export the reference's own
 * names (threadcompute, compute) with the reference's exact signatures, so the
 * unmodified .pyx files link against them.
 */
#ifndef GDSCAN_H
#define GDSCAN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GD_OK 0
#define GD_ERR_ARG (-1)      /* invalid argument (wsize/wstep <= 0, perc outside [0,1], ...) */
#define GD_ERR_HIP (-2)      /* HIP runtime failure (no device, out of memory, launch error) */
#define GD_ERR_UNSORTED (-4) /* positions not non-decreasing (slide_right assumes sorted) */
#define GD_ERR_BOUNDS (-5)   /* a window's B slice runs past blen (reference: out-of-bounds read) */
#define GD_ERR_SIZE (-6)     /* empty population / unsupported window size */
#define GD_ERR_NOPACK (-7)   /* a readable track with no packed form (gd_ptrack_read; keeps the reference layout) */

#define GD_DEFAULT_SEED 20261015ULL

/* window set: which windows are computed */
#define GD_WINDOWS_THREADED 0 /* threadcompute(): 100-window tasks, none if regend/wstep < 103 */
#define GD_WINDOWS_SERIAL 1   /* compute(): every start with start + wsize <= regend + wstep */

/* ---- FET: Fisher's exact test score (95th percentile of -log10 p) + bootstrap std ---- */
int gd_fet_threadcompute(const double *avals, const double *bvals, const int *apos, const int *bpos, int regstart,
                         int regend, int wsize, int wstep, int alen, int blen, double perc, double *scores,
                         double *stddev);
int gd_fet_compute(const double *avals, const double *bvals, const int *apos, const int *bpos, int regstart,
                   int regend, int wsize, int wstep, int alen, int blen, double perc, double *scores,
                   double *stddev);
/* explicit seed and window set */
int gd_fet_scan_host(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                     int wsize, int wstep, int alen, int blen, double perc, uint64_t seed, int window_set,
                     double *scores, double *stddev);
/* FET table probabilities.  GD_FET_REFERENCE reproduces the
 * reference's u64 binomials (cFisher.c:245-284, 473-483), which wrap or overflow to 0 from
 * C(68, 31) on (tables of >= 68 individuals); GD_FET_EXACT runs the same two-tailed test
 * over hypergeometric probabilities from ln k! in double-double (~1e-13 relative). */
#define GD_FET_REFERENCE 0
#define GD_FET_EXACT 1
int gd_set_fet_mode(int mode); /* mode of every call without one; returns the previous mode */
int gd_get_fet_mode(void);
int gd_fet_scan_host_ex(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                        int wsize, int wstep, int alen, int blen, double perc, int mode, uint64_t seed,
                        int window_set, double *scores, double *stddev);

/* ---- CSS: cluster separation score (classical MDS) + Monte-Carlo p ---- */
int gd_css_threadcompute(const double *avals, const double *bvals, const int *apos, const int *bpos, int regstart,
                         int regend, int wsize, int wstep, int alen, int blen, int treshold, int runs,
                         int drosophila, int mds, double *scores, double *p);
int gd_css_compute(const double *avals, const double *bvals, const int *apos, const int *bpos, int regstart,
                   int regend, int wsize, int wstep, int alen, int blen, int treshold, int runs, int drosophila,
                   int mds, double *scores, double *p);
int gd_css_scan_host(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                     int wsize, int wstep, int alen, int blen, int treshold, int runs, uint64_t seed,
                     int window_set, double *scores, double *p);
/* with the reference's options (cluster_separation_scorer, css.c:181-223):
 *   drosophila 1: compare_freq (css.c:245-264), mean |a - b| of the two populations'
 *                 allele frequencies; needs asize = bsize = 1 (else GD_ERR_ARG: the
 *                 reference fills only D[0][1] and reads uninitialised memory)
 *   mds 0: classical MDS; 1: SMACOF from 4 drand48 starts (smacof_runs, css.c:807-835);
 *   2: classical MDS refined by one SMACOF run (css.c:211-213).  The SMACOF starts of
 *   window w come from drand48 stream (seed, w, 2) (the reference: time-seeded). */
int gd_css_scan_host_ex(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                        int wsize, int wstep, int alen, int blen, int treshold, int runs, int drosophila, int mds,
                        uint64_t seed, int window_set, double *scores, double *p);

/* diagnostics: gd_css_scan_host_ex (count metric, runs > 0 and treshold > 0, else GD_ERR_ARG)
 * that also returns the coordinates its permutation test read (the classical-MDS X of
 * css.c:545-556, or SMACOF's for mds 1 / 2): X (host) holds gd_window_count(...) rows of
 * 2 (asize + bsize) doubles, point i of window w at X[w * 2m + 2i], X[w * 2m + 2i + 1]; rows
 * of windows with scores[w] == 0 are unspecified.  Lets a test re-run significance_treshold
 * (css.c:727-752) on the device's own X, isolating the permutation kernel from the solver. */
int gd_css_coords_host(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                       int wsize, int wstep, int alen, int blen, int treshold, int runs, int mds, uint64_t seed,
                       int window_set, double *scores, double *p, double *X);

/* ---- device-resident batched scans (all pointers are device pointers except `chroms`) ---- */
typedef struct gd_chrom {
  int64_t a_off, b_off; /* element offsets of this chromosome in avals/apos and bvals/bpos */
  int32_t alen, blen;   /* element counts */
  int32_t regend;       /* region end (chromosome length); windows are [w*wstep, w*wstep+wsize] */
  int32_t w_first;      /* window-range shard: the first window (chromosome index) this descriptor
                           computes; 0 = the chromosome's start */
  int64_t w_out;        /* index in scores/stddev|p of window w_first */
  uint64_t seed;        /* RNG seed of this chromosome's bootstrap / permutations */
  int32_t w_count;      /* windows computed from w_first on (0 = to the end of the window set) */
  int32_t pad_;
} gd_chrom;
/* A window-range shard (gdscan.shard.plan_window_shards, the reference's 100-window task
 * with its SNP span, threadfisher.c:106-116, threadcss.c:114-124) is the chromosome's
 * arrays from the first element at position >= w_first * wstep to the last element a
 * window of the range reads, with the chromosome's regend and seed: its windows
 * w_first .. w_first + w_count - 1 of the chromosome's window set are computed, with the
 * chromosome's per-window seeds, and written at w_out + (w - w_first).  The slice must
 * start on a whole row (get_population_size reads the first run); outputs equal the
 * whole-chromosome scan's bit for bit.  Packed batches take w_first = w_count = 0. */

typedef struct gd_ctx gd_ctx;
gd_ctx *gd_ctx_create(int device); /* NULL on failure */
void gd_ctx_destroy(gd_ctx *ctx);

/* Number of windows of one chromosome a scan writes: [0, n).  Pure arithmetic. */
int gd_window_count(int regend, int wsize, int wstep, int window_set);

int gd_fet_scan_device(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                       const int32_t *apos, const int32_t *bpos, int wsize, int wstep, double perc,
                       int window_set, double *scores, double *stddev, void *hip_stream);
int gd_fet_scan_device_ex(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                          const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize, int wstep,
                          double perc, int mode, int window_set, double *scores, double *stddev, void *hip_stream);

int gd_css_scan_device(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                       const int32_t *apos, const int32_t *bpos, int wsize, int wstep, int treshold, int runs,
                       int window_set, double *scores, double *p, void *hip_stream);
int gd_css_scan_device_ex(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                          const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize, int wstep,
                          int treshold, int runs, int drosophila, int mds, int window_set, double *scores, double *p,
                          void *hip_stream);

/* the same batch from host memory (offsets into host arrays; outputs are caller-owned
 * host arrays holding every chromosome's w_out + regend/wstep windows) */
int gd_fet_scan_host_batch(const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                           const int *apos, const int *bpos, int wsize, int wstep, double perc, int window_set,
                           double *scores, double *stddev);
int gd_fet_scan_host_batch_ex(const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                              const int *apos, const int *bpos, int wsize, int wstep, double perc, int mode,
                              int window_set, double *scores, double *stddev);
int gd_css_scan_host_batch(const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                           const int *apos, const int *bpos, int wsize, int wstep, int treshold, int runs,
                           int window_set, double *scores, double *p);
int gd_css_scan_host_batch_ex(const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                              const int *apos, const int *bpos, int wsize, int wstep, int treshold, int runs,
                              int drosophila, int mds, int window_set, double *scores, double *p);

/* ---- packed genotype tracks (second half) ----
 * The four values VCFConvert.py:8-17 writes, as 2-bit codes; one position per SNP row
 * (the reference layout repeats it per individual).  Population P of a chromosome with
 * nrows rows is nrows x GD_PACK_WORDS(Psize) uint64 words: individual k of row r sits in
 * bits 2 (k mod 32) of word r * GD_PACK_WORDS(Psize) + k / 32; padding codes are 0.
 * A packed chromosome scans exactly like its expanded form (individual k of row r at
 * element r * size, both populations at the row's position): same windows, same
 * scores, same bootstrap / permutation streams. */
#define GD_PACK_WORDS(size) (((size) + 31) / 32)
#define GD_CODE_HET 0u     /* value 0 (heterozygous / other call) */
#define GD_CODE_MAJOR 1u   /* value 3 (homozygous major) */
#define GD_CODE_MINOR 2u   /* value -3 (homozygous minor) */
#define GD_CODE_MISSING 3u /* value -10000 (missing) */
typedef struct gd_pchrom {
  int64_t row_off;        /* first row of this chromosome in rowpos */
  int64_t a_word, b_word; /* first word of its rows in acodes / bcodes */
  int32_t nrows, asize, bsize;
  int32_t regend;         /* region end; windows are [w*wstep, w*wstep+wsize] */
  int64_t w_out;          /* index in scores/stddev|p of window 0 */
  uint64_t seed;
} gd_pchrom;
/* get_population_size() of both tracks (comparative.c:25-34) and the number of rows both
 * hold whole (min(alen / asize, blen / bsize)); host memory.  GD_ERR_ARG (outputs still
 * set) unless alen = nrows * asize and blen = nrows * bsize: a partial row or unequal row
 * counts have no packed form */
int gd_pack_shape(const int *apos, const int *bpos, int alen, int blen, int *asize, int *bsize, int *nrows);
/* packs nrows rows (host memory; outputs hold nrows * GD_PACK_WORDS(size) words and nrows
 * positions).  GD_ERR_ARG when a value is not one of the four codes or an individual's
 * position (A or B) differs from its row's (apos[r * asize]): such tracks keep the
 * reference layout (gd_*_scan_*). */
int gd_pack_chrom(const double *avals, const double *bvals, const int *apos, const int *bpos, int asize, int bsize,
                  int nrows, uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos);
/* the same on host threads (GD_HOST_THREADS, else the CPU affinity capped by OMP_NUM_THREADS and
 * 16): what the reference-signature host entry points use before anything crosses PCIe */
int gd_pack_chrom_mt(const double *avals, const double *bvals, const int *apos, const int *bpos, int asize,
                     int bsize, int nrows, uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos);
/* the same on the device (device pointers; a reference-layout track already in HBM) */
int gd_pack_chrom_device(const double *avals, const double *bvals, const int32_t *apos, const int32_t *bpos,
                         int asize, int bsize, int nrows, uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos,
                         void *hip_stream);
/* scans of packed batches: device pointers (except `chroms`) ... */
int gd_fet_scan_packed_device(gd_ctx *ctx, const gd_pchrom *chroms, int nchrom, const uint64_t *acodes,
                              const uint64_t *bcodes, const int32_t *rowpos, int wsize, int wstep, double perc,
                              int mode, int window_set, double *scores, double *stddev, void *hip_stream);
/* CSS: count metric only (drosophila = 0); mds 0 / 1 / 2 as gd_css_scan_host_ex */
int gd_css_scan_packed_device(gd_ctx *ctx, const gd_pchrom *chroms, int nchrom, const uint64_t *acodes,
                              const uint64_t *bcodes, const int32_t *rowpos, int wsize, int wstep, int treshold,
                              int runs, int mds, int window_set, double *scores, double *p, void *hip_stream);
/* ... and from host memory (the codes cross PCIe: 2 bits per genotype + 4 B per row) */
int gd_fet_scan_packed_host(const gd_pchrom *chroms, int nchrom, const uint64_t *acodes, const uint64_t *bcodes,
                            const int32_t *rowpos, int wsize, int wstep, double perc, int mode, int window_set,
                            double *scores, double *stddev);
int gd_css_scan_packed_host(const gd_pchrom *chroms, int nchrom, const uint64_t *acodes, const uint64_t *bcodes,
                            const int32_t *rowpos, int wsize, int wstep, int treshold, int runs, int mds,
                            int window_set, double *scores, double *p);

/* ---- region filters after the scan ----
 * A track is the list of windows a tool's tabular file holds (score != 0), in file
 * order.  Array arguments may be host or device memory; ctx NULL selects the process-wide
 * context of the current HIP device (hipGetDevice), hip_stream NULL the context's stream.
 * Blocking. */
#define GD_SELECT_GE 0 /* keep vals >= thr (FET scores, CSS top-k scores) */
#define GD_SELECT_LE 1 /* keep vals <= thr (CSS p-values) */
/* FilterFisherScores.py:84-87: out3 = {limit, cmedian(scores), scoreatpercentile(stddev,
 * percentile)}, limit = median + qnorm * upperquant; qnorm = norm.ppf(normquantile) is the
 * caller's (scipy.special.ndtri).  Non-finite scores: GD_ERR_ARG (numpy.histogram raises). */
int gd_fet_region_limit(gd_ctx *ctx, const double *scores, const double *stddev, int64_t n, double qnorm,
                        double percentile, double *out3, void *hip_stream);
/* SignificantCSSRegions.py:102-120: Benjamini-Hochberg p threshold; *k = 0 ("NONE found")
 * when no p passes */
int gd_css_fdr_threshold(gd_ctx *ctx, const double *p, int64_t n, double fdr, double *testp, int64_t *k,
                         void *hip_stream);
/* SignificantCSSRegions.py:125-126: scores[argsort(scores)[::-1][num_top - 1]] (NaN ranks
 * first, Python indexing; out of range: GD_ERR_ARG) */
int gd_css_top_limit(gd_ctx *ctx, const double *scores, int64_t n, int64_t num_top, double *limit,
                     void *hip_stream);
/* FilterFisherScores.py:92-114 / SignificantCSSRegions.py:123-150: keep the windows passing
 * `cmp thr` and merge them into segments: a segment breaks where the sequence changes or
 * start - max_gap > previous kept start; it is written as (index of its first window,
 * min(last start + max_gap, seq_end[seq])), seq_end = chromosome length - 1.  region_first
 * / region_end need room for *nselected entries (n is always enough). */
int gd_merge_regions(gd_ctx *ctx, const double *vals, const int32_t *seq, const int64_t *start, int64_t n, int cmp,
                     double thr, int64_t max_gap, const int64_t *seq_end, int nseq, int64_t *region_first,
                     int64_t *region_end, int64_t *nregions, int64_t *nselected, void *hip_stream);

/* ---- configuration / diagnostics ---- */
void gd_set_seed(uint64_t seed);     /* seed used by the reference-signature entry points called from the
                                       calling thread (thread-local; every thread starts at GD_DEFAULT_SEED) */
uint64_t gd_get_seed(void);          /* the calling thread's seed */
const char *gd_last_error(void);     /* thread-local message for the last failing call */
int gd_last_status(void);            /* thread-local status (GD_ERR_*) that went with that message */
int gd_device_count(void);

/* timing of the last device scan on this thread (ms, HIP events on the scan's
 * streams), indexed by GD_STAGE_*; returns the number of stages.
 *   MEM     first kernel -> end of the HBM-bound passes (window bounds, per-SNP test)
 *   WINDOW  first kernel -> end of the fast window kernels (overlapped with MEM)
 *   GENERAL duration of the literal per-window path for declined windows
 *   TOTAL   first kernel -> last kernel of the scan */
#define GD_STAGE_MEM 0
#define GD_STAGE_WINDOW 1
#define GD_STAGE_GENERAL 2
#define GD_STAGE_TOTAL 3
#define GD_NSTAGES 4
int gd_last_stage_ms(float *ms, int n);

/* ---- synthetic tracks generated on the device (identical to gdscan/synth.py) ---- */
int gd_synth_device(int chrom, int nsnp, int asize, int bsize, uint64_t seed, const double *freq_table,
                    double *avals, double *bvals, int32_t *apos, int32_t *bpos, void *hip_stream);

/* ---- HyperBrowser track I/O: GTrack "valued points" reader and the
 * tools' tabular writer (FisherExactTestSNPTool.py:162-189, ClusterSeparationScore.py:180-205) ---- */
typedef struct gd_gtrack gd_gtrack;
gd_gtrack *gd_gtrack_read(const char *path); /* NULL on failure (gd_last_error) */
void gd_gtrack_free(gd_gtrack *t);
int gd_gtrack_nseq(const gd_gtrack *t);                   /* sequences, in first-seen order */
const char *gd_gtrack_seqid(const gd_gtrack *t, int s);
int64_t gd_gtrack_len(const gd_gtrack *t, int s);         /* elements of sequence s */
int gd_gtrack_copy(const gd_gtrack *t, int s, int32_t *starts, double *vals);
/* the same files parsed straight into packed genotype tracks (2-bit codes, one position
 * per row; no f64 intermediate): per sequence, size = get_population_size() (the leading
 * run of equal positions, comparative.c:25-34) and nrows rows of `size` individuals at one
 * position.  NULL (gd_last_error) on failure; gd_last_status() is GD_ERR_NOPACK for a
 * readable track with no packed form -- a value other than 3, 0, -3, -10000, a sequence whose
 * positions do not come in whole rows, a population above 2^31 -- which keeps the reference
 * layout (gd_gtrack_read).  A pair of tracks scans packed (gd_pchrom) when
 * each shared sequence has the same rowpos in both. */
typedef struct gd_ptrack gd_ptrack;
gd_ptrack *gd_ptrack_read(const char *path);
void gd_ptrack_free(gd_ptrack *t);
int gd_ptrack_nseq(const gd_ptrack *t); /* sequences, in first-seen order */
const char *gd_ptrack_seqid(const gd_ptrack *t, int s);
int gd_ptrack_shape(const gd_ptrack *t, int s, int32_t *size, int64_t *nrows);
/* codes: nrows * GD_PACK_WORDS(size) words; rowpos: nrows */
int gd_ptrack_copy(const gd_ptrack *t, int s, uint64_t *codes, int32_t *rowpos);
/* appends (or creates) `path`: optional header line, then one line per window with
 * scores[i] != 0: "seqid\t<i*wstep>\t<score>\t<other>", floats as Python 2 str() */
int gd_write_tabular(const char *path, int append, const char *header, const char *seqid, int wstep, int64_t n,
                     const double *scores, const double *other);
int gd_format_py2_float(double x, char *buf, int cap); /* returns the text length */
/* the tools' result files read back for the region filters (FilterFisherScores.py:117-131,
 * SignificantCSSRegions.py:157-173): rows "seqid\tstart\tcol2\tcol3", '#' lines skipped */
typedef struct gd_tabular gd_tabular;
gd_tabular *gd_tabular_read(const char *path); /* NULL on failure (gd_last_error) */
void gd_tabular_free(gd_tabular *t);
int64_t gd_tabular_rows(const gd_tabular *t);
int gd_tabular_nseq(const gd_tabular *t);          /* seqids in first-seen order */
const char *gd_tabular_seqid(const gd_tabular *t, int s);
int gd_tabular_copy(const gd_tabular *t, int32_t *seq, int64_t *start, double *col2, double *col3);

#ifdef __cplusplus
}
#endif
#endif
