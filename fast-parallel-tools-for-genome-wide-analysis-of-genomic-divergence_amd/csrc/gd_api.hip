/*
 * gd_api.hip -- C ABI glue: device contexts, workspaces, the device-resident
 * batched scans and the reference-signature host entry points (include/gdscan.h).
 *
 * The host entry points mirror the reference drivers' contracts:
 *   threadcompute() threadfisher.c:47-100 / threadcss.c:52-109   (window set: GD_WINDOWS_THREADED)
 *   compute()       cFisher.c:38-115     / css.c:49-156          (window set: GD_WINDOWS_SERIAL)
 * input arrays are read-only, outputs are written only at computed windows, and
 * the caller owns every buffer.  Unlike the reference they return a status, do
 * not print, and are reentrant.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <string>
#include <vector>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_internal.h"

/* kernels (gd_fet_kernels.hip, gd_css_kernels.hip, gd_synth.hip) */
__global__ void k_binom_table(uint64_t *tab);
__global__ void k_popsize(gd_chrom_dev *ch, const int32_t *apos, const int32_t *bpos, unsigned *flags);
__global__ void k_bounds(const gd_chrom_dev *ch, const int32_t *apos, const int32_t *bpos, int wsize, int wstep,
                         int32_t *lo_a, int32_t *hi_a, int32_t *lo_b, unsigned *flags);
__global__ void k_snp_fet(const gd_chrom_dev *ch, const double *avals, const double *bvals, const uint64_t *binom,
                          const int *lut_hdr, const double *lut, double *snp_score, int skip_table_held);
__global__ void k_fet_lut_build(const gd_chrom_dev *ch, const uint64_t *binom, const int *hdr, double *lut,
                                int64_t cap);
__global__ void k_fet_lut_publish(const gd_chrom_dev *ch, const uint64_t *binom, int *hdr, int64_t cap);
template <int BLOCK, bool GLOBAL_SCRATCH>
__global__ void k_fet_window_general(const gd_chrom_dev *ch, int nchrom, const int32_t *wlist,
                                     const unsigned *wlist_count, int64_t wtotal, const int32_t *lo_a,
                                     const int32_t *hi_a, const int32_t *lo_b, const double *avals,
                                     const double *bvals, const double *snp_score, const uint64_t *binom,
                                     const int *lut_hdr, const double *lut, double perc, double *scores,
                                     double *stddev, unsigned *flags,
                                     int32_t *huge_list, unsigned *huge_count, double *gscratch,
                                     int64_t gscratch_n);
int gd_packed_bounds_launch(const gd_chrom_dev *d_ch, int nchrom, const int64_t *row_off, const int32_t *rowpos,
                            int64_t max_rows, int wsize, int wstep, int32_t *lo_a, int32_t *hi_a, int32_t *lo_b,
                            unsigned *flags, hipStream_t s);
int gd_packed_snp_fet_launch(const gd_chrom_dev *d_ch, int nchrom, const int64_t *word_off, const uint64_t *acodes,
                             const uint64_t *bcodes, int64_t max_rows, const uint64_t *binom, const int *lut_hdr,
                             const double *lut, double *snp, hipStream_t s);
int gd_pack_device_launch(const double *avals, const double *bvals, const int32_t *apos, const int32_t *bpos,
                          int asize, int bsize, int nrows, uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos,
                          unsigned *bad, hipStream_t s);
int gd_fet_fast_windows_per_block();
__global__ void k_fet_setup(gd_chrom_dev *ch, int nchrom, const int32_t *apos, const int32_t *bpos, unsigned *flags,
                            const uint64_t *binom, int *hdr, double *lut, int64_t cap, unsigned *done);
int gd_bounds_elems_per_block();
int gd_fet_fast_init(hipStream_t s);
int gd_fet_window_prepare(int64_t wtotal, int32_t *slow_list, unsigned *slow_count, hipStream_t s,
                          bool *force_general);
int gd_fet_window_fast_launch(const gd_chrom_dev *ch, int nchrom, const int32_t *blk_off, int blk_begin,
                              int blk_count, const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b,
                              const double *snp_score, const double *avals, const double *bvals,
                              const uint64_t *binom, const int *lut_hdr, const double *lut, int fused, double perc,
                              double *scores, double *stddev, unsigned *flags, int32_t *slow_list,
                              unsigned *slow_count, hipStream_t s);
int gd_css_tier(int m);
int gd_css_launch(int mp, int drosophila, int mds, const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl,
                  uint32_t *planes, const int32_t *lo_a, const int32_t *hi_a, const int32_t *lo_b,
                  const double *avals, const double *bvals, const int64_t *word_off, const uint64_t *acodes,
                  const uint64_t *bcodes, int64_t wtotal, int64_t max_rows_words, int treshold, int runs,
                  double *scores, double *p, double *xbuf, uint8_t *status, unsigned *flags, double *slab,
                  hipStream_t s, hipEvent_t ev_perm);
int gd_synth_launch(int chrom, int nsnp, int asize, int bsize, uint64_t seed, const double *freq_table,
                    double *avals, double *bvals, int32_t *apos, int32_t *bpos, hipStream_t s);

/* general-path grid (gd_internal.h): resident capacity of the current device (CU counts
 * cached per device: a process may drive devices of different sizes) */
int64_t gd_css_big_grid(int64_t wtotal, int mp) {
  constexpr int NDEV = 64;
  static std::atomic<int> cus[NDEV];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  int n = dev < NDEV ? cus[dev].load() : 0;
  if (n == 0) {
    int v = 0;
    n = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
    if (dev < NDEV) cus[dev].store(n);
  }
  int64_t grid = (int64_t)n * (mp <= 256 ? 4 : mp <= 1024 ? 2 : 1); /* 2048 tier: one ~120 KB-LDS workgroup per CU */
  if (const char *e = getenv("GD_CSS_BIG_GRID")) {
    const long long g = atoll(e);
    if (g > 0) grid = g;
  }
  return wtotal < grid ? wtotal : grid;
}

/* ------------------------------------------------------------------ errors */
static thread_local std::string g_err;
static thread_local int g_status = GD_OK; /* the status that went with g_err (gd_last_status) */
/* seed of the reference-signature entry points: per calling thread (gd_set_seed affects
 * only the thread that calls it; every thread starts at GD_DEFAULT_SEED), so two threads
 * that each set a seed and call fisher_exact_tester cannot race on it */
static thread_local uint64_t g_seed = GD_DEFAULT_SEED;
static std::atomic<int> g_fet_mode{GD_FET_REFERENCE};
static thread_local float g_stage_ms[GD_NSTAGES];

static int fail(int code, const std::string &msg) {
  g_err = msg;
  g_status = code;
  return code;
}
/* for gd_gtrack.cpp / gd_pack.cpp */
void gd_set_error(const char *msg) {
  g_err = msg ? msg : "";
  g_status = GD_ERR_ARG;
}
void gd_set_status_error(int code, const char *msg) {
  g_err = msg ? msg : "";
  g_status = code;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail(GD_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

/* ----------------------------------------------------------------- context */
struct gd_ctx {
  int device = 0;
  std::mutex mu;
  hipStream_t stream = nullptr;  /* used by the host entry points */
  hipStream_t stream2 = nullptr;    /* window kernels of the pipelined scans (lowest priority) */
  hipStream_t stream_mem = nullptr; /* HBM-bound passes of the pipelined scans (highest priority) */
  hipEvent_t gev[GD_MAX_GROUPS] = {};
  char *ws = nullptr;
  size_t ws_cap = 0;
  double *gscratch = nullptr;
  size_t gscratch_cap = 0; /* doubles */
  uint64_t *binom = nullptr;       /* FET table buffer (gd_common.h), reference mode */
  uint64_t *binom_exact = nullptr; /* the same, exact mode */
  /* FET score table, cached across scans for the last (asize, bsize) */
  int *lut_hdr = nullptr;
  double *lut = nullptr;
  /* host-API staging buffers (device) */
  char *io = nullptr;
  size_t io_cap = 0;
  hipEvent_t ev[GD_NSTAGES + 1] = {};
  unsigned *h_flags = nullptr; /* pinned */
  char *h_stage = nullptr;     /* pinned staging of the per-call descriptors (h2d) */
  size_t h_stage_cap = 0, h_stage_off = 0;
  hipEvent_t stage_ev = nullptr; /* after the last copy out of h_stage (recorded by h2d) */
  bool stage_live = false;       /* stage_ev was recorded since the buffer was last reset */
  unsigned *h_flags_dev = nullptr; /* one device word (packer status) */
  char *h_pack = nullptr;          /* pinned: host-packed tracks of the reference-signature calls */
  size_t h_pack_cap = 0;
  bool pack_inflight = false; /* copies out of h_pack may still run (a call returned mid-upload) */
};

static int ctx_init(gd_ctx *c, int device) {
  c->device = device;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  {
    /* the memory passes feed the window kernels: give them the CUs first */
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, least));
    HIP_TRY(hipStreamCreateWithPriority(&c->stream_mem, hipStreamNonBlocking, greatest));
  }
  for (auto &e : c->gev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_TRY(hipMalloc(&c->binom, sizeof(uint64_t) * GD_FET_TAB_WORDS));
  HIP_TRY(hipMalloc(&c->binom_exact, sizeof(uint64_t) * GD_FET_TAB_WORDS));
  hipLaunchKernelGGL(k_binom_table, dim3((GD_BINOM_ENTRIES + 255) / 256), dim3(256), 0, c->stream, c->binom);
  hipLaunchKernelGGL(k_binom_table, dim3((GD_BINOM_ENTRIES + 255) / 256), dim3(256), 0, c->stream, c->binom_exact);
  HIP_TRY(hipGetLastError());
  if (gd_fet_fast_init(c->stream) != GD_OK) return GD_ERR_HIP;
  {
    /* behind the binomials (disjoint from the kernel's writes): the mode word, then
     * ln k! as double-double for exact mode */
    std::vector<uint64_t> tail(GD_FET_TAB_WORDS - GD_BINOM_ENTRIES, 0);
    tail[0] = GD_FET_REFERENCE;
    HIP_TRY(hipMemcpy(c->binom + GD_BINOM_ENTRIES, tail.data(), sizeof(uint64_t) * tail.size(),
                      hipMemcpyHostToDevice));
    tail[0] = GD_FET_EXACT;
    for (int k = 0; k <= GD_BINOM_NMAX; ++k) {
      const long double L = lgammal((long double)k + 1.0L);
      const double hi = (double)L, lo = (double)(L - (long double)hi);
      std::memcpy(&tail[GD_FET_LF_OFF - GD_BINOM_ENTRIES + k], &hi, sizeof hi);
      std::memcpy(&tail[GD_FET_LF_OFF - GD_BINOM_ENTRIES + GD_BINOM_NMAX + 1 + k], &lo, sizeof lo);
    }
    HIP_TRY(hipMemcpy(c->binom_exact + GD_BINOM_ENTRIES, tail.data(), sizeof(uint64_t) * tail.size(),
                      hipMemcpyHostToDevice));
  }
  for (auto &e : c->ev) HIP_TRY(hipEventCreate(&e));
  HIP_TRY(hipEventCreateWithFlags(&c->stage_ev, hipEventDisableTiming));
  HIP_TRY(hipMalloc(&c->lut_hdr, 4 * sizeof(int)));
  HIP_TRY(hipMemsetAsync(c->lut_hdr, 0, 4 * sizeof(int), c->stream));
  HIP_TRY(hipMalloc(&c->lut, sizeof(double) * GD_LUT_CAP));
  HIP_TRY(hipHostMalloc(&c->h_flags, 64));
  HIP_TRY(hipMalloc(&c->h_flags_dev, 64));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GD_OK;
}

extern "C" gd_ctx *gd_ctx_create(int device) {
  gd_ctx *c = new gd_ctx();
  if (ctx_init(c, device) != GD_OK) {
    gd_ctx_destroy(c);
    return nullptr;
  }
  return c;
}

extern "C" void gd_ctx_destroy(gd_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->ws);
  (void)hipFree(c->gscratch);
  (void)hipFree(c->binom);
  (void)hipFree(c->binom_exact);
  (void)hipFree(c->lut_hdr);
  (void)hipFree(c->lut);
  (void)hipFree(c->io);
  for (auto &e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto &e : c->gev)
    if (e) (void)hipEventDestroy(e);
  if (c->stage_ev) {
    (void)hipEventSynchronize(c->stage_ev);
    (void)hipEventDestroy(c->stage_ev);
  }
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  if (c->stream_mem) (void)hipStreamDestroy(c->stream_mem);
  if (c->h_flags) (void)hipHostFree(c->h_flags);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->h_pack) (void)hipHostFree(c->h_pack);
  if (c->h_flags_dev) (void)hipFree(c->h_flags_dev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static gd_ctx *default_ctx(int *status) {
  static std::mutex m;
  static std::vector<gd_ctx *> ctxs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> g(m);
  if ((int)ctxs.size() <= dev) ctxs.resize(dev + 1, nullptr);
  if (!ctxs[dev]) {
    ctxs[dev] = gd_ctx_create(dev);
    if (!ctxs[dev]) {
      *status = GD_ERR_HIP;
      return nullptr;
    }
  }
  *status = GD_OK;
  return ctxs[dev];
}

static int grow(char **buf, size_t *cap, size_t need) {
  if (need <= *cap) return GD_OK;
  if (*buf) HIP_TRY(hipFree(*buf));
  *buf = nullptr;
  *cap = 0;
  size_t n = std::max(need, (size_t)1 << 20);
  n += n / 4;
  HIP_TRY(hipMalloc(buf, n));
  *cap = n;
  return GD_OK;
}

/* -------------------------------------------------------------- windows */
extern "C" int gd_window_count(int regend, int wsize, int wstep, int window_set) {
  if (wsize <= 0 || wstep <= 0 || regend <= 0) return 0;
  int64_t end = 0;
  if (window_set == GD_WINDOWS_SERIAL) {
    /* while (start + wsize <= regend + wstep)  (cFisher.c:81, css.c:117) */
    const int64_t lim = (int64_t)regend + wstep - wsize;
    end = lim >= 0 ? lim / wstep + 1 : 0;
  } else {
    /* threadfisher.c:55-58,191-239 / threadcss.c:60-63,226-276 */
    const int num_windows = regend / wstep - 3;
    const int num_tasks = num_windows / 100;
    if (num_tasks <= 0) return 0;
    for (int64_t t = 0; t <= num_tasks; ++t) {
      int64_t stop = (t + 1) * 100 * (int64_t)wstep + (wsize - wstep);
      if (stop >= regend) stop = (int64_t)regend + wstep;
      const int64_t first = t * 100 * (int64_t)wstep;
      if (first + wsize > stop) continue;
      const int64_t last = (stop - wsize) / wstep; /* largest w with w*wstep + wsize <= stop */
      end = std::max(end, last + 1);
    }
  }
  return (int)std::min<int64_t>(end, regend / wstep);
}

/* -------------------------------------------------------- workspace carve */
struct Carve {
  char *base;
  size_t off = 0;
  template <class T>
  T *take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T *p = (T *)(base ? base + off : nullptr);
    off += n * sizeof(T);
    return p;
  }
};

struct ScanPlan {
  std::vector<gd_chrom_dev> h;
  int64_t wtotal = 0;
  int64_t elems_a = 0, elems_b = 0;
  int32_t max_alen = 0, max_blen = 0;
};

static int make_plan(const gd_chrom *chroms, int nchrom, int wsize, int wstep, int window_set, ScanPlan *pl) {
  if (nchrom < 0 || (nchrom > 0 && !chroms)) return fail(GD_ERR_ARG, "bad chromosome list");
  if (wsize <= 0 || wstep <= 0) return fail(GD_ERR_ARG, "wsize and wstep must be positive");
  if (window_set != GD_WINDOWS_THREADED && window_set != GD_WINDOWS_SERIAL)
    return fail(GD_ERR_ARG, "unknown window set");
  pl->h.resize(nchrom);
  int64_t wb = 0;
  for (int c = 0; c < nchrom; ++c) {
    const gd_chrom &s = chroms[c];
    if (s.alen < 0 || s.blen < 0 || s.a_off < 0 || s.b_off < 0) return fail(GD_ERR_ARG, "negative extent");
    if (s.w_first < 0 || s.w_count < 0) return fail(GD_ERR_ARG, "negative window range");
    gd_chrom_dev &d = pl->h[c];
    std::memset(&d, 0, sizeof d);
    d.a_off = s.a_off;
    d.b_off = s.b_off;
    d.alen = s.alen;
    d.blen = s.blen;
    d.regend = s.regend;
    d.w_out = s.w_out;
    d.seed = s.seed;
    /* the chromosome's window set [0, n), restricted to [w_first, w_first + w_count) */
    const int64_t n = (s.alen > 0 && s.blen > 0) ? gd_window_count(s.regend, wsize, wstep, window_set) : 0;
    const int64_t hi = s.w_count > 0 ? std::min<int64_t>(n, (int64_t)s.w_first + s.w_count) : n;
    d.w_first = s.w_first;
    d.wend = (int32_t)std::max<int64_t>(0, hi - s.w_first);
    d.w_base = wb;
    wb += d.wend;
    pl->elems_a = std::max<int64_t>(pl->elems_a, s.a_off + s.alen);
    pl->elems_b = std::max<int64_t>(pl->elems_b, s.b_off + s.blen);
    pl->max_alen = std::max(pl->max_alen, s.alen);
    pl->max_blen = std::max(pl->max_blen, s.blen);
  }
  if (wb > INT32_MAX) return fail(GD_ERR_ARG, "too many windows in one batch");
  pl->wtotal = wb;
  return GD_OK;
}

/* a packed batch (include/gdscan.h): descriptors and device pointers to the codes */
struct PackedIn {
  const gd_pchrom *pc;
  const uint64_t *acodes, *bcodes;
  const int32_t *rowpos;
};

/* the packed chromosomes as their expanded forms: element extents nrows * size, sizes
 * known up front; a_off = b_off = the first row (the per-SNP score array is indexed
 * a_off + row, and nothing reads element-indexed values) */
static int make_plan_packed(const PackedIn &pk, int nchrom, int wsize, int wstep, int window_set, ScanPlan *pl,
                            std::vector<int64_t> *row_off, std::vector<int64_t> *word_off, int64_t *max_rows) {
  if (nchrom < 0 || (nchrom > 0 && !pk.pc)) return fail(GD_ERR_ARG, "bad chromosome list");
  if (nchrom > 0 && (!pk.acodes || !pk.bcodes || !pk.rowpos)) return fail(GD_ERR_ARG, "null packed buffer");
  std::vector<gd_chrom> ch(nchrom);
  for (int c = 0; c < nchrom; ++c) {
    const gd_pchrom &q = pk.pc[c];
    if (q.nrows < 0 || q.row_off < 0 || q.a_word < 0 || q.b_word < 0) return fail(GD_ERR_ARG, "negative extent");
    if (q.nrows > 0 && (q.asize <= 0 || q.bsize <= 0)) return fail(GD_ERR_SIZE, "empty population");
    if ((int64_t)q.nrows * std::max(q.asize, q.bsize) > INT32_MAX) return fail(GD_ERR_SIZE, "chromosome too long");
    std::memset(&ch[c], 0, sizeof(gd_chrom));
    ch[c].a_off = ch[c].b_off = q.row_off;
    ch[c].alen = q.nrows > 0 ? q.nrows * q.asize : 0;
    ch[c].blen = q.nrows > 0 ? q.nrows * q.bsize : 0;
    ch[c].regend = q.regend;
    ch[c].w_out = q.w_out;
    ch[c].seed = q.seed;
  }
  int st = make_plan(ch.data(), nchrom, wsize, wstep, window_set, pl);
  if (st) return st;
  row_off->assign(nchrom, 0);
  word_off->assign(2 * (size_t)nchrom, 0);
  *max_rows = 1;
  pl->elems_a = 1;
  for (int c = 0; c < nchrom; ++c) {
    const gd_pchrom &q = pk.pc[c];
    gd_chrom_dev &d = pl->h[c];
    d.asize = q.asize;
    d.bsize = q.bsize;
    d.nrows = q.nrows;
    (*row_off)[c] = q.row_off;
    (*word_off)[2 * c] = q.a_word;
    (*word_off)[2 * c + 1] = q.b_word;
    *max_rows = std::max<int64_t>(*max_rows, q.nrows);
    pl->elems_a = std::max<int64_t>(pl->elems_a, q.row_off + q.nrows); /* rows of snp_score */
  }
  return GD_OK;
}

/* Host -> device copy of a per-call descriptor array through the context's pinned
 * staging buffer, so the copy is a plain asynchronous DMA (a pageable source makes
 * hipMemcpyAsync stage it synchronously).  stage_ev follows the last staged copy: a call
 * starts by waiting for it (stage_reset) before it rewrites the buffer, so a call that
 * returned early on an error path, before its stream sync, cannot leave a DMA reading
 * memory the next call overwrites. */
static int stage_reset(gd_ctx *c) {
  if (c->stage_live) HIP_TRY(hipEventSynchronize(c->stage_ev));
  c->stage_live = false;
  c->h_stage_off = 0;
  return GD_OK;
}

static int h2d(gd_ctx *c, void *dst, const void *src, size_t bytes, hipStream_t s) {
  const size_t need = (c->h_stage_off + bytes + 255) & ~(size_t)255;
  if (need > c->h_stage_cap) {
    /* every staged copy so far (this call's, on s) has landed before the buffer is freed */
    if (c->stage_live) HIP_TRY(hipEventSynchronize(c->stage_ev));
    c->stage_live = false;
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->h_stage_cap = 0;
    c->h_stage_off = 0;
    const size_t cap = std::max<size_t>(std::max<size_t>(need, 2 * bytes + 256), 1 << 16);
    HIP_TRY(hipHostMalloc(&c->h_stage, cap));
    c->h_stage_cap = cap;
  }
  char *p = c->h_stage + c->h_stage_off;
  std::memcpy(p, src, bytes);
  c->h_stage_off = (c->h_stage_off + bytes + 255) & ~(size_t)255;
  HIP_TRY(hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipEventRecord(c->stage_ev, s));
  c->stage_live = true;
  return GD_OK;
}

static int flags_to_status(unsigned f) {
  if (f & (GD_FLAG_UNSORTED_A | GD_FLAG_UNSORTED_B)) return fail(GD_ERR_UNSORTED, "positions are not sorted");
  if (f & GD_FLAG_B_BOUNDS) return fail(GD_ERR_BOUNDS, "a window's B slice runs past blen");
  if (f & GD_FLAG_BAD_SIZE) return fail(GD_ERR_SIZE, "empty population or unsupported window size");
  return GD_OK;
}

/* --------------------------------------------------------------- FET scan */
/* pk != NULL: a packed batch (chroms, avals .. bpos unused) */
static int fet_scan_locked(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                           const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize, int wstep,
                           double perc, int mode, int window_set, double *scores, double *stddev, hipStream_t s,
                           const PackedIn *pk = nullptr) {
  if (!(perc >= 0.0 && perc <= 1.0)) return fail(GD_ERR_ARG, "percentile must lie in [0, 1]");
  if (mode != GD_FET_REFERENCE && mode != GD_FET_EXACT)
    return fail(GD_ERR_ARG, "FET mode must be GD_FET_REFERENCE (0) or GD_FET_EXACT (1)");
  const uint64_t *binom = mode == GD_FET_EXACT ? ctx->binom_exact : ctx->binom;
  ScanPlan pl;
  std::vector<int64_t> row_off, word_off;
  int64_t max_rows = 1;
  int st = pk ? make_plan_packed(*pk, nchrom, wsize, wstep, window_set, &pl, &row_off, &word_off, &max_rows)
              : make_plan(chroms, nchrom, wsize, wstep, window_set, &pl);
  if (st) return st;
  for (float &m : g_stage_ms) m = 0.f;
  if (pl.wtotal == 0) return GD_OK;
  HIP_TRY(hipSetDevice(ctx->device));

  /* fast-kernel workgroups are aligned to chromosomes: blk_off[c] = first workgroup of c */
  const int wpb = gd_fet_fast_windows_per_block();
  std::vector<int32_t> blk_off(nchrom + 1, 0);
  for (int c = 0; c < nchrom; ++c) blk_off[c + 1] = blk_off[c] + (pl.h[c].wend + wpb - 1) / wpb;

  Carve cv{nullptr};
  /* flags: [0] status bits, [4] declined-window count, [8] dense-window count, [12] the
   * setup kernel's done counter -- zeroed by one memset per scan */
  const size_t nflags = 16;
  auto layout = [&](Carve &k, gd_chrom_dev **d_ch, int32_t **d_blk, unsigned **flags, int32_t **lo_a,
                    int32_t **hi_a, int32_t **lo_b, double **snp, int32_t **list, int32_t **huge) {
    *d_ch = k.take<gd_chrom_dev>(nchrom);
    *d_blk = k.take<int32_t>(nchrom + 1);
    *flags = k.take<unsigned>(nflags);
    *lo_a = k.take<int32_t>(pl.wtotal);
    *hi_a = k.take<int32_t>(pl.wtotal);
    *lo_b = k.take<int32_t>(pl.wtotal);
    *snp = k.take<double>(pl.elems_a);
    *list = k.take<int32_t>(pl.wtotal);
    *huge = k.take<int32_t>(pl.wtotal);
  };
  gd_chrom_dev *d_ch;
  unsigned *flags;
  int32_t *d_blk, *lo_a, *hi_a, *lo_b, *list, *huge;
  double *snp;
  int64_t *d_roff = nullptr, *d_woff = nullptr;
  auto layout_all = [&](Carve &k) {
    layout(k, &d_ch, &d_blk, &flags, &lo_a, &hi_a, &lo_b, &snp, &list, &huge);
    if (pk) {
      d_roff = k.take<int64_t>(nchrom);
      d_woff = k.take<int64_t>(2 * (size_t)nchrom);
    }
  };
  layout_all(cv);
  if ((st = grow(&ctx->ws, &ctx->ws_cap, cv.off))) return st;
  Carve real{ctx->ws};
  layout_all(real);
  unsigned *list_count = flags + 4, *huge_count = flags + 8;
  if ((st = stage_reset(ctx))) return st;
  if (pk) {
    if ((st = h2d(ctx, d_roff, row_off.data(), sizeof(int64_t) * nchrom, s))) return st;
    if ((st = h2d(ctx, d_woff, word_off.data(), sizeof(int64_t) * 2 * nchrom, s))) return st;
  }
  if ((st = h2d(ctx, d_ch, pl.h.data(), sizeof(gd_chrom_dev) * nchrom, s))) return st;
  if ((st = h2d(ctx, d_blk, blk_off.data(), sizeof(int32_t) * (nchrom + 1), s))) return st;
  HIP_TRY(hipMemsetAsync(flags, 0, nflags * sizeof(unsigned), s));
  HIP_TRY(hipEventRecord(ctx->ev[0], s));
  /* Pipeline over chromosome groups: the passes (prologue, then each group's bounds) run in
   * order on the high-priority stream sm; group g's window kernel waits for its own bounds
   * pass only, the window kernels alternating between stream2 and the caller's stream s so
   * that one starts while the other drains.  Two equal groups (r05 sweep, C2 per scan: 2
   * groups 2.216-2.227 ms, 1 group 2.253, 3 groups 2.299; doubling groups 1, 2, 4, ... with
   * the later bounds passes at one workgroup per CU 2.230-2.238, on the whole GPU 2.357-2.392;
   * the same with the window kernels' LDS padded to six workgroups per CU, so that a bounds
   * workgroup always fits beside them, 2.300-2.312).  A pass that runs beside a window kernel
   * displaces window workgroups (LDS, VGPRs and wave slots are all but full at seven per CU),
   * so it costs its own slot-time wherever it is scheduled: the bounds pass is hidden only
   * for the second group's share.  (GD_GROUPS=<n>: diagnostics.) */
  const char *uf = getenv("GD_FET_UNFUSED");
  const bool fused = !pk && !(uf && uf[0] == '1'); /* packed: the per-SNP pass reads 2 bits per genotype */
  int G = std::min(nchrom, 2);
  if (const char *eg = getenv("GD_GROUPS")) G = std::max(1, std::min(std::min(nchrom, GD_MAX_GROUPS), atoi(eg)));
  hipStream_t sm = G > 1 ? ctx->stream_mem : s, s2 = G > 1 ? ctx->stream2 : s;
  if (G > 1) HIP_TRY(hipStreamWaitEvent(sm, ctx->ev[0], 0));
  bool force_general = false;
  if ((st = gd_fet_window_prepare(pl.wtotal, list, list_count, sm, &force_general))) return st;
  if (!pk) {
    /* population sizes and the score table for chromosome 0's sizes in one launch (the table
     * build is a no-op when the context holds it) */
    hipLaunchKernelGGL(k_fet_setup, dim3(256), dim3(256), 0, sm, d_ch, nchrom, apos, bpos, flags, binom, ctx->lut_hdr,
                       ctx->lut, (int64_t)GD_LUT_CAP, flags + 12);
  } else {
    hipLaunchKernelGGL(k_fet_lut_build, dim3(512), dim3(256), 0, sm, d_ch, binom, ctx->lut_hdr, ctx->lut,
                       (int64_t)GD_LUT_CAP);
    hipLaunchKernelGGL(k_fet_lut_publish, dim3(1), dim3(1), 0, sm, d_ch, binom, ctx->lut_hdr, (int64_t)GD_LUT_CAP);
  }
  if (fused) {
    /* the per-SNP pass for chromosomes whose sizes the table does not hold (every workgroup
     * exits at once otherwise): before any bounds pass, on a grid that costs nothing then */
    int64_t amax = 1;
    for (int c = 0; c < nchrom; ++c) amax = std::max<int64_t>(amax, pl.h[c].alen);
    const unsigned gxs = (unsigned)std::min<int64_t>((amax + 255) / 256, std::max(1, 1024 / nchrom));
    hipLaunchKernelGGL(k_snp_fet, dim3(gxs, nchrom), dim3(256), 0, sm, d_ch, avals, bvals, binom, ctx->lut_hdr,
                       ctx->lut, snp, 1);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev[1], sm)); /* end of the prologue */
  std::vector<int> cuts(G + 1);
  for (int g = 0; g <= G; ++g) cuts[g] = (int)((int64_t)nchrom * g / G);
  if (const char *e0 = getenv("GD_GROUP0")) { /* diagnostics: the first group's chromosomes, the rest split evenly */
    const int n0 = std::max(1, std::min(nchrom - (G - 1), atoi(e0)));
    if (G > 1) {
      cuts[1] = n0;
      for (int g = 2; g <= G; ++g) cuts[g] = n0 + (int)((int64_t)(nchrom - n0) * (g - 1) / (G - 1));
    }
  }
  auto bounds_pass = [&](int g) -> int {
    const int c0 = cuts[g], nc = cuts[g + 1] - cuts[g];
    int64_t amax = 1, mx = 1;
    for (int c = c0; c < c0 + nc; ++c) {
      amax = std::max<int64_t>(amax, pl.h[c].alen);
      mx = std::max<int64_t>(mx, std::max(pl.h[c].alen, pl.h[c].blen) + 1);
    }
    if (pk) {
      int r;
      if ((r = gd_packed_bounds_launch(d_ch + c0, nc, d_roff + c0, pk->rowpos, max_rows, wsize, wstep, lo_a, hi_a,
                                       lo_b, flags, sm)) ||
          (r = gd_packed_snp_fet_launch(d_ch + c0, nc, d_woff + 2 * c0, pk->acodes, pk->bcodes, max_rows, binom,
                                        ctx->lut_hdr, ctx->lut, snp, sm)))
        return fail(r, "packed pass launch failed");
    } else {
      const int64_t epb = gd_bounds_elems_per_block();
      const unsigned gxb = (unsigned)std::min<int64_t>((mx + epb - 1) / epb, std::max(1, 8192 / nc));
      hipLaunchKernelGGL(k_bounds, dim3(gxb, nc, 2), dim3(256), 0, sm, d_ch + c0, apos, bpos, wsize, wstep, lo_a,
                         hi_a, lo_b, flags);
      if (!fused) {
        const unsigned gxs = (unsigned)std::min<int64_t>((amax + 255) / 256, std::max(1, 8192 / nc));
        hipLaunchKernelGGL(k_snp_fet, dim3(gxs, nc), dim3(256), 0, sm, d_ch + c0, avals, bvals, binom, ctx->lut_hdr,
                           ctx->lut, snp, 0);
      }
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ctx->gev[g], sm));
    return GD_OK;
  };
  auto window_pass = [&](int g) -> int {
    const int c0 = cuts[g], c1 = cuts[g + 1];
    hipStream_t sw = (g & 1) ? s : s2;
    if (G > 1) HIP_TRY(hipStreamWaitEvent(sw, ctx->gev[g], 0));
    const int r = gd_fet_window_fast_launch(d_ch, nchrom, d_blk, blk_off[c0], blk_off[c1] - blk_off[c0], lo_a, hi_a,
                                            lo_b, snp, avals, bvals, binom, ctx->lut_hdr, ctx->lut, fused ? 1 : 0, perc,
                                            scores, stddev, flags, list, list_count, sw);
    return r ? fail(r, "fast window kernel launch failed") : GD_OK;
  };
  /* submission order bounds 0, bounds 1, windows 0, bounds 2, windows 1, ...: every window
   * kernel is queued as soon as its bounds are, behind the next group's bounds pass */
  for (int g = 0; g < G; ++g) {
    if ((st = bounds_pass(g))) return st;
    if (g > 0 && !force_general && (st = window_pass(g - 1))) return st;
  }
  if (!force_general && (st = window_pass(G - 1))) return st;
  if (G > 1) {
    /* ev[2] after every group's window kernel: the odd groups ran on s, the others on s2 */
    HIP_TRY(hipEventRecord(ctx->ev[4], s2));
    HIP_TRY(hipStreamWaitEvent(s, ctx->ev[4], 0));
    HIP_TRY(hipStreamWaitEvent(s, ctx->gev[G - 1], 0));
  }
  HIP_TRY(hipEventRecord(ctx->ev[2], s));
  {
    /* windows the fast path declined: literal one-workgroup-per-window path */
    const unsigned gx = (unsigned)std::min<int64_t>(pl.wtotal, 4096);
    hipLaunchKernelGGL((k_fet_window_general<64, false>), dim3(gx), dim3(64), 0, s, d_ch, nchrom, list,
                       list_count, pl.wtotal, lo_a, hi_a, lo_b, avals, bvals, snp, binom,
                       fused ? ctx->lut_hdr : (const int *)nullptr, ctx->lut, perc, scores,
                       stddev, flags, huge, huge_count, (double *)nullptr, (int64_t)0);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev[3], s));
  HIP_TRY(hipMemcpyAsync(ctx->h_flags, flags, 16 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const unsigned nhuge = ctx->h_flags[8];
  if (nhuge > 0 && !(ctx->h_flags[0] & ~GD_FLAG_B_BOUNDS)) {
    /* windows too dense for LDS: one 256-thread workgroup each, scratch in HBM */
    const int64_t nmax = std::max<int64_t>(pl.max_alen, 1);
    int64_t np2 = 1;
    while (np2 < nmax) np2 <<= 1;
    const int64_t per = np2 + 2 * nmax + (nmax + 1) / 2 + 2;
    const int slots = 4;
    if ((size_t)(per * slots) > ctx->gscratch_cap) {
      (void)hipFree(ctx->gscratch);
      ctx->gscratch = nullptr;
      ctx->gscratch_cap = 0;
      HIP_TRY(hipMalloc(&ctx->gscratch, sizeof(double) * per * slots));
      ctx->gscratch_cap = per * slots;
    }
    hipLaunchKernelGGL((k_fet_window_general<256, true>), dim3(slots), dim3(256), 0, s, d_ch, nchrom, huge,
                       huge_count, (int64_t)0, lo_a, hi_a, lo_b, avals, bvals, snp, binom,
                       fused ? ctx->lut_hdr : (const int *)nullptr, ctx->lut, perc, scores,
                       stddev, flags, (int32_t *)nullptr, (unsigned *)nullptr, ctx->gscratch, per);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(ctx->h_flags, flags, 16 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  float ms;
  /* stage times (HIP events from the scan's first kernel): MEM = the prologue (setup and
   * every group's bounds / per-SNP passes), WINDOW = the end of the last fast window kernel,
   * GENERAL = the literal path after it, TOTAL */
  if (hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]) == hipSuccess) g_stage_ms[GD_STAGE_MEM] = ms;
  if (hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[2]) == hipSuccess) g_stage_ms[GD_STAGE_WINDOW] = ms;
  if (hipEventElapsedTime(&ms, ctx->ev[2], ctx->ev[3]) == hipSuccess) g_stage_ms[GD_STAGE_GENERAL] = ms;
  if (hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[3]) == hipSuccess) g_stage_ms[GD_STAGE_TOTAL] = ms;
  return flags_to_status(ctx->h_flags[0]);
}

extern "C" int gd_fet_scan_device_ex(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                                     const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize,
                                     int wstep, double perc, int mode, int window_set, double *scores,
                                     double *stddev, void *hip_stream) {
  if (!ctx) return fail(GD_ERR_ARG, "null context");
  std::lock_guard<std::mutex> g(ctx->mu);
  return fet_scan_locked(ctx, chroms, nchrom, avals, bvals, apos, bpos, wsize, wstep, perc, mode, window_set,
                         scores, stddev, (hipStream_t)hip_stream);
}

extern "C" int gd_fet_scan_device(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                                  const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize,
                                  int wstep, double perc, int window_set, double *scores, double *stddev,
                                  void *hip_stream) {
  return gd_fet_scan_device_ex(ctx, chroms, nchrom, avals, bvals, apos, bpos, wsize, wstep, perc,
                               g_fet_mode.load(), window_set, scores, stddev, hip_stream);
}

extern "C" int gd_pack_rows_mt(const double *avals, const double *bvals, const int *apos, const int *bpos, int asize,
                               int bsize, int64_t r0, int64_t r1, uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos);

/* The reference-signature host entry points over packed tracks.  When every chromosome's
 * host arrays are whole rows of the four genotype codes with one position per row
 * (gd_pack_shape and gd_pack_chrom_mt accept them -- the tracks VCFConvert writes), they are
 * packed on host threads into the context's pinned buffer, and 2 bits per genotype plus 4 B
 * per row cross PCIe instead of 12 B per genotype; the packed scan equals the reference-
 * layout scan of the same tracks (tests/test_packed.py, test_host_pack_gpu.py).  Returns
 * GD_HOST_NOPACK (nothing done) when a chromosome has no packed form: the caller then ships
 * the reference layout.  GD_HOST_NOPACK=1 in the environment disables the route. */
static constexpr int GD_HOST_NOPACK = 1;

template <class Run>
static int host_packed(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                       const int *apos, const int *bpos, int wstep, double *out0, double *out1, Run run) {
  if (const char *e = getenv("GD_HOST_NOPACK"))
    if (e[0] == '1') return GD_HOST_NOPACK;
  std::vector<gd_pchrom> pc(nchrom);
  int64_t rows = 0, wa_tot = 0, wb_tot = 0, nw = 0;
  for (int c = 0; c < nchrom; ++c) {
    const gd_chrom &h = chroms[c];
    if (h.w_first != 0 || h.w_count != 0) return GD_HOST_NOPACK; /* window-range shards: reference layout */
    int asz = 0, bsz = 0, nr = 0;
    if (h.alen > 0 && h.blen > 0) {
      const std::string saved = g_err; /* a refusal here is not the call's error */
      const int saved_st = g_status;
      if (gd_pack_shape(apos + h.a_off, bpos + h.b_off, h.alen, h.blen, &asz, &bsz, &nr) != GD_OK) {
        g_err = saved;
        g_status = saved_st;
        return GD_HOST_NOPACK;
      }
    }
    gd_pchrom &q = pc[c];
    std::memset(&q, 0, sizeof q);
    q.row_off = rows;
    q.a_word = wa_tot;
    q.b_word = wb_tot;
    q.nrows = nr;
    q.asize = asz > 0 ? asz : 1;
    q.bsize = bsz > 0 ? bsz : 1;
    q.regend = h.regend;
    q.w_out = h.w_out;
    q.seed = h.seed;
    rows += nr;
    wa_tot += (int64_t)nr * GD_PACK_WORDS(q.asize);
    wb_tot += (int64_t)nr * GD_PACK_WORDS(q.bsize);
    nw = std::max<int64_t>(nw, h.w_out + std::max(h.regend, 0) / wstep);
  }
  if (nw == 0) return GD_OK;
  /* an earlier call that returned between its uploads (a failed HIP call) may have left DMA
   * reading the pinned buffer: drain it before the packer threads overwrite it */
  if (ctx->pack_inflight) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->pack_inflight = false;
  }
  /* pinned layout: A codes, B codes, row positions */
  const size_t ba = sizeof(uint64_t) * std::max<int64_t>(wa_tot, 1), bb = sizeof(uint64_t) * std::max<int64_t>(wb_tot, 1);
  const size_t br = sizeof(int32_t) * std::max<int64_t>(rows, 1), need = ba + bb + br + 512;
  if (need > ctx->h_pack_cap) {
    HIP_TRY(hipStreamSynchronize(ctx->stream)); /* no copy out of the old buffer is in flight */
    if (ctx->h_pack) (void)hipHostFree(ctx->h_pack);
    ctx->h_pack = nullptr;
    ctx->h_pack_cap = 0;
    const size_t cap = need + need / 4;
    HIP_TRY(hipHostMalloc(&ctx->h_pack, cap));
    ctx->h_pack_cap = cap;
  }
  uint64_t *hac = reinterpret_cast<uint64_t *>(ctx->h_pack), *hbc = hac + ba / 8;
  int32_t *hrp = reinterpret_cast<int32_t *>(hbc + bb / 8);
  int st;
  const size_t dneed = ba + bb + br + 2 * sizeof(double) * nw + 1024;
  if ((st = grow(&ctx->io, &ctx->io_cap, dneed))) return st;
  Carve k{ctx->io};
  uint64_t *ca = k.take<uint64_t>(ba / 8), *cb = k.take<uint64_t>(bb / 8);
  int32_t *rp = k.take<int32_t>(br / 4);
  double *o0 = k.take<double>(nw), *o1 = k.take<double>(nw);
  hipStream_t s = ctx->stream;
  HIP_TRY(hipMemcpyAsync(o0, out0, sizeof(double) * nw, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(o1, out1, sizeof(double) * nw, hipMemcpyHostToDevice, s));
  /* chunks of ~8M genotypes: chunk j's codes cross PCIe (DMA from pinned memory) while the
   * host threads pack chunk j + 1 */
  ctx->pack_inflight = true;
  for (int c = 0; c < nchrom; ++c) {
    const gd_chrom &h = chroms[c];
    const gd_pchrom &q = pc[c];
    if (q.nrows == 0) continue;
    const int wa = GD_PACK_WORDS(q.asize), wb = GD_PACK_WORDS(q.bsize);
    const int64_t chunk = std::max<int64_t>(1, ((int64_t)8 << 20) / (q.asize + q.bsize));
    for (int64_t r0 = 0; r0 < q.nrows; r0 += chunk) {
      const int64_t r1 = std::min<int64_t>(q.nrows, r0 + chunk);
      const std::string saved = g_err;
      const int saved_st = g_status;
      if (gd_pack_rows_mt(avals + h.a_off, bvals + h.b_off, apos + h.a_off, bpos + h.b_off, q.asize, q.bsize, r0, r1,
                          hac + q.a_word, hbc + q.b_word, hrp + q.row_off) != GD_OK) {
        g_err = saved;
        g_status = saved_st;
        HIP_TRY(hipStreamSynchronize(s)); /* the chunks already on their way read the pinned buffer */
        ctx->pack_inflight = false;
        return GD_HOST_NOPACK;
      }
      HIP_TRY(hipMemcpyAsync(ca + q.a_word + r0 * wa, hac + q.a_word + r0 * wa, sizeof(uint64_t) * (r1 - r0) * wa,
                             hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(cb + q.b_word + r0 * wb, hbc + q.b_word + r0 * wb, sizeof(uint64_t) * (r1 - r0) * wb,
                             hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(rp + q.row_off + r0, hrp + q.row_off + r0, sizeof(int32_t) * (r1 - r0),
                             hipMemcpyHostToDevice, s));
    }
  }
  const PackedIn pk{pc.data(), ca, cb, rp};
  if ((st = run(ctx, pk, nchrom, o0, o1, s))) {
    if (hipStreamSynchronize(s) == hipSuccess) ctx->pack_inflight = false; /* the pinned buffer may still be read */
    return st;
  }
  HIP_TRY(hipMemcpyAsync(out0, o0, sizeof(double) * nw, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(out1, o1, sizeof(double) * nw, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  ctx->pack_inflight = false;
  return GD_OK;
}

/* one chromosome from host memory: H2D, device scan, D2H of the outputs; packed when the
 * tracks allow it and the call passes a packed runner (host_packed) */
struct NoPack {};
template <class Run, class RunP = NoPack>
static int host_scan(const double *avals, const double *bvals, const int *apos, const int *bpos, int regend,
                     int wsize, int wstep, int alen, int blen, double *out0, double *out1, uint64_t seed, Run run,
                     RunP runp = NoPack{}) {
  if (wsize <= 0 || wstep <= 0) return fail(GD_ERR_ARG, "wsize and wstep must be positive");
  if (alen < 0 || blen < 0) return fail(GD_ERR_ARG, "negative array length");
  if (alen == 0 || blen == 0 || regend <= 0) return GD_OK;
  if (!avals || !bvals || !apos || !bpos || !out0 || !out1) return fail(GD_ERR_ARG, "null buffer");
  int st;
  gd_ctx *ctx = default_ctx(&st);
  if (!ctx) return fail(GD_ERR_HIP, "no HIP device available");
  std::lock_guard<std::mutex> g(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->device));
  if constexpr (!std::is_same<RunP, NoPack>::value) {
    gd_chrom one;
    std::memset(&one, 0, sizeof one);
    one.alen = alen;
    one.blen = blen;
    one.regend = regend;
    one.seed = seed;
    st = host_packed(ctx, &one, 1, avals, bvals, apos, bpos, wstep, out0, out1, runp);
    if (st != GD_HOST_NOPACK) return st;
  }
  const int64_t nwin = regend / wstep;
  Carve cv{nullptr};
  auto lay = [&](Carve &k, double **av, double **bv, int32_t **ap, int32_t **bp, double **o0, double **o1) {
    *av = k.take<double>(alen);
    *bv = k.take<double>(blen);
    *ap = k.take<int32_t>(alen);
    *bp = k.take<int32_t>(blen);
    *o0 = k.take<double>(std::max<int64_t>(nwin, 1));
    *o1 = k.take<double>(std::max<int64_t>(nwin, 1));
  };
  double *av, *bv, *o0, *o1;
  int32_t *ap, *bp;
  lay(cv, &av, &bv, &ap, &bp, &o0, &o1);
  if ((st = grow(&ctx->io, &ctx->io_cap, cv.off))) return st;
  Carve real{ctx->io};
  lay(real, &av, &bv, &ap, &bp, &o0, &o1);
  hipStream_t s = ctx->stream;
  HIP_TRY(hipMemcpyAsync(av, avals, sizeof(double) * alen, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(bv, bvals, sizeof(double) * blen, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(ap, apos, sizeof(int32_t) * alen, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(bp, bpos, sizeof(int32_t) * blen, hipMemcpyHostToDevice, s));
  if (nwin > 0) {
    HIP_TRY(hipMemcpyAsync(o0, out0, sizeof(double) * nwin, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(o1, out1, sizeof(double) * nwin, hipMemcpyHostToDevice, s));
  }
  gd_chrom ch;
  std::memset(&ch, 0, sizeof ch);
  ch.alen = alen;
  ch.blen = blen;
  ch.regend = regend;
  ch.seed = seed;
  st = run(ctx, &ch, av, bv, ap, bp, o0, o1, s);
  if (st) return st;
  if (nwin > 0) {
    HIP_TRY(hipMemcpyAsync(out0, o0, sizeof(double) * nwin, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(out1, o1, sizeof(double) * nwin, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return GD_OK;
}

static int css_scan_locked(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                           const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize, int wstep,
                           int treshold, int runs, int drosophila, int mds, int window_set, double *scores, double *p,
                           hipStream_t s, const PackedIn *pk = nullptr, double *x_out = nullptr);

/* several chromosomes from host memory in one device scan: H2D of the inputs and of
 * the caller's outputs (kept at uncomputed windows), the batched scan, D2H */
template <class Run, class RunP = NoPack>
static int host_batch(const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals, const int *apos,
                      const int *bpos, int wstep, double *out0, double *out1, Run run, RunP runp = NoPack{}) {
  if (nchrom < 0 || (nchrom > 0 && !chroms)) return fail(GD_ERR_ARG, "bad chromosome list");
  if (wstep <= 0) return fail(GD_ERR_ARG, "wsize and wstep must be positive");
  int64_t na = 0, nb = 0, nw = 0;
  for (int c = 0; c < nchrom; ++c) {
    const gd_chrom &h = chroms[c];
    if (h.alen < 0 || h.blen < 0 || h.a_off < 0 || h.b_off < 0 || h.w_out < 0)
      return fail(GD_ERR_ARG, "negative extent");
    na = std::max<int64_t>(na, h.a_off + h.alen);
    nb = std::max<int64_t>(nb, h.b_off + h.blen);
    /* the caller's output span of this descriptor: its window range (window-range shards) */
    const int64_t span = std::max<int64_t>(0, std::max(h.regend, 0) / wstep - std::max(h.w_first, 0));
    nw = std::max<int64_t>(nw, h.w_out + (h.w_count > 0 ? std::min<int64_t>(h.w_count, span) : span));
  }
  if (nchrom == 0 || nw == 0) return GD_OK;
  if (!avals || !bvals || !apos || !bpos || !out0 || !out1) return fail(GD_ERR_ARG, "null buffer");
  int st;
  gd_ctx *ctx = default_ctx(&st);
  if (!ctx) return fail(GD_ERR_HIP, "no HIP device available");
  std::lock_guard<std::mutex> g(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->device));
  if constexpr (!std::is_same<RunP, NoPack>::value) {
    st = host_packed(ctx, chroms, nchrom, avals, bvals, apos, bpos, wstep, out0, out1, runp);
    if (st != GD_HOST_NOPACK) return st;
  }
  Carve cv{nullptr};
  auto lay = [&](Carve &k, double **av, double **bv, int32_t **ap, int32_t **bp, double **o0, double **o1) {
    *av = k.take<double>(std::max<int64_t>(na, 1));
    *bv = k.take<double>(std::max<int64_t>(nb, 1));
    *ap = k.take<int32_t>(std::max<int64_t>(na, 1));
    *bp = k.take<int32_t>(std::max<int64_t>(nb, 1));
    *o0 = k.take<double>(nw);
    *o1 = k.take<double>(nw);
  };
  double *av, *bv, *o0, *o1;
  int32_t *ap, *bp;
  lay(cv, &av, &bv, &ap, &bp, &o0, &o1);
  if ((st = grow(&ctx->io, &ctx->io_cap, cv.off))) return st;
  Carve real{ctx->io};
  lay(real, &av, &bv, &ap, &bp, &o0, &o1);
  hipStream_t s = ctx->stream;
  if (na) {
    HIP_TRY(hipMemcpyAsync(av, avals, sizeof(double) * na, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ap, apos, sizeof(int32_t) * na, hipMemcpyHostToDevice, s));
  }
  if (nb) {
    HIP_TRY(hipMemcpyAsync(bv, bvals, sizeof(double) * nb, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(bp, bpos, sizeof(int32_t) * nb, hipMemcpyHostToDevice, s));
  }
  HIP_TRY(hipMemcpyAsync(o0, out0, sizeof(double) * nw, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(o1, out1, sizeof(double) * nw, hipMemcpyHostToDevice, s));
  st = run(ctx, av, bv, ap, bp, o0, o1, s);
  if (st) return st;
  HIP_TRY(hipMemcpyAsync(out0, o0, sizeof(double) * nw, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(out1, o1, sizeof(double) * nw, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return GD_OK;
}

extern "C" int gd_fet_scan_host_batch_ex(const gd_chrom *chroms, int nchrom, const double *avals,
                                         const double *bvals, const int *apos, const int *bpos, int wsize, int wstep,
                                         double perc, int mode, int window_set, double *scores, double *stddev) {
  return host_batch(chroms, nchrom, avals, bvals, apos, bpos, wstep, scores, stddev,
                    [&](gd_ctx *ctx, double *av, double *bv, int32_t *ap, int32_t *bp, double *o0, double *o1,
                        hipStream_t s) {
                      return fet_scan_locked(ctx, chroms, nchrom, av, bv, ap, bp, wsize, wstep, perc, mode,
                                             window_set, o0, o1, s);
                    },
                    [&](gd_ctx *ctx, const PackedIn &pk, int n, double *o0, double *o1, hipStream_t s) {
                      return fet_scan_locked(ctx, nullptr, n, nullptr, nullptr, nullptr, nullptr, wsize, wstep, perc,
                                             mode, window_set, o0, o1, s, &pk);
                    });
}

extern "C" int gd_fet_scan_host_batch(const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                                      const int *apos, const int *bpos, int wsize, int wstep, double perc,
                                      int window_set, double *scores, double *stddev) {
  return gd_fet_scan_host_batch_ex(chroms, nchrom, avals, bvals, apos, bpos, wsize, wstep, perc, g_fet_mode.load(),
                                   window_set, scores, stddev);
}

extern "C" int gd_css_scan_host_batch_ex(const gd_chrom *chroms, int nchrom, const double *avals,
                                         const double *bvals, const int *apos, const int *bpos, int wsize, int wstep,
                                         int treshold, int runs, int drosophila, int mds, int window_set,
                                         double *scores, double *p) {
  auto ref = [&](gd_ctx *ctx, double *av, double *bv, int32_t *ap, int32_t *bp, double *o0, double *o1,
                 hipStream_t s) {
    return css_scan_locked(ctx, chroms, nchrom, av, bv, ap, bp, wsize, wstep, treshold, runs, drosophila, mds,
                           window_set, o0, o1, s);
  };
  if (drosophila) /* allele frequencies, not genotype codes: the reference layout */
    return host_batch(chroms, nchrom, avals, bvals, apos, bpos, wstep, scores, p, ref);
  return host_batch(chroms, nchrom, avals, bvals, apos, bpos, wstep, scores, p, ref,
                    [&](gd_ctx *ctx, const PackedIn &pk, int n, double *o0, double *o1, hipStream_t s) {
                      return css_scan_locked(ctx, nullptr, n, nullptr, nullptr, nullptr, nullptr, wsize, wstep,
                                             treshold, runs, 0, mds, window_set, o0, o1, s, &pk);
                    });
}

extern "C" int gd_css_scan_host_batch(const gd_chrom *chroms, int nchrom, const double *avals, const double *bvals,
                                      const int *apos, const int *bpos, int wsize, int wstep, int treshold,
                                      int runs, int window_set, double *scores, double *p) {
  return gd_css_scan_host_batch_ex(chroms, nchrom, avals, bvals, apos, bpos, wsize, wstep, treshold, runs, 0, 0,
                                   window_set, scores, p);
}

extern "C" int gd_fet_scan_host_ex(const double *avals, const double *bvals, const int *apos, const int *bpos,
                                   int regend, int wsize, int wstep, int alen, int blen, double perc, int mode,
                                   uint64_t seed, int window_set, double *scores, double *stddev) {
  if (mode != GD_FET_REFERENCE && mode != GD_FET_EXACT)
    return fail(GD_ERR_ARG, "FET mode must be GD_FET_REFERENCE (0) or GD_FET_EXACT (1)");
  return host_scan(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, scores, stddev, seed,
                   [&](gd_ctx *ctx, gd_chrom *ch, double *av, double *bv, int32_t *ap, int32_t *bp, double *o0,
                       double *o1, hipStream_t s) {
                     return fet_scan_locked(ctx, ch, 1, av, bv, ap, bp, wsize, wstep, perc, mode, window_set, o0,
                                            o1, s);
                   },
                   [&](gd_ctx *ctx, const PackedIn &pk, int n, double *o0, double *o1, hipStream_t s) {
                     return fet_scan_locked(ctx, nullptr, n, nullptr, nullptr, nullptr, nullptr, wsize, wstep, perc,
                                            mode, window_set, o0, o1, s, &pk);
                   });
}

extern "C" int gd_fet_scan_host(const double *avals, const double *bvals, const int *apos, const int *bpos,
                                int regend, int wsize, int wstep, int alen, int blen, double perc, uint64_t seed,
                                int window_set, double *scores, double *stddev) {
  return gd_fet_scan_host_ex(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, perc, g_fet_mode.load(),
                             seed, window_set, scores, stddev);
}

extern "C" int gd_fet_threadcompute(const double *avals, const double *bvals, const int *apos, const int *bpos,
                                    int regstart, int regend, int wsize, int wstep, int alen, int blen,
                                    double perc, double *scores, double *stddev) {
  (void)regstart; /* ignored by the reference too (threadfisher.c:110) */
  return gd_fet_scan_host(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, perc, g_seed,
                          GD_WINDOWS_THREADED, scores, stddev);
}

extern "C" int gd_fet_compute(const double *avals, const double *bvals, const int *apos, const int *bpos,
                              int regstart, int regend, int wsize, int wstep, int alen, int blen, double perc,
                              double *scores, double *stddev) {
  (void)regstart; /* ignored by the reference too (cFisher.c:60) */
  return gd_fet_scan_host(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, perc, g_seed,
                          GD_WINDOWS_SERIAL, scores, stddev);
}

/* --------------------------------------------------------------- CSS scan */
/* pk != NULL: a packed batch (count metric only) */
static int css_scan_locked(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                           const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize, int wstep,
                           int treshold, int runs, int drosophila, int mds, int window_set, double *scores, double *p,
                           hipStream_t s, const PackedIn *pk, double *x_out) {
  if (drosophila != 0 && drosophila != 1) return fail(GD_ERR_ARG, "drosophila must be 0 or 1");
  if (mds < 0 || mds > 2) return fail(GD_ERR_ARG, "mds must be 0 (classical), 1 (SMACOF) or 2 (SMACOF + classical)");
  if (pk && drosophila)
    return fail(GD_ERR_ARG, "packed tracks carry genotype codes, not the drosophila allele frequencies");
  ScanPlan pl;
  std::vector<int64_t> row_off, word_off;
  int64_t max_rows = 1;
  int st = pk ? make_plan_packed(*pk, nchrom, wsize, wstep, window_set, &pl, &row_off, &word_off, &max_rows)
              : make_plan(chroms, nchrom, wsize, wstep, window_set, &pl);
  if (st) return st;
  for (float &m : g_stage_ms) m = 0.f;
  if (pl.wtotal == 0) return GD_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  /* pass 1: population sizes + window bounds; the CSS kernels are specialised on
   * m = asize + bsize and the bit planes are sized by it, so read the sizes back */
  Carve cv{nullptr};
  int64_t *d_roff = nullptr, *d_woff = nullptr; /* packed batches: row and word offsets */
  auto layout1 = [&](Carve &k, gd_chrom_dev **d_ch, unsigned **flags, int32_t **lo_a, int32_t **hi_a,
                     int32_t **lo_b) {
    *d_ch = k.take<gd_chrom_dev>(nchrom);
    *flags = k.take<unsigned>(16);
    *lo_a = k.take<int32_t>(pl.wtotal);
    *hi_a = k.take<int32_t>(pl.wtotal);
    *lo_b = k.take<int32_t>(pl.wtotal);
    if (pk) {
      d_roff = k.take<int64_t>(nchrom);
      d_woff = k.take<int64_t>(2 * (size_t)nchrom);
    }
  };
  gd_chrom_dev *d_ch;
  unsigned *flags;
  int32_t *lo_a, *hi_a, *lo_b;
  layout1(cv, &d_ch, &flags, &lo_a, &hi_a, &lo_b);
  const size_t fixed = cv.off;
  if ((st = grow(&ctx->ws, &ctx->ws_cap, fixed))) return st;
  {
    Carve real{ctx->ws};
    layout1(real, &d_ch, &flags, &lo_a, &hi_a, &lo_b);
  }
  HIP_TRY(hipMemcpyAsync(d_ch, pl.h.data(), sizeof(gd_chrom_dev) * nchrom, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(flags, 0, 16 * sizeof(unsigned), s));
  HIP_TRY(hipEventRecord(ctx->ev[0], s));
  if (pk) {
    HIP_TRY(hipMemcpyAsync(d_roff, row_off.data(), sizeof(int64_t) * nchrom, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_woff, word_off.data(), sizeof(int64_t) * 2 * nchrom, hipMemcpyHostToDevice, s));
    if ((st = gd_packed_bounds_launch(d_ch, nchrom, d_roff, pk->rowpos, max_rows, wsize, wstep, lo_a, hi_a, lo_b,
                                      flags, s)))
      return fail(st, "packed bounds launch failed");
  } else {
    hipLaunchKernelGGL(k_popsize, dim3(nchrom), dim3(64), 0, s, d_ch, apos, bpos, flags);
    const int64_t mx = std::max(pl.max_alen, pl.max_blen) + 1;
    const int64_t epb = gd_bounds_elems_per_block();
    const unsigned gx = (unsigned)std::min<int64_t>((mx + epb - 1) / epb, std::max(1, 8192 / nchrom));
    hipLaunchKernelGGL(k_bounds, dim3(gx, nchrom, 2), dim3(256), 0, s, d_ch, apos, bpos, wsize, wstep, lo_a,
                       hi_a, lo_b, flags);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(pl.h.data(), d_ch, sizeof(gd_chrom_dev) * nchrom, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(ctx->h_flags, flags, 16 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if ((st = flags_to_status(ctx->h_flags[0]))) return st;

  /* pass 2: bit planes, per-window MDS, permutations */
  int mmax = 0;
  int64_t words = 0, max_words = 1;
  std::vector<gd_css_planes> hp(nchrom);
  for (int c = 0; c < nchrom; ++c) {
    const gd_chrom_dev &d = pl.h[c];
    gd_css_planes &q = hp[c];
    std::memset(&q, 0, sizeof q);
    if (d.wend <= 0 || d.asize <= 0 || d.bsize <= 0) continue;
    mmax = std::max(mmax, d.asize + d.bsize);
    const int64_t wa = ((int64_t)d.alen / d.asize + 31) / 32 + 3, wb = ((int64_t)d.blen / d.bsize + 31) / 32 + 3;
    if (wa > INT32_MAX || wb > INT32_MAX) return fail(GD_ERR_SIZE, "chromosome too long");
    q.wa = (int32_t)wa;
    q.wb = (int32_t)wb;
    q.pa = words;
    words += (2 * (int64_t)d.asize + 1) * wa;
    q.pb = words;
    words += (2 * (int64_t)d.bsize + 1) * wb;
    max_words = std::max(max_words, std::max(wa * d.asize, wb * d.bsize));
  }
  const int mp = gd_css_tier(mmax);
  if (mp == 0) return fail(GD_ERR_SIZE, "asize + bsize above the largest supported cohort (GD_CSS_BIG_MAX = 2048)");
  if (mds != 0 && mp > GD_CSS_SMACOF_MAX)
    return fail(GD_ERR_SIZE, "SMACOF (mds 1 / 2) above the largest supported cohort (GD_CSS_SMACOF_MAX)");
  /* the general path (m above the register tiers): one matrix slab per workgroup */
  const int64_t slab_doubles = mp > GD_CSS_TIER_MAX ? gd_css_big_grid(pl.wtotal, mp) * gd_css_big_slab_per_wg(mp) : 1;
  if (drosophila)
    for (int c = 0; c < nchrom; ++c) {
      const gd_chrom_dev &d = pl.h[c];
      if (d.wend > 0 && d.asize > 0 && d.bsize > 0 && (d.asize != 1 || d.bsize != 1))
        return fail(GD_ERR_ARG, "the drosophila metric compares one allele frequency per population "
                                "(asize = bsize = 1; compare_freq, css.c:245-264)");
    }
  const bool perms = (runs > 0 && treshold > 0) || mds == 2; /* xbuf/status carry coordinates */
  auto layout2 = [&](Carve &k, gd_css_planes **d_pl, uint32_t **planes, double **xbuf, uint8_t **status,
                     double **slab) {
    layout1(k, &d_ch, &flags, &lo_a, &hi_a, &lo_b);
    *d_pl = k.take<gd_css_planes>(nchrom);
    *planes = k.take<uint32_t>(std::max<int64_t>(words, 1));
    *xbuf = k.take<double>(perms ? pl.wtotal * 2 * mp : 1);
    *status = k.take<uint8_t>(perms ? pl.wtotal : 1);
    *slab = k.take<double>(slab_doubles);
  };
  gd_css_planes *d_pl;
  uint32_t *planes;
  double *xbuf, *slab;
  uint8_t *status;
  Carve cv2{nullptr};
  layout2(cv2, &d_pl, &planes, &xbuf, &status, &slab);
  if (cv2.off > ctx->ws_cap) {
    /* growing reallocates: keep the pass-1 results (descriptors, flags, bounds) */
    char *old = ctx->ws;
    ctx->ws = nullptr;
    ctx->ws_cap = 0;
    if ((st = grow(&ctx->ws, &ctx->ws_cap, cv2.off))) {
      (void)hipFree(old);
      return st;
    }
    HIP_TRY(hipMemcpyAsync(ctx->ws, old, fixed, hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    (void)hipFree(old);
  }
  {
    Carve real{ctx->ws};
    layout2(real, &d_pl, &planes, &xbuf, &status, &slab);
  }
  HIP_TRY(hipMemcpyAsync(d_ch, pl.h.data(), sizeof(gd_chrom_dev) * nchrom, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_pl, hp.data(), sizeof(gd_css_planes) * nchrom, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(planes, 0, sizeof(uint32_t) * std::max<int64_t>(words, 1), s));
  if (perms) HIP_TRY(hipMemsetAsync(status, 0, pl.wtotal, s));
  HIP_TRY(hipEventRecord(ctx->ev[1], s));
  st = gd_css_launch(mp, drosophila, mds, d_ch, nchrom, d_pl, planes, lo_a, hi_a, lo_b, avals, bvals, d_woff,
                     pk ? pk->acodes : nullptr, pk ? pk->bcodes : nullptr, pl.wtotal, max_words, treshold, runs,
                     scores, p, xbuf, status, flags, slab, s, ctx->ev[2]);
  if (st) return fail(st, "CSS kernel launch failed");
  HIP_TRY(hipEventRecord(ctx->ev[3], s));
  if (x_out && perms) {
    /* diagnostics (gd_css_coords_host): the coordinates the permutation stage read, one
     * row of 2 m doubles per window of the batch (xbuf rows are 2 mp wide) */
    HIP_TRY(hipMemcpy2DAsync(x_out, sizeof(double) * 2 * mmax, xbuf, sizeof(double) * 2 * mp,
                             sizeof(double) * 2 * mmax, pl.wtotal, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipMemcpyAsync(ctx->h_flags, flags, 16 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  float ms;
  if (hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]) == hipSuccess) g_stage_ms[GD_STAGE_MEM] = ms;
  /* CSS stages: MEM = population sizes + bounds, WINDOW = bit planes + MDS (+ SMACOF),
   * GENERAL = the permutation test */
  if (hipEventElapsedTime(&ms, ctx->ev[1], ctx->ev[2]) == hipSuccess) g_stage_ms[GD_STAGE_WINDOW] = ms;
  if (hipEventElapsedTime(&ms, ctx->ev[2], ctx->ev[3]) == hipSuccess) g_stage_ms[GD_STAGE_GENERAL] = ms;
  if (hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[3]) == hipSuccess) g_stage_ms[GD_STAGE_TOTAL] = ms;
  return flags_to_status(ctx->h_flags[0]);
}

/* CSS needs the window bounds and sizes laid out by css_scan_locked; the
 * pipeline reads them back from the context's workspace */
extern "C" int gd_css_scan_device_ex(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                                     const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize,
                                     int wstep, int treshold, int runs, int drosophila, int mds, int window_set,
                                     double *scores, double *p, void *hip_stream) {
  if (!ctx) return fail(GD_ERR_ARG, "null context");
  std::lock_guard<std::mutex> g(ctx->mu);
  return css_scan_locked(ctx, chroms, nchrom, avals, bvals, apos, bpos, wsize, wstep, treshold, runs, drosophila, mds,
                         window_set, scores, p, (hipStream_t)hip_stream);
}

extern "C" int gd_css_scan_device(gd_ctx *ctx, const gd_chrom *chroms, int nchrom, const double *avals,
                                  const double *bvals, const int32_t *apos, const int32_t *bpos, int wsize,
                                  int wstep, int treshold, int runs, int window_set, double *scores, double *p,
                                  void *hip_stream) {
  return gd_css_scan_device_ex(ctx, chroms, nchrom, avals, bvals, apos, bpos, wsize, wstep, treshold, runs, 0, 0,
                               window_set, scores, p, hip_stream);
}

extern "C" int gd_css_scan_host_ex(const double *avals, const double *bvals, const int *apos, const int *bpos,
                                   int regend, int wsize, int wstep, int alen, int blen, int treshold, int runs,
                                   int drosophila, int mds, uint64_t seed, int window_set, double *scores,
                                   double *p) {
  auto ref = [&](gd_ctx *ctx, gd_chrom *ch, double *av, double *bv, int32_t *ap, int32_t *bp, double *o0,
                 double *o1, hipStream_t s) {
    return css_scan_locked(ctx, ch, 1, av, bv, ap, bp, wsize, wstep, treshold, runs, drosophila, mds, window_set, o0,
                           o1, s);
  };
  if (drosophila) /* allele frequencies, not genotype codes: the reference layout */
    return host_scan(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, scores, p, seed, ref);
  return host_scan(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, scores, p, seed, ref,
                   [&](gd_ctx *ctx, const PackedIn &pk, int n, double *o0, double *o1, hipStream_t s) {
                     return css_scan_locked(ctx, nullptr, n, nullptr, nullptr, nullptr, nullptr, wsize, wstep,
                                            treshold, runs, 0, mds, window_set, o0, o1, s, &pk);
                   });
}

extern "C" int gd_css_coords_host(const double *avals, const double *bvals, const int *apos, const int *bpos,
                                  int regend, int wsize, int wstep, int alen, int blen, int treshold, int runs,
                                  int mds, uint64_t seed, int window_set, double *scores, double *p, double *X) {
  if (runs <= 0 || treshold <= 0) return fail(GD_ERR_ARG, "coordinates are kept only for a permutation test");
  if (!X) return fail(GD_ERR_ARG, "null buffer");
  return host_scan(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, scores, p, seed,
                   [&](gd_ctx *ctx, gd_chrom *ch, double *av, double *bv, int32_t *ap, int32_t *bp, double *o0,
                       double *o1, hipStream_t s) {
                     return css_scan_locked(ctx, ch, 1, av, bv, ap, bp, wsize, wstep, treshold, runs, 0, mds,
                                            window_set, o0, o1, s, nullptr, X);
                   });
}

extern "C" int gd_css_scan_host(const double *avals, const double *bvals, const int *apos, const int *bpos,
                                int regend, int wsize, int wstep, int alen, int blen, int treshold, int runs,
                                uint64_t seed, int window_set, double *scores, double *p) {
  return gd_css_scan_host_ex(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, treshold, runs, 0, 0, seed,
                             window_set, scores, p);
}

extern "C" int gd_css_threadcompute(const double *avals, const double *bvals, const int *apos, const int *bpos,
                                    int regstart, int regend, int wsize, int wstep, int alen, int blen,
                                    int treshold, int runs, int drosophila, int mds, double *scores, double *p) {
  (void)regstart; /* ignored by the reference too (threadcss.c) */
  return gd_css_scan_host_ex(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, treshold, runs, drosophila,
                             mds, g_seed, GD_WINDOWS_THREADED, scores, p);
}

extern "C" int gd_css_compute(const double *avals, const double *bvals, const int *apos, const int *bpos,
                              int regstart, int regend, int wsize, int wstep, int alen, int blen, int treshold,
                              int runs, int drosophila, int mds, double *scores, double *p) {
  (void)regstart; /* ignored by the reference too (css.c:78) */
  return gd_css_scan_host_ex(avals, bvals, apos, bpos, regend, wsize, wstep, alen, blen, treshold, runs, drosophila,
                             mds, g_seed, GD_WINDOWS_SERIAL, scores, p);
}

/* ------------------------------------------------------------- utilities */
extern "C" void gd_set_seed(uint64_t seed) { g_seed = seed; }
extern "C" uint64_t gd_get_seed(void) { return g_seed; }
/* ------------------------------------------------------------ packed tracks */
extern "C" int gd_fet_scan_packed_device(gd_ctx *ctx, const gd_pchrom *chroms, int nchrom, const uint64_t *acodes,
                                         const uint64_t *bcodes, const int32_t *rowpos, int wsize, int wstep,
                                         double perc, int mode, int window_set, double *scores, double *stddev,
                                         void *hip_stream) {
  if (!ctx) return fail(GD_ERR_ARG, "null context");
  std::lock_guard<std::mutex> g(ctx->mu);
  const PackedIn pk{chroms, acodes, bcodes, rowpos};
  return fet_scan_locked(ctx, nullptr, nchrom, nullptr, nullptr, nullptr, nullptr, wsize, wstep, perc, mode,
                         window_set, scores, stddev, (hipStream_t)hip_stream, &pk);
}

extern "C" int gd_css_scan_packed_device(gd_ctx *ctx, const gd_pchrom *chroms, int nchrom, const uint64_t *acodes,
                                         const uint64_t *bcodes, const int32_t *rowpos, int wsize, int wstep,
                                         int treshold, int runs, int mds, int window_set, double *scores, double *p,
                                         void *hip_stream) {
  if (!ctx) return fail(GD_ERR_ARG, "null context");
  std::lock_guard<std::mutex> g(ctx->mu);
  const PackedIn pk{chroms, acodes, bcodes, rowpos};
  return css_scan_locked(ctx, nullptr, nchrom, nullptr, nullptr, nullptr, nullptr, wsize, wstep, treshold, runs, 0,
                         mds, window_set, scores, p, (hipStream_t)hip_stream, &pk);
}

/* a packed batch from host memory: H2D of the codes, positions and the caller's outputs
 * (kept at uncomputed windows), the device scan, D2H */
template <class Run>
static int packed_host(const gd_pchrom *chroms, int nchrom, const uint64_t *acodes, const uint64_t *bcodes,
                       const int32_t *rowpos, int wstep, double *out0, double *out1, Run run) {
  if (nchrom < 0 || (nchrom > 0 && !chroms)) return fail(GD_ERR_ARG, "bad chromosome list");
  if (wstep <= 0) return fail(GD_ERR_ARG, "wsize and wstep must be positive");
  int64_t nrow = 0, nwa = 0, nwb = 0, nw = 0;
  for (int c = 0; c < nchrom; ++c) {
    const gd_pchrom &q = chroms[c];
    if (q.nrows < 0 || q.row_off < 0 || q.a_word < 0 || q.b_word < 0 || q.w_out < 0)
      return fail(GD_ERR_ARG, "negative extent");
    if (q.nrows > 0 && (q.asize <= 0 || q.bsize <= 0)) return fail(GD_ERR_SIZE, "empty population");
    nrow = std::max<int64_t>(nrow, q.row_off + q.nrows);
    nwa = std::max<int64_t>(nwa, q.a_word + (int64_t)q.nrows * GD_PACK_WORDS(std::max(q.asize, 0)));
    nwb = std::max<int64_t>(nwb, q.b_word + (int64_t)q.nrows * GD_PACK_WORDS(std::max(q.bsize, 0)));
    if (q.regend > 0) nw = std::max<int64_t>(nw, q.w_out + q.regend / wstep);
  }
  if (nrow == 0 || nw == 0) return GD_OK;
  if (!acodes || !bcodes || !rowpos || !out0 || !out1) return fail(GD_ERR_ARG, "null buffer");
  int st;
  gd_ctx *ctx = default_ctx(&st);
  if (!ctx) return st ? st : fail(GD_ERR_HIP, "no HIP device available");
  std::lock_guard<std::mutex> g(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t need = sizeof(uint64_t) * (nwa + nwb) + sizeof(int32_t) * nrow + 2 * sizeof(double) * nw + 1024;
  if ((st = grow(&ctx->io, &ctx->io_cap, need))) return st;
  Carve k{ctx->io};
  uint64_t *ca = k.take<uint64_t>(nwa), *cb = k.take<uint64_t>(nwb);
  int32_t *rp = k.take<int32_t>(nrow);
  double *o0 = k.take<double>(nw), *o1 = k.take<double>(nw);
  hipStream_t s = ctx->stream;
  HIP_TRY(hipMemcpyAsync(ca, acodes, sizeof(uint64_t) * nwa, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(cb, bcodes, sizeof(uint64_t) * nwb, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(rp, rowpos, sizeof(int32_t) * nrow, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(o0, out0, sizeof(double) * nw, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(o1, out1, sizeof(double) * nw, hipMemcpyHostToDevice, s));
  const PackedIn pk{chroms, ca, cb, rp};
  if ((st = run(ctx, pk, o0, o1, s))) return st;
  HIP_TRY(hipMemcpyAsync(out0, o0, sizeof(double) * nw, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(out1, o1, sizeof(double) * nw, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return GD_OK;
}

extern "C" int gd_fet_scan_packed_host(const gd_pchrom *chroms, int nchrom, const uint64_t *acodes,
                                       const uint64_t *bcodes, const int32_t *rowpos, int wsize, int wstep,
                                       double perc, int mode, int window_set, double *scores, double *stddev) {
  return packed_host(chroms, nchrom, acodes, bcodes, rowpos, wstep, scores, stddev,
                     [&](gd_ctx *ctx, const PackedIn &pk, double *o0, double *o1, hipStream_t s) {
                       return fet_scan_locked(ctx, nullptr, nchrom, nullptr, nullptr, nullptr, nullptr, wsize, wstep,
                                              perc, mode, window_set, o0, o1, s, &pk);
                     });
}

extern "C" int gd_css_scan_packed_host(const gd_pchrom *chroms, int nchrom, const uint64_t *acodes,
                                       const uint64_t *bcodes, const int32_t *rowpos, int wsize, int wstep,
                                       int treshold, int runs, int mds, int window_set, double *scores, double *p) {
  return packed_host(chroms, nchrom, acodes, bcodes, rowpos, wstep, scores, p,
                     [&](gd_ctx *ctx, const PackedIn &pk, double *o0, double *o1, hipStream_t s) {
                       return css_scan_locked(ctx, nullptr, nchrom, nullptr, nullptr, nullptr, nullptr, wsize, wstep,
                                              treshold, runs, 0, mds, window_set, o0, o1, s, &pk);
                     });
}

extern "C" int gd_pack_chrom_device(const double *avals, const double *bvals, const int32_t *apos,
                                    const int32_t *bpos, int asize, int bsize, int nrows, uint64_t *acodes,
                                    uint64_t *bcodes, int32_t *rowpos, void *hip_stream) {
  if (asize <= 0 || bsize <= 0 || nrows < 0) return fail(GD_ERR_ARG, "population sizes must be positive");
  if (nrows == 0) return GD_OK;
  int st;
  gd_ctx *ctx = default_ctx(&st);
  if (!ctx) return st ? st : fail(GD_ERR_HIP, "no HIP device available");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
  HIP_TRY(hipMemsetAsync(ctx->h_flags_dev, 0, sizeof(unsigned), s));
  if ((st = gd_pack_device_launch(avals, bvals, apos, bpos, asize, bsize, nrows, acodes, bcodes, rowpos,
                                  ctx->h_flags_dev, s)))
    return fail(st, "pack kernel launch failed");
  HIP_TRY(hipMemcpyAsync(ctx->h_flags, ctx->h_flags_dev, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (ctx->h_flags[0]) return fail(GD_ERR_ARG, "a value is not a genotype code or a row's positions differ");
  return GD_OK;
}

extern "C" int gd_set_fet_mode(int mode) {
  if (mode != GD_FET_REFERENCE && mode != GD_FET_EXACT)
    return fail(GD_ERR_ARG, "FET mode must be GD_FET_REFERENCE (0) or GD_FET_EXACT (1)");
  return g_fet_mode.exchange(mode);
}
extern "C" int gd_get_fet_mode(void) { return g_fet_mode.load(); }
extern "C" const char *gd_last_error(void) { return g_err.c_str(); }
extern "C" int gd_last_status(void) { return g_status; }
extern "C" int gd_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
extern "C" int gd_last_stage_ms(float *ms, int n) {
  for (int i = 0; i < n && i < GD_NSTAGES; ++i) ms[i] = g_stage_ms[i];
  return GD_NSTAGES;
}

extern "C" int gd_synth_device(int chrom, int nsnp, int asize, int bsize, uint64_t seed, const double *freq_table,
                               double *avals, double *bvals, int32_t *apos, int32_t *bpos, void *hip_stream) {
  if (nsnp <= 0 || asize <= 0 || bsize <= 0) return fail(GD_ERR_ARG, "bad synthetic sizes");
  return gd_synth_launch(chrom, nsnp, asize, bsize, seed, freq_table, avals, bvals, apos, bpos,
                         (hipStream_t)hip_stream);
}

/* ------------------------------------------------- region filters (gd_regions.hip) */
int gd_rg_fet_limit(const double *scores, const double *stddev, int64_t n, double qnorm, double percentile,
                    double *out, hipStream_t s);
int gd_rg_fdr_threshold(const double *p, int64_t n, double fdr, double *testp, int64_t *k_out, hipStream_t s);
int gd_rg_top_limit(const double *scores, int64_t n, int64_t num_top, double *limit, hipStream_t s);
int gd_rg_merge(const double *vals, const int32_t *seq, const int64_t *start, int64_t n, int cmp, double thr,
                int64_t gap, const int64_t *seq_end, int nseq, int64_t *region_first, int64_t *region_end,
                int64_t *nregions, int64_t *nselected, hipStream_t s);

/* ctx == NULL: the process-wide context of the current HIP device (hipGetDevice); stream NULL: the context's */
template <class F>
static int with_ctx(gd_ctx *ctx, void *hip_stream, F &&f) {
  int st = GD_OK;
  if (!ctx) ctx = default_ctx(&st);
  if (!ctx) return st ? st : fail(GD_ERR_HIP, "no device context");
  std::lock_guard<std::mutex> g(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->device));
  return f(hip_stream ? (hipStream_t)hip_stream : ctx->stream);
}

extern "C" int gd_fet_region_limit(gd_ctx *ctx, const double *scores, const double *stddev, int64_t n,
                                   double qnorm, double percentile, double *out3, void *hip_stream) {
  return with_ctx(ctx, hip_stream,
                  [&](hipStream_t s) { return gd_rg_fet_limit(scores, stddev, n, qnorm, percentile, out3, s); });
}

extern "C" int gd_css_fdr_threshold(gd_ctx *ctx, const double *p, int64_t n, double fdr, double *testp,
                                    int64_t *k, void *hip_stream) {
  return with_ctx(ctx, hip_stream, [&](hipStream_t s) { return gd_rg_fdr_threshold(p, n, fdr, testp, k, s); });
}

extern "C" int gd_css_top_limit(gd_ctx *ctx, const double *scores, int64_t n, int64_t num_top, double *limit,
                                void *hip_stream) {
  return with_ctx(ctx, hip_stream, [&](hipStream_t s) { return gd_rg_top_limit(scores, n, num_top, limit, s); });
}

extern "C" int gd_merge_regions(gd_ctx *ctx, const double *vals, const int32_t *seq, const int64_t *start,
                                int64_t n, int cmp, double thr, int64_t max_gap, const int64_t *seq_end, int nseq,
                                int64_t *region_first, int64_t *region_end, int64_t *nregions, int64_t *nselected,
                                void *hip_stream) {
  return with_ctx(ctx, hip_stream, [&](hipStream_t s) {
    return gd_rg_merge(vals, seq, start, n, cmp, thr, max_gap, seq_end, nseq, region_first, region_end, nregions,
                       nselected, s);
  });
}
