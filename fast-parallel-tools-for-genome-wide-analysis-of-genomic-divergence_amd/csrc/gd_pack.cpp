/*
 * gd_pack.cpp -- host packer of reference-layout tracks into packed genotype tracks
 * (include/gdscan.h, "packed genotype tracks").
 *
 * The reference layout is what HyperBrowser hands the statistics
 * (FisherExactScoreStat.py:35-40): one f64 value and one i32 position per (SNP row,
 * individual), SNP-major, values from VCFConvert.py:8-17 (3, 0, -3, -10000).  The
 * packed form keeps one position per row and a 2-bit code per genotype; it exists only
 * for tracks whose rows are whole (every individual of row r, A and B alike, at the
 * row's position) and whose values are the four codes -- exactly the tracks on which
 * the reference's window slicing (slide_right on A, npos from A, B read by the same row
 * index: SURVEY.md Q4) behaves as a per-row scan.  Anything else is refused with
 * GD_ERR_ARG and keeps the reference layout.
 */
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/gdscan.h"

void gd_set_error(const char *msg); /* gd_api.hip */

namespace {

int pk_fail(int code, const char *msg) {
  gd_set_error(msg);
  return code;
}

/* get_population_size(), comparative.c:25-34: the leading run of pos[0] */
int popsize(const int *pos, int len) {
  int n = 0;
  while (n < len && pos[n] == pos[0]) ++n;
  return n;
}

bool code_of(double x, uint64_t *c) {
  if (x == 3.0)
    *c = GD_CODE_MAJOR;
  else if (x == -3.0)
    *c = GD_CODE_MINOR;
  else if (x == 0.0)
    *c = GD_CODE_HET;
  else if (x == -10000.0)
    *c = GD_CODE_MISSING;
  else
    return false;
  return true;
}

}  // namespace

extern "C" int gd_pack_shape(const int *apos, const int *bpos, int alen, int blen, int *asize, int *bsize,
                             int *nrows) {
  if (alen < 0 || blen < 0 || !asize || !bsize || !nrows) return pk_fail(GD_ERR_ARG, "bad arguments");
  if ((alen > 0 && !apos) || (blen > 0 && !bpos)) return pk_fail(GD_ERR_ARG, "null positions");
  *asize = alen > 0 ? popsize(apos, alen) : 0;
  *bsize = blen > 0 ? popsize(bpos, blen) : 0;
  *nrows = (*asize > 0 && *bsize > 0) ? (alen / *asize < blen / *bsize ? alen / *asize : blen / *bsize) : 0;
  /* a partial trailing row, or A and B holding different row counts, has no packed form
   * (the reference layout reads B past A's rows: GD_ERR_BOUNDS in its scans) */
  if ((int64_t)*nrows * *asize != alen || (int64_t)*nrows * *bsize != blen)
    return pk_fail(GD_ERR_ARG, "the tracks do not consist of whole rows of asize / bsize individuals "
                               "(both populations, the same row count)");
  return GD_OK;
}

/* Rows [r0, r1) of one population, branch-free so the compiler vectorises the value tests:
 * code = 1 (3), 2 (-3), 3 (-10000), 0 (0, or -0); ok stays true only while every value is
 * one of the four and every position equals the row's (rowpos) */
static bool pack_pop_rows(const double *vals, const int *pos, const int32_t *rowpos, int size, int64_t r0, int64_t r1,
                          uint64_t *codes) {
  const int W = GD_PACK_WORDS(size);
  unsigned bad = 0;
  for (int64_t r = r0; r < r1; ++r) {
    const double *v = vals + r * size;
    const int *ps = pos + r * size;
    const int32_t p0 = rowpos[r];
    uint64_t *out = codes + r * W;
    for (int w = 0; w < W; ++w) {
      const int k0 = 32 * w, k1 = std::min(size, k0 + 32);
      uint64_t word = 0;
      for (int k = k0; k < k1; ++k) {
        const double x = v[k];
        const unsigned maj = x == 3.0, mnr = x == -3.0, mis = x == -10000.0, het = x == 0.0;
        bad |= (maj | mnr | mis | het) ^ 1u;
        bad |= (unsigned)(ps[k] != p0);
        word |= (uint64_t)(maj * GD_CODE_MAJOR | mnr * GD_CODE_MINOR | mis * GD_CODE_MISSING) << (2 * (k - k0));
      }
      out[w] = word;
    }
  }
  return bad == 0;
}

/* The same rows four genotypes at a time (AVX2 + BMI2, chosen at run time): the four value
 * tests are vector compares whose movemasks give 4 bits each, pdep spreads "major or
 * missing" to the codes' low bits and "minor or missing" to their high bits, and the
 * positions are one 4-lane compare against the row's */
__attribute__((target("avx2,bmi2"))) static bool pack_pop_rows_avx2(const double *vals, const int *pos,
                                                                     const int32_t *rowpos, int size, int64_t r0,
                                                                     int64_t r1, uint64_t *codes) {
  const int W = GD_PACK_WORDS(size);
  const __m256d c_maj = _mm256_set1_pd(3.0), c_mnr = _mm256_set1_pd(-3.0), c_mis = _mm256_set1_pd(-10000.0),
                c_het = _mm256_setzero_pd();
  unsigned bad = 0;
  for (int64_t r = r0; r < r1; ++r) {
    const double *v = vals + r * size;
    const int *ps = pos + r * size;
    const int32_t p0 = rowpos[r];
    const __m128i pp = _mm_set1_epi32(p0);
    uint64_t *out = codes + r * W;
    for (int w = 0; w < W; ++w) {
      const int k0 = 32 * w, k1 = std::min(size, k0 + 32);
      uint64_t word = 0;
      int k = k0;
      for (; k + 4 <= k1; k += 4) {
        const __m256d x = _mm256_loadu_pd(v + k);
        const unsigned maj = (unsigned)_mm256_movemask_pd(_mm256_cmp_pd(x, c_maj, _CMP_EQ_OQ));
        const unsigned mnr = (unsigned)_mm256_movemask_pd(_mm256_cmp_pd(x, c_mnr, _CMP_EQ_OQ));
        const unsigned mis = (unsigned)_mm256_movemask_pd(_mm256_cmp_pd(x, c_mis, _CMP_EQ_OQ));
        const unsigned het = (unsigned)_mm256_movemask_pd(_mm256_cmp_pd(x, c_het, _CMP_EQ_OQ));
        const unsigned peq = (unsigned)_mm_movemask_ps(
            _mm_castsi128_ps(_mm_cmpeq_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i *>(ps + k)), pp)));
        bad |= ((maj | mnr | mis | het) & peq) ^ 0xFu;
        const uint64_t c8 = _pdep_u32(maj | mis, 0x55u) | _pdep_u32(mnr | mis, 0xAAu);
        word |= c8 << (2 * (k - k0));
      }
      for (; k < k1; ++k) {
        const double x = v[k];
        const unsigned maj = x == 3.0, mnr = x == -3.0, mis = x == -10000.0, het = x == 0.0;
        bad |= (maj | mnr | mis | het) ^ 1u;
        bad |= (unsigned)(ps[k] != p0);
        word |= (uint64_t)(maj * GD_CODE_MAJOR | mnr * GD_CODE_MINOR | mis * GD_CODE_MISSING) << (2 * (k - k0));
      }
      out[w] = word;
    }
  }
  return bad == 0;
}

static bool pack_rows(const double *vals, const int *pos, const int32_t *rowpos, int size, int64_t r0, int64_t r1,
                      uint64_t *codes) {
  static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi2");
  return avx2 ? pack_pop_rows_avx2(vals, pos, rowpos, size, r0, r1, codes)
              : pack_pop_rows(vals, pos, rowpos, size, r0, r1, codes);
}

/* Host threads for the packer: GD_HOST_THREADS, else the process's CPU affinity capped by
 * OMP_NUM_THREADS (the GPU box's CPU share) and by 16 */
static int pack_threads() {
  if (const char *e = getenv("GD_HOST_THREADS")) return std::max(1, atoi(e));
  int n = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
  if (n <= 0) n = (int)std::thread::hardware_concurrency();
  if (const char *e = getenv("OMP_NUM_THREADS"))
    if (atoi(e) > 0) n = std::min(n, atoi(e));
  return std::max(1, std::min(n, 16));
}

/* A persistent pool of host threads for the packer (created on first use, pack_threads()
 * strong with the caller): a job is a number of pieces handed out by a counter; the caller
 * works on pieces too and returns when every piece is done.  One job at a time, process-wide:
 * host calls on different contexts or devices from different threads pack one after the
 * other (their device work still overlaps); the host-path figures in DESIGN.md are single
 * caller numbers.  A forked child inherits none of the worker threads: the pthread_atfork
 * child handler leaks their handles (joining threads that do not exist in the child would
 * hang), re-creates the locks, and the child packs on its calling thread alone. */
namespace {
class PackPool {
 public:
  static PackPool &get() {
    static PackPool pool(pack_threads());
    return pool;
  }
  int size() const { return (int)workers_.size() + 1; }
  template <class F>
  void run(int64_t npiece, F &&f) {
    std::lock_guard<std::mutex> one(job_mu_);
    if (npiece <= 0) return;
    std::function<void(int64_t)> fn(std::forward<F>(f));
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      npiece_ = npiece;
      next_.store(0);
      done_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    const int64_t mine = work();
    std::unique_lock<std::mutex> g(mu_);
    done_ += mine;
    cv_done_.wait(g, [&] { return done_ == npiece_; });
    fn_ = nullptr;
  }

 private:
  explicit PackPool(int n) {
    for (int t = 1; t < n; ++t) workers_.emplace_back([this] { loop(); });
    self_ = this;
    pthread_atfork(nullptr, nullptr, &PackPool::after_fork_child);
  }
  static void after_fork_child() {
    PackPool *p = self_;
    if (!p) return;
    (void)new std::vector<std::thread>(std::move(p->workers_)); /* never joined or destroyed */
    p->workers_.clear();
    new (&p->mu_) std::mutex();
    new (&p->job_mu_) std::mutex();
    new (&p->cv_) std::condition_variable();
    new (&p->cv_done_) std::condition_variable();
  }
  static inline PackPool *self_ = nullptr;
  ~PackPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  int64_t work() {
    int64_t n = 0;
    for (int64_t k; (k = next_.fetch_add(1)) < npiece_;) {
      (*fn_)(k);
      ++n;
    }
    return n;
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      const int64_t mine = work();
      std::lock_guard<std::mutex> g(mu_);
      done_ += mine;
      if (done_ == npiece_) cv_done_.notify_all();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_, job_mu_;
  std::condition_variable cv_, cv_done_;
  std::function<void(int64_t)> *fn_ = nullptr;
  int64_t npiece_ = 0, done_ = 0;
  std::atomic<int64_t> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};
}  // namespace

/* rows [r0, r1) of a chromosome on the pool: pieces of ~64k genotypes, each packed A then
 * B after its row positions (rowpos[r] = apos[r * asize]; B is compared with A's) */
extern "C" int gd_pack_rows_mt(const double *avals, const double *bvals, const int *apos, const int *bpos, int asize,
                               int bsize, int64_t r0, int64_t r1, uint64_t *acodes, uint64_t *bcodes,
                               int32_t *rowpos) {
  if (r1 <= r0) return GD_OK;
  const int64_t piece = std::max<int64_t>(1, (int64_t)(1 << 16) / (asize + bsize));
  const int64_t npiece = (r1 - r0 + piece - 1) / piece;
  std::atomic<bool> ok{true};
  PackPool::get().run(npiece, [&](int64_t k) {
    if (!ok.load(std::memory_order_relaxed)) return;
    const int64_t a = r0 + k * piece, b = std::min<int64_t>(r1, a + piece);
    for (int64_t r = a; r < b; ++r) rowpos[r] = apos[r * asize];
    if (!pack_rows(avals, apos, rowpos, asize, a, b, acodes) || !pack_rows(bvals, bpos, rowpos, bsize, a, b, bcodes))
      ok.store(false);
  });
  if (!ok.load())
    return pk_fail(GD_ERR_ARG, "a value is not one of the genotype codes 3, 0, -3, -10000, or a row's individuals "
                               "do not share one position (A and B)");
  return GD_OK;
}

/* gd_pack_chrom on the host thread pool (include/gdscan.h) */
extern "C" int gd_pack_chrom_mt(const double *avals, const double *bvals, const int *apos, const int *bpos, int asize,
                                int bsize, int nrows, uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos) {
  if (asize <= 0 || bsize <= 0 || nrows < 0) return pk_fail(GD_ERR_ARG, "population sizes must be positive");
  if (nrows == 0) return GD_OK;
  if (!avals || !bvals || !apos || !bpos || !acodes || !bcodes || !rowpos) return pk_fail(GD_ERR_ARG, "null buffer");
  return gd_pack_rows_mt(avals, bvals, apos, bpos, asize, bsize, 0, nrows, acodes, bcodes, rowpos);
}

extern "C" int gd_pack_chrom(const double *avals, const double *bvals, const int *apos, const int *bpos, int asize,
                             int bsize, int nrows, uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos) {
  if (asize <= 0 || bsize <= 0 || nrows < 0) return pk_fail(GD_ERR_ARG, "population sizes must be positive");
  if (nrows == 0) return GD_OK;
  if (!avals || !bvals || !apos || !bpos || !acodes || !bcodes || !rowpos)
    return pk_fail(GD_ERR_ARG, "null buffer");
  const int wa = GD_PACK_WORDS(asize), wb = GD_PACK_WORDS(bsize);
  for (int64_t r = 0; r < nrows; ++r) {
    const int32_t p0 = apos[r * asize];
    rowpos[r] = p0;
    for (int pop = 0; pop < 2; ++pop) {
      const int size = pop ? bsize : asize, W = pop ? wb : wa;
      const double *v = (pop ? bvals : avals) + r * size;
      const int *ps = (pop ? bpos : apos) + r * size;
      uint64_t *out = (pop ? bcodes : acodes) + r * W;
      std::memset(out, 0, sizeof(uint64_t) * W);
      for (int k = 0; k < size; ++k) {
        uint64_t c;
        if (!code_of(v[k], &c))
          return pk_fail(GD_ERR_ARG, "a value is not one of the genotype codes 3, 0, -3, -10000");
        if (ps[k] != p0)
          return pk_fail(GD_ERR_ARG, "a row's individuals do not share one position (A and B)");
        out[k >> 5] |= c << (2 * (k & 31));
      }
    }
  }
  return GD_OK;
}
