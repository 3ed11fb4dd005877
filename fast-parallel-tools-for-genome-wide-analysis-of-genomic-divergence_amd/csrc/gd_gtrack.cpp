/*
 * gd_gtrack.cpp -- HyperBrowser track I/O around the scan.
 *
 * Reader: GTrack "valued points" files as written by the reference's converter
 * (tools/VCFConvert.py:44-86: header lines starting with '#', a "###" line naming the
 * columns -- seqid, start, value, genomeid -- then one line per (SNP, individual) in
 * population-list order).  Per seqid, in file order, it yields exactly the arrays
 * HyperBrowser hands the statistics (startsAsNumpyArray -> int32, valsAsNumpyArray ->
 * float64; FisherExactScoreStat.py:36-40).  The file is memory-mapped and parsed in one
 * pass per chunk, chunks split at line boundaries and parsed on up to 16 threads;
 * integer-valued tokens (all genotype codes) take a fast path, anything else goes
 * through strtod.
 *
 * Writer: the tools' tabular result lines (FisherExactTestSNPTool.py:162-189,
 * ClusterSeparationScore.py:180-205): "seqid\tstart\tscore\tstddev|p" for every window
 * with score != 0, start = i * wStep, floats printed like Python 2's str(float)
 * ('%.12g', plus ".0" when the text would read as an integer; quirk Q11).
 */
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/gdscan.h"

void gd_set_error(const char *msg); /* gd_api.hip */
void gd_set_status_error(int code, const char *msg);

struct gd_gtrack {
  std::vector<std::string> seqid;
  std::vector<std::vector<int32_t>> starts;
  std::vector<std::vector<double>> vals;
};

namespace {

struct Columns {
  int seqid = 0, start = 1, value = 2, ncol = 4;
};

/* split [p, e) on tabs into at most `max` fields */
int split_tabs(const char *p, const char *e, const char **fb, const char **fe, int max) {
  int n = 0;
  const char *s = p;
  for (const char *q = p;; ++q) {
    if (q == e || *q == '\t') {
      if (n < max) {
        fb[n] = s;
        fe[n] = q;
      }
      ++n;
      if (q == e) break;
      s = q + 1;
    }
  }
  return n;
}

bool parse_int(const char *b, const char *e, int64_t *out) {
  if (b == e) return false;
  bool neg = false;
  if (*b == '-' || *b == '+') {
    neg = *b == '-';
    ++b;
  }
  if (b == e) return false;
  int64_t v = 0;
  for (; b < e; ++b) {
    if (*b < '0' || *b > '9') return false;
    v = v * 10 + (*b - '0');
    if (v > (int64_t)1 << 53) return false;
  }
  *out = neg ? -v : v;
  return true;
}

bool parse_value(const char *b, const char *e, double *out) {
  int64_t iv;
  if (parse_int(b, e, &iv)) {
    *out = (double)iv;
    return true;
  }
  std::string s(b, e);
  char *end = nullptr;
  errno = 0;
  const double v = strtod(s.c_str(), &end);
  if (end == s.c_str() || *end != '\0') return false;
  *out = v;
  return true;
}

/* Python 2 str(float): '%.12g', plus ".0" when the text has no '.', exponent or letter */
int py2_float(char *buf, size_t cap, double x) {
  if (std::isnan(x)) return snprintf(buf, cap, "nan");
  if (std::isinf(x)) return snprintf(buf, cap, x > 0 ? "inf" : "-inf");
  int n = snprintf(buf, cap, "%.12g", x);
  if (!strpbrk(buf, ".e")) n += snprintf(buf + n, cap - n, ".0");
  return n;
}

}  // namespace

namespace {

/* runs of consecutive lines with the same seqid, parsed from one chunk of the file */
struct Run {
  std::string seqid;
  std::vector<int32_t> starts;
  std::vector<double> vals;
};

struct Chunk {
  std::vector<Run> runs;
  bool ok = true;
  std::string err;
};

/* parse the data lines of [p, end): '#' lines are comments (column headers are read
 * up front, before the data) */
void parse_chunk(const char *p, const char *end, const Columns &col, Chunk *out) {
  Run *cur = nullptr;
  while (p < end) {
    const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
    const char *le = nl ? nl : end;
    const char *line_end = (le > p && le[-1] == '\r') ? le - 1 : le;
    if (line_end > p && p[0] != '#') {
      const char *fb[32], *fe[32];
      const int n = split_tabs(p, line_end, fb, fe, 32);
      int64_t pos;
      double val;
      if (n <= col.seqid || n <= col.start || n <= col.value || !parse_int(fb[col.start], fe[col.start], &pos) ||
          pos < INT32_MIN || pos > INT32_MAX || !parse_value(fb[col.value], fe[col.value], &val)) {
        out->ok = false;
        out->err = "malformed data line: " + std::string(p, (size_t)std::min<ptrdiff_t>(line_end - p, 80));
        return;
      }
      const size_t nlen = (size_t)(fe[col.seqid] - fb[col.seqid]);
      if (!cur || nlen != cur->seqid.size() || memcmp(fb[col.seqid], cur->seqid.data(), nlen) != 0) {
        out->runs.emplace_back();
        cur = &out->runs.back();
        cur->seqid.assign(fb[col.seqid], nlen);
      }
      cur->starts.push_back((int32_t)pos);
      cur->vals.push_back(val);
    }
    p = nl ? nl + 1 : end;
  }
}

}  // namespace

namespace {

/* a GTrack file mapped read-only, its column header read (leading '#' lines: the "###"
 * line names the columns) and its data split into up to 16 chunks at line boundaries */
struct MappedTrack {
  const char *data = nullptr;
  size_t size = 0;
  Columns col;
  std::vector<const char *> cut; /* chunk k is [cut[k], cut[k + 1]) */
  std::string err;

  ~MappedTrack() {
    if (data) munmap((void *)data, size);
  }

  bool open_file(const char *path) {
    if (!path) {
      err = "null path";
      return false;
    }
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
      err = std::string("cannot open ") + path + ": " + strerror(errno);
      return false;
    }
    struct stat st;
    if (fstat(fd, &st) != 0) {
      close(fd);
      err = "fstat failed";
      return false;
    }
    size = (size_t)st.st_size;
    if (size > 0) {
      void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m == MAP_FAILED) {
        close(fd);
        size = 0;
        err = "mmap failed";
        return false;
      }
      madvise(m, size, MADV_SEQUENTIAL);
      data = (const char *)m;
    }
    close(fd);
    const char *p = data, *end = data + size;
    while (p < end && *p == '#') {
      const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
      const char *le = nl ? nl : end;
      const char *line_end = (le > p && le[-1] == '\r') ? le - 1 : le;
      if (line_end - p > 3 && p[1] == '#' && p[2] == '#' && p[3] != '#') {
        const char *fb[32], *fe[32];
        const int n = split_tabs(p + 3, line_end, fb, fe, 32);
        Columns c;
        c.seqid = c.start = c.value = -1;
        c.ncol = n;
        for (int k = 0; k < n && k < 32; ++k) {
          const std::string name(fb[k], fe[k]);
          if (name == "seqid") c.seqid = k;
          if (name == "start") c.start = k;
          if (name == "value") c.value = k;
        }
        if (c.seqid < 0 || c.start < 0 || c.value < 0) err = std::string(path) + ": column header lacks seqid/start/value";
        col = c;
      }
      p = nl ? nl + 1 : end;
    }
    if (!err.empty()) return false;
    if (p < end) {
      const size_t bytes = (size_t)(end - p);
      /* one thread per 16 MiB, at most 16 (GD_GTRACK_CHUNK: bytes per thread, for tests) */
      size_t per = (size_t)1 << 24;
      if (const char *e = getenv("GD_GTRACK_CHUNK")) per = std::max<size_t>(1, strtoull(e, nullptr, 10));
      const unsigned hw = std::thread::hardware_concurrency();
      const int T = (int)std::min<size_t>(std::max(1u, std::min(hw, 16u)), std::max<size_t>(1, bytes / per));
      cut.assign(T + 1, p);
      cut[T] = end;
      for (int k = 1; k < T; ++k) {
        const char *q = p + bytes * k / T;
        if (q < cut[k - 1]) q = cut[k - 1];
        const char *nl = (const char *)memchr(q, '\n', (size_t)(end - q));
        cut[k] = nl ? nl + 1 : end;
      }
    }
    return true;
  }

  int chunks() const { return cut.empty() ? 0 : (int)cut.size() - 1; }

  /* fn(k) on chunk k, chunks 1.. on their own threads */
  template <class F>
  void parallel(F fn) const {
    std::vector<std::thread> th;
    for (int k = 1; k < chunks(); ++k) th.emplace_back(fn, k);
    if (chunks() > 0) fn(0);
    for (auto &x : th) x.join();
  }
};

}  // namespace

extern "C" gd_gtrack *gd_gtrack_read(const char *path) {
  MappedTrack mt;
  if (!mt.open_file(path)) {
    gd_set_error(mt.err.c_str());
    return nullptr;
  }
  /* data: chunks parsed in parallel, runs merged in order */
  std::vector<Chunk> chunks(mt.chunks());
  mt.parallel([&](int k) { parse_chunk(mt.cut[k], mt.cut[k + 1], mt.col, &chunks[k]); });
  for (auto &c : chunks)
    if (!c.ok) {
      gd_set_error((std::string(path) + ": " + c.err).c_str());
      return nullptr;
    }
  gd_gtrack *t = new gd_gtrack();
  std::unordered_map<std::string, int> index;
  for (auto &c : chunks)
    for (auto &r : c.runs) {
      auto it = index.find(r.seqid);
      int s;
      if (it == index.end()) {
        s = (int)t->seqid.size();
        index.emplace(r.seqid, s);
        t->seqid.push_back(r.seqid);
        t->starts.emplace_back(std::move(r.starts));
        t->vals.emplace_back(std::move(r.vals));
        continue;
      }
      s = it->second;
      t->starts[s].insert(t->starts[s].end(), r.starts.begin(), r.starts.end());
      t->vals[s].insert(t->vals[s].end(), r.vals.begin(), r.vals.end());
    }
  return t;
}

extern "C" void gd_gtrack_free(gd_gtrack *t) { delete t; }

extern "C" int gd_gtrack_nseq(const gd_gtrack *t) { return t ? (int)t->seqid.size() : 0; }

extern "C" const char *gd_gtrack_seqid(const gd_gtrack *t, int s) {
  return (t && s >= 0 && s < (int)t->seqid.size()) ? t->seqid[s].c_str() : nullptr;
}

extern "C" int64_t gd_gtrack_len(const gd_gtrack *t, int s) {
  return (t && s >= 0 && s < (int)t->seqid.size()) ? (int64_t)t->starts[s].size() : -1;
}

extern "C" int gd_gtrack_copy(const gd_gtrack *t, int s, int32_t *starts, double *vals) {
  if (!t || s < 0 || s >= (int)t->seqid.size()) {
    gd_set_error("bad sequence index");
    return GD_ERR_ARG;
  }
  const size_t n = t->starts[s].size();
  if (starts && n) memcpy(starts, t->starts[s].data(), n * sizeof(int32_t));
  if (vals && n) memcpy(vals, t->vals[s].data(), n * sizeof(double));
  return GD_OK;
}

/* ------------------------------------------------------------------------------------
 * Packing reader: the same files parsed straight into packed genotype tracks (2-bit
 * codes, one position per row; include/gdscan.h "packed genotype tracks"), with no f64
 * value or per-element position ever materialised.  The chunk parsers keep one byte per
 * genotype and the positions run-length encoded (a row is a run of `size` equal
 * positions); the merge joins the runs of each sequence in file order, takes the
 * population size from the leading run (get_population_size, comparative.c:25-34) and
 * checks every run holds whole rows; then each chunk packs its own bytes into the final
 * words (words shared by two chunks are or-ed atomically).
 */
struct gd_ptrack {
  std::vector<std::string> seqid;
  std::vector<int32_t> size;
  std::vector<std::vector<uint64_t>> codes; /* nrows * GD_PACK_WORDS(size) words */
  std::vector<std::vector<int32_t>> rowpos; /* nrows */
};

namespace {

struct PRun {
  std::string seqid;
  std::vector<uint8_t> codes; /* one per line */
  std::vector<int32_t> rpos;  /* positions, run-length encoded */
  std::vector<int64_t> rlen;
  int seq = -1;
  int64_t first = 0; /* index of codes[0] among its sequence's elements */
};

struct PChunk {
  std::vector<PRun> runs;
  bool ok = true;
  bool nopack = false; /* a readable track with no packed form (GD_ERR_NOPACK) */
  std::string err;
};

/* VCFConvert.py:9-18 values -> GD_CODE_* */
bool genotype_code(double x, uint8_t *c) {
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

void parse_packed_chunk(const char *p, const char *end, const Columns &col, PChunk *out) {
  PRun *cur = nullptr;
  while (p < end) {
    const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
    const char *le = nl ? nl : end;
    const char *line_end = (le > p && le[-1] == '\r') ? le - 1 : le;
    if (line_end > p && p[0] != '#') {
      const char *fb[32], *fe[32];
      const int n = split_tabs(p, line_end, fb, fe, 32);
      int64_t pos;
      double val;
      uint8_t code;
      if (n <= col.seqid || n <= col.start || n <= col.value || !parse_int(fb[col.start], fe[col.start], &pos) ||
          pos < INT32_MIN || pos > INT32_MAX || !parse_value(fb[col.value], fe[col.value], &val)) {
        out->ok = false;
        out->err = "malformed data line: " + std::string(p, (size_t)std::min<ptrdiff_t>(line_end - p, 80));
        return;
      }
      if (!genotype_code(val, &code)) {
        out->ok = false;
        out->nopack = true;
        out->err = "a value is not one of the genotype codes 3, 0, -3, -10000: " +
                   std::string(p, (size_t)std::min<ptrdiff_t>(line_end - p, 80));
        return;
      }
      const size_t nlen = (size_t)(fe[col.seqid] - fb[col.seqid]);
      if (!cur || nlen != cur->seqid.size() || memcmp(fb[col.seqid], cur->seqid.data(), nlen) != 0) {
        out->runs.emplace_back();
        cur = &out->runs.back();
        cur->seqid.assign(fb[col.seqid], nlen);
      }
      cur->codes.push_back(code);
      if (!cur->rpos.empty() && cur->rpos.back() == (int32_t)pos) {
        ++cur->rlen.back();
      } else {
        cur->rpos.push_back((int32_t)pos);
        cur->rlen.push_back(1);
      }
    }
    p = nl ? nl + 1 : end;
  }
}

/* or the run's codes into its sequence's words: element e of the sequence is individual
 * e mod size of row e / size */
void pack_run(const PRun &r, int64_t size, uint64_t *words) {
  const int64_t W = GD_PACK_WORDS(size);
  int64_t row = r.first / size, k = r.first % size;
  int64_t widx = row * W + (k >> 5);
  uint64_t acc = 0;
  for (uint8_t c : r.codes) {
    acc |= (uint64_t)c << (2 * (k & 31));
    if (++k == size) {
      __atomic_fetch_or(&words[widx], acc, __ATOMIC_RELAXED);
      acc = 0;
      k = 0;
      ++row;
      widx = row * W;
    } else if ((k & 31) == 0) {
      __atomic_fetch_or(&words[widx], acc, __ATOMIC_RELAXED);
      acc = 0;
      ++widx;
    }
  }
  if (acc) __atomic_fetch_or(&words[widx], acc, __ATOMIC_RELAXED);
}

}  // namespace

extern "C" gd_ptrack *gd_ptrack_read(const char *path) {
  MappedTrack mt;
  if (!mt.open_file(path)) {
    gd_set_error(mt.err.c_str());
    return nullptr;
  }
  std::vector<PChunk> chunks(mt.chunks());
  mt.parallel([&](int k) { parse_packed_chunk(mt.cut[k], mt.cut[k + 1], mt.col, &chunks[k]); });
  for (auto &c : chunks)
    if (!c.ok) {
      gd_set_status_error(c.nopack ? GD_ERR_NOPACK : GD_ERR_ARG, (std::string(path) + ": " + c.err).c_str());
      return nullptr;
    }
  /* merge: the runs of each sequence in file order, their position runs joined */
  std::unique_ptr<gd_ptrack> t(new gd_ptrack());
  std::unordered_map<std::string, int> index;
  std::vector<std::vector<int32_t>> rpos;
  std::vector<std::vector<int64_t>> rlen;
  std::vector<int64_t> nel;
  for (auto &c : chunks)
    for (auto &r : c.runs) {
      auto it = index.find(r.seqid);
      if (it == index.end()) {
        it = index.emplace(r.seqid, (int)t->seqid.size()).first;
        t->seqid.push_back(r.seqid);
        rpos.emplace_back();
        rlen.emplace_back();
        nel.push_back(0);
      }
      const int s = it->second;
      r.seq = s;
      r.first = nel[s];
      nel[s] += (int64_t)r.codes.size();
      for (size_t j = 0; j < r.rpos.size(); ++j) {
        if (!rpos[s].empty() && rpos[s].back() == r.rpos[j]) {
          rlen[s].back() += r.rlen[j];
        } else {
          rpos[s].push_back(r.rpos[j]);
          rlen[s].push_back(r.rlen[j]);
        }
      }
      std::vector<int32_t>().swap(r.rpos);
      std::vector<int64_t>().swap(r.rlen);
    }
  const int ns = (int)t->seqid.size();
  t->size.resize(ns);
  t->codes.resize(ns);
  t->rowpos.resize(ns);
  for (int s = 0; s < ns; ++s) {
    const int64_t size = rlen[s][0];
    if (size > INT32_MAX) {
      gd_set_status_error(GD_ERR_NOPACK,
                          (std::string(path) + ": population size above 2^31 in sequence " + t->seqid[s]).c_str());
      return nullptr;
    }
    std::vector<int32_t> &rp = t->rowpos[s];
    rp.reserve((size_t)(nel[s] / size));
    for (size_t j = 0; j < rpos[s].size(); ++j) {
      if (rlen[s][j] % size != 0) {
        gd_set_status_error(GD_ERR_NOPACK,
                            (std::string(path) + ": sequence " + t->seqid[s] + " does not consist of whole rows of " +
                      std::to_string(size) + " individuals at one position (position " +
                      std::to_string(rpos[s][j]) + " holds " + std::to_string(rlen[s][j]) +
                      " elements); such a track keeps the reference layout (gd_gtrack_read)")
                         .c_str());
        return nullptr;
      }
      rp.insert(rp.end(), (size_t)(rlen[s][j] / size), rpos[s][j]);
    }
    t->size[s] = (int32_t)size;
    t->codes[s].assign(rp.size() * (size_t)GD_PACK_WORDS(size), 0);
    std::vector<int32_t>().swap(rpos[s]);
    std::vector<int64_t>().swap(rlen[s]);
  }
  mt.parallel([&](int k) {
    for (const PRun &r : chunks[k].runs) pack_run(r, t->size[r.seq], t->codes[r.seq].data());
  });
  return t.release();
}

extern "C" void gd_ptrack_free(gd_ptrack *t) { delete t; }

extern "C" int gd_ptrack_nseq(const gd_ptrack *t) { return t ? (int)t->seqid.size() : 0; }

extern "C" const char *gd_ptrack_seqid(const gd_ptrack *t, int s) {
  return (t && s >= 0 && s < (int)t->seqid.size()) ? t->seqid[s].c_str() : nullptr;
}

extern "C" int gd_ptrack_shape(const gd_ptrack *t, int s, int32_t *size, int64_t *nrows) {
  if (!t || s < 0 || s >= (int)t->seqid.size() || !size || !nrows) {
    gd_set_error("bad sequence index");
    return GD_ERR_ARG;
  }
  *size = t->size[s];
  *nrows = (int64_t)t->rowpos[s].size();
  return GD_OK;
}

extern "C" int gd_ptrack_copy(const gd_ptrack *t, int s, uint64_t *codes, int32_t *rowpos) {
  if (!t || s < 0 || s >= (int)t->seqid.size()) {
    gd_set_error("bad sequence index");
    return GD_ERR_ARG;
  }
  if (codes && !t->codes[s].empty()) memcpy(codes, t->codes[s].data(), t->codes[s].size() * sizeof(uint64_t));
  if (rowpos && !t->rowpos[s].empty()) memcpy(rowpos, t->rowpos[s].data(), t->rowpos[s].size() * sizeof(int32_t));
  return GD_OK;
}

extern "C" int gd_write_tabular(const char *path, int append, const char *header, const char *seqid, int wstep,
                                int64_t n, const double *scores, const double *other) {
  if (!path || !seqid || wstep <= 0 || n < 0 || (n > 0 && (!scores || !other))) {
    gd_set_error("bad tabular-writer arguments");
    return GD_ERR_ARG;
  }
  FILE *f = fopen(path, append ? "ab" : "wb");
  if (!f) {
    gd_set_error((std::string("cannot open ") + path + ": " + strerror(errno)).c_str());
    return GD_ERR_ARG;
  }
  std::vector<char> buf(1 << 20);
  setvbuf(f, buf.data(), _IOFBF, buf.size());
  if (header) fprintf(f, "%s\n", header);
  char a[64], b[64];
  for (int64_t i = 0; i < n; ++i) {
    if (scores[i] == 0) continue; /* 0 and -0.0 mean "no window" (Q5) */
    py2_float(a, sizeof a, scores[i]);
    py2_float(b, sizeof b, other[i]);
    fprintf(f, "%s\t%lld\t%s\t%s\n", seqid, (long long)(i * (int64_t)wstep), a, b);
  }
  const int bad = ferror(f);
  if (fclose(f) != 0 || bad) {
    gd_set_error("write failed");
    return GD_ERR_ARG;
  }
  return GD_OK;
}

extern "C" int gd_format_py2_float(double x, char *buf, int cap) {
  if (!buf || cap <= 0) return GD_ERR_ARG;
  return py2_float(buf, (size_t)cap, x);
}

/* ------------------------------------------------------------------------------------
 * Tabular reader for the region filters: the tools' result files as
 * FilterFisherScores.preProcessPvalues / SignificantCSSRegions.preProcessPvalues read
 * them (FilterFisherScores.py:117-131, SignificantCSSRegions.py:157-173): every line
 * that is non-empty and does not start with '#' is "seqid \t start \t col2 \t col3 ...";
 * the address is (seqid, start), col2/col3 parse like Python float().  A line with
 * fewer than four fields is an error (the tools raise IndexError).  The start must be
 * an integer (the merge calls int() on it); it is kept as int64 and written back in
 * canonical decimal.
 */
struct gd_tabular {
  std::vector<std::string> seqid;
  std::vector<int32_t> seq;
  std::vector<int64_t> start;
  std::vector<double> c2, c3;
};

namespace {

struct TabChunk {
  std::vector<std::string> names; /* chunk-local first-seen order */
  std::vector<int32_t> seq;
  std::vector<int64_t> start;
  std::vector<double> c2, c3;
  bool ok = true;
  std::string err;
};

void parse_tab_chunk(const char *p, const char *end, TabChunk *out) {
  int cur = -1;
  std::unordered_map<std::string, int> local;
  while (p < end) {
    const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
    const char *le = nl ? nl : end;
    const char *line_end = (le > p && le[-1] == '\r') ? le - 1 : le;
    if (le > p && p[0] != '#') {
      const char *fb[4], *fe[4];
      const int n = split_tabs(p, line_end, fb, fe, 4);
      int64_t pos;
      double a, b;
      if (n < 4 || !parse_int(fb[1], fe[1], &pos) || !parse_value(fb[2], fe[2], &a) ||
          !parse_value(fb[3], fe[3], &b)) {
        out->ok = false;
        out->err = "malformed result line: " + std::string(p, (size_t)std::min<ptrdiff_t>(line_end - p, 80));
        return;
      }
      const size_t nlen = (size_t)(fe[0] - fb[0]);
      if (cur < 0 || nlen != out->names[cur].size() || memcmp(fb[0], out->names[cur].data(), nlen) != 0) {
        std::string name(fb[0], nlen);
        auto it = local.find(name);
        if (it == local.end()) {
          cur = (int)out->names.size();
          local.emplace(name, cur);
          out->names.push_back(std::move(name));
        } else {
          cur = it->second;
        }
      }
      out->seq.push_back(cur);
      out->start.push_back(pos);
      out->c2.push_back(a);
      out->c3.push_back(b);
    }
    p = nl ? nl + 1 : end;
  }
}

}  // namespace

extern "C" gd_tabular *gd_tabular_read(const char *path) {
  if (!path) {
    gd_set_error("null path");
    return nullptr;
  }
  const int fd = open(path, O_RDONLY);
  if (fd < 0) {
    gd_set_error((std::string("cannot open ") + path + ": " + strerror(errno)).c_str());
    return nullptr;
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    gd_set_error("fstat failed");
    return nullptr;
  }
  const size_t size = (size_t)st.st_size;
  const char *data = nullptr;
  if (size > 0) {
    void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      close(fd);
      gd_set_error("mmap failed");
      return nullptr;
    }
    madvise(m, size, MADV_SEQUENTIAL);
    data = (const char *)m;
  }
  close(fd);
  std::vector<TabChunk> chunks;
  std::string err;
  if (size > 0) {
    const char *p = data, *end = data + size;
    unsigned hw = std::thread::hardware_concurrency();
    int T = (int)std::min<size_t>(std::max(1u, std::min(hw, 16u)), std::max<size_t>(1, size >> 24));
    std::vector<const char *> cut(T + 1);
    cut[0] = p;
    cut[T] = end;
    for (int k = 1; k < T; ++k) {
      const char *q = p + size * k / T;
      if (q < cut[k - 1]) q = cut[k - 1];
      const char *nl = (const char *)memchr(q, '\n', (size_t)(end - q));
      cut[k] = nl ? nl + 1 : end;
    }
    chunks.resize(T);
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k) th.emplace_back(parse_tab_chunk, cut[k], cut[k + 1], &chunks[k]);
    parse_tab_chunk(cut[0], cut[1], &chunks[0]);
    for (auto &x : th) x.join();
    for (auto &c : chunks)
      if (!c.ok && err.empty()) err = c.err;
    munmap((void *)data, size);
  }
  if (!err.empty()) {
    gd_set_error((std::string(path) + ": " + err).c_str());
    return nullptr;
  }
  gd_tabular *t = new gd_tabular();
  std::unordered_map<std::string, int> index;
  size_t rows = 0;
  for (auto &c : chunks) rows += c.seq.size();
  t->seq.reserve(rows);
  t->start.reserve(rows);
  t->c2.reserve(rows);
  t->c3.reserve(rows);
  for (auto &c : chunks) {
    std::vector<int32_t> glob(c.names.size());
    for (size_t k = 0; k < c.names.size(); ++k) {
      auto it = index.find(c.names[k]);
      if (it == index.end()) {
        glob[k] = (int32_t)t->seqid.size();
        index.emplace(c.names[k], glob[k]);
        t->seqid.push_back(c.names[k]);
      } else {
        glob[k] = it->second;
      }
    }
    for (int32_t s : c.seq) t->seq.push_back(glob[s]);
    t->start.insert(t->start.end(), c.start.begin(), c.start.end());
    t->c2.insert(t->c2.end(), c.c2.begin(), c.c2.end());
    t->c3.insert(t->c3.end(), c.c3.begin(), c.c3.end());
  }
  return t;
}

extern "C" void gd_tabular_free(gd_tabular *t) { delete t; }

extern "C" int64_t gd_tabular_rows(const gd_tabular *t) { return t ? (int64_t)t->seq.size() : 0; }

extern "C" int gd_tabular_nseq(const gd_tabular *t) { return t ? (int)t->seqid.size() : 0; }

extern "C" const char *gd_tabular_seqid(const gd_tabular *t, int s) {
  return (t && s >= 0 && s < (int)t->seqid.size()) ? t->seqid[s].c_str() : nullptr;
}

extern "C" int gd_tabular_copy(const gd_tabular *t, int32_t *seq, int64_t *start, double *col2, double *col3) {
  if (!t) {
    gd_set_error("null table");
    return GD_ERR_ARG;
  }
  const size_t n = t->seq.size();
  if (!n) return GD_OK;
  if (seq) memcpy(seq, t->seq.data(), n * sizeof(int32_t));
  if (start) memcpy(start, t->start.data(), n * sizeof(int64_t));
  if (col2) memcpy(col2, t->c2.data(), n * sizeof(double));
  if (col3) memcpy(col3, t->c3.data(), n * sizeof(double));
  return GD_OK;
}
