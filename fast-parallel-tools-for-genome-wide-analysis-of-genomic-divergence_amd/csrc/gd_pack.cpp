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
#include <cstdint>
#include <cstring>

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
