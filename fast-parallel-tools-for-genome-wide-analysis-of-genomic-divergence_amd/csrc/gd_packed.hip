/*
 * gd_packed.hip -- scans over packed genotype tracks (second
 * half): the four genotype values VCFConvert.py:8-17 writes (3, 0, -3, -10000) as 2-bit
 * codes, one position per SNP row instead of one per (row, individual).
 *
 * Layout (include/gdscan.h): population P of a chromosome is nrows x W(P) uint64 words,
 * W = GD_PACK_WORDS(size); individual k of row r sits in bits 2(k mod 32) of word
 * r W + k / 32; codes 0 het (0), 1 hom-major (3), 2 hom-minor (-3), 3 missing (-10000);
 * padding codes are 0.  Both populations share the rows' positions.  12 B per genotype
 * (f64 value + i32 position) become 2 bits + 4 B per row.
 *
 * The windows of a packed chromosome are the reference's windows over its expanded
 * form (every individual of row r at element r * size), so the scans reuse the window
 * kernels unchanged:
 *   k_bounds_rows      slide_right() (comparative.c:49-71) on row positions: element
 *                      bounds lo_a = r asize, hi_a, lo_b = r bsize of every window
 *   k_snp_fet_packed   fetcount (cFisher.c:208-238) from the codes (popcounts of the
 *                      code planes) + the score table -> per-SNP -log10 p
 *   k_css_pack_codes   the CSS bit planes ("== 3", "== -3") of every individual
 *   k_pack_device      device packer for reference-layout tracks already in HBM
 */
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_fet_rows.h"
#include "gd_internal.h"

namespace {

/* floor(a / b), b > 0 */
__device__ __forceinline__ int64_t pk_fdiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

constexpr uint64_t PK_LO = 0x5555555555555555ull;

}  // namespace

/* slide_right() on the rows: row r (0 <= r <= nrows; r == nrows is the +inf sentinel)
 * owns the windows whose start lies in (pos[r-1], pos[r]] (lo) and whose inclusive stop
 * lies in [pos[r-1], pos[r]) (hi), exactly as element r * size of the expanded track in
 * k_bounds; rows inside a run of equal positions own nothing.  Grid (x, chrom). */
__global__ void __launch_bounds__(256) k_bounds_rows(const gd_chrom_dev *ch, const int64_t *row_off,
                                                     const int32_t *rowpos, int wsize, int wstep, int32_t *lo_a,
                                                     int32_t *hi_a, int32_t *lo_b, unsigned *flags) {
  const gd_chrom_dev &d = ch[blockIdx.y];
  const int64_t wend = d.wend, nrows = d.nrows;
  if (wend <= 0) return;
  const int32_t *pos = rowpos + row_off[blockIdx.y];
  int32_t *lo = lo_a + d.w_base, *hi = hi_a + d.w_base, *lb = lo_b + d.w_base;
  bool unsorted = false;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const bool first = r == 0, last = r == nrows;
    const int64_t p = last ? 0 : pos[r], pp = first ? 0 : pos[r - 1];
    if (!first && !last) unsorted |= p < pp;
    if (!first && !last && p == pp) continue;
    int64_t f = first ? 0 : pk_fdiv(pp, wstep) + 1 - d.w_first;
    int64_t l = last ? wend - 1 : pk_fdiv(p, wstep) - d.w_first;
    f = f < 0 ? 0 : f;
    l = l > wend - 1 ? wend - 1 : l;
    for (int64_t w = f; w <= l; ++w) {
      lo[w] = (int32_t)(r * d.asize);
      lb[w] = (int32_t)(r * d.bsize);
    }
    f = first ? 0 : -pk_fdiv(wsize - pp, wstep) - d.w_first;
    l = last ? wend - 1 : -pk_fdiv(wsize - p, wstep) - 1 - d.w_first;
    f = f < 0 ? 0 : f;
    l = l > wend - 1 ? wend - 1 : l;
    for (int64_t w = f; w <= l; ++w) hi[w] = (int32_t)(r * d.asize);
  }
  if (unsorted) atomicOr(flags, GD_FLAG_UNSORTED_A);
}

/* per-SNP -log10 p from the codes: a row's four counts are popcounts of its words' low
 * code bits without the high bits (code 1, value 3) and high without low (code 2, -3).
 * Written at snp_score[d.a_off + r] (a_off holds the chromosome's first row here). */
__global__ void __launch_bounds__(256) k_snp_fet_packed(const gd_chrom_dev *ch, const int64_t *word_off,
                                                        const uint64_t *acodes, const uint64_t *bcodes,
                                                        const uint64_t *binom, const int *lut_hdr, const double *lut,
                                                        double *snp_score) {
  const gd_chrom_dev &d = ch[blockIdx.y];
  if (d.wend <= 0) return;
  const int asize = d.asize, bsize = d.bsize, wa = GD_PACK_WORDS(asize), wb = GD_PACK_WORDS(bsize);
  const uint64_t *ca = acodes + word_off[2 * blockIdx.y], *cb = bcodes + word_off[2 * blockIdx.y + 1];
  const bool use_lut = gd_lut_holds(lut_hdr, asize, bsize, binom);
  const int lut_nb = (bsize + 1) * (bsize + 2) / 2;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < d.nrows; r += (int64_t)gridDim.x * blockDim.x) {
    int f[4] = {0, 0, 0, 0};
    for (int k = 0; k < wa; ++k) {
      const uint64_t w = ca[r * wa + k], lo = w & PK_LO, hi = (w >> 1) & PK_LO;
      f[0] += __popcll(lo & ~hi);
      f[1] += __popcll(hi & ~lo);
    }
    for (int k = 0; k < wb; ++k) {
      const uint64_t w = cb[r * wb + k], lo = w & PK_LO, hi = (w >> 1) & PK_LO;
      f[2] += __popcll(lo & ~hi);
      f[3] += __popcll(hi & ~lo);
    }
    snp_score[d.a_off + r] =
        use_lut ? lut[(int64_t)gd_pair_index(f[0], f[1], asize) * lut_nb + gd_pair_index(f[2], f[3], bsize)]
                : gd_fet_score_from_p(fet_p_two_tailed(f[0], f[1], f[2], f[3], binom));
  }
}

/* CSS bit planes from the codes (k_css_pack's layout: individual i's "== 3" plane at
 * pa + 2i wa, "== -3" at pa + (2i+1) wa; packed codes are never irregular, so the
 * irregular-value plane stays zero) */
__global__ void __launch_bounds__(256) k_css_pack_codes(const gd_chrom_dev *ch, const gd_css_planes *pl,
                                                        const int64_t *word_off, const uint64_t *acodes,
                                                        const uint64_t *bcodes, uint32_t *planes) {
  const gd_chrom_dev &d = ch[blockIdx.y];
  const int pop = blockIdx.z;
  if (d.wend <= 0) return;
  const int s = pop ? d.bsize : d.asize;
  if (s <= 0) return;
  const int W = GD_PACK_WORDS(s);
  const int64_t rows = d.nrows;
  const uint64_t *codes = (pop ? bcodes : acodes) + word_off[2 * blockIdx.y + pop];
  const gd_css_planes p = pl[blockIdx.y];
  const int64_t nw = pop ? p.wb : p.wa;
  uint32_t *base = planes + (pop ? p.pb : p.pa);
  const int64_t items = ((rows + 31) >> 5) * s;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < items; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = t / s;
    const int i = (int)(t - w * s);
    const int64_t r0 = w * 32;
    const int nb = (int)min<int64_t>(32, rows - r0);
    const uint64_t *src = codes + r0 * W + (i >> 5);
    const int sh = 2 * (i & 31);
    uint32_t P = 0, N = 0;
    for (int k = 0; k < nb; ++k) {
      const uint32_t c = (uint32_t)(src[(int64_t)k * W] >> sh) & 3u;
      P |= (uint32_t)(c == GD_CODE_MAJOR) << k;
      N |= (uint32_t)(c == GD_CODE_MINOR) << k;
    }
    base[(int64_t)(2 * i) * nw + w] = P;
    base[(int64_t)(2 * i + 1) * nw + w] = N;
  }
}

/* the packer on the device (gd_pack_chrom's rules): one thread per (row, population,
 * word); a value outside the four codes, or an individual whose position differs from
 * the row's (pos[r * asize] of A), raises *bad */
__global__ void __launch_bounds__(256) k_pack_device(const double *avals, const double *bvals, const int32_t *apos,
                                                     const int32_t *bpos, int asize, int bsize, int nrows,
                                                     uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos,
                                                     unsigned *bad) {
  const int wa = GD_PACK_WORDS(asize), wb = GD_PACK_WORDS(bsize), per = wa + wb;
  bool err = false;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < (int64_t)nrows * per;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / per;
    const int k = (int)(t - r * per);
    const bool pb = k >= wa;
    const int kk = pb ? k - wa : k, size = pb ? bsize : asize;
    const double *v = (pb ? bvals : avals) + r * size;
    const int32_t *ps = (pb ? bpos : apos) + r * size;
    const int32_t p0 = apos[r * asize];
    if (k == 0) rowpos[r] = p0;
    uint64_t word = 0;
    const int i1 = min(size, 32 * kk + 32);
    for (int i = 32 * kk; i < i1; ++i) {
      const double x = v[i];
      const uint64_t c = x == 3.0 ? GD_CODE_MAJOR : x == -3.0 ? GD_CODE_MINOR : x == 0.0 ? GD_CODE_HET : GD_CODE_MISSING;
      err |= !(x == 3.0 || x == -3.0 || x == 0.0 || x == -10000.0) || ps[i] != p0;
      word |= c << (2 * (i & 31));
    }
    (pb ? bcodes + r * wb : acodes + r * wa)[kk] = word;
  }
  if (err) atomicOr(bad, 1u);
}

int gd_packed_bounds_launch(const gd_chrom_dev *d_ch, int nchrom, const int64_t *row_off, const int32_t *rowpos,
                            int64_t max_rows, int wsize, int wstep, int32_t *lo_a, int32_t *hi_a, int32_t *lo_b,
                            unsigned *flags, hipStream_t s) {
  const unsigned gx = (unsigned)std::min<int64_t>((max_rows + 256) / 256, std::max(1, 16384 / std::max(nchrom, 1)));
  hipLaunchKernelGGL(k_bounds_rows, dim3(std::max(1u, gx), nchrom), dim3(256), 0, s, d_ch, row_off, rowpos, wsize,
                     wstep, lo_a, hi_a, lo_b, flags);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

int gd_packed_snp_fet_launch(const gd_chrom_dev *d_ch, int nchrom, const int64_t *word_off, const uint64_t *acodes,
                             const uint64_t *bcodes, int64_t max_rows, const uint64_t *binom, const int *lut_hdr,
                             const double *lut, double *snp, hipStream_t s) {
  const unsigned gx = (unsigned)std::min<int64_t>((max_rows + 255) / 256, std::max(1, 16384 / std::max(nchrom, 1)));
  hipLaunchKernelGGL(k_snp_fet_packed, dim3(std::max(1u, gx), nchrom), dim3(256), 0, s, d_ch, word_off, acodes,
                     bcodes, binom, lut_hdr, lut, snp);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

int gd_packed_css_planes_launch(const gd_chrom_dev *d_ch, int nchrom, const gd_css_planes *d_pl,
                                const int64_t *word_off, const uint64_t *acodes, const uint64_t *bcodes,
                                int64_t max_rows_words, uint32_t *planes, hipStream_t s) {
  const unsigned gx = (unsigned)std::min<int64_t>((max_rows_words * 8 + 255) / 256, std::max(1, 16384 / nchrom));
  hipLaunchKernelGGL(k_css_pack_codes, dim3(std::max(1u, gx), nchrom, 2), dim3(256), 0, s, d_ch, d_pl, word_off,
                     acodes, bcodes, planes);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

int gd_pack_device_launch(const double *avals, const double *bvals, const int32_t *apos, const int32_t *bpos,
                          int asize, int bsize, int nrows, uint64_t *acodes, uint64_t *bcodes, int32_t *rowpos,
                          unsigned *bad, hipStream_t s) {
  const int64_t items = (int64_t)nrows * (GD_PACK_WORDS(asize) + GD_PACK_WORDS(bsize));
  const unsigned gx = (unsigned)std::min<int64_t>((items + 255) / 256, 16384);
  hipLaunchKernelGGL(k_pack_device, dim3(std::max(1u, gx)), dim3(256), 0, s, avals, bvals, apos, bpos, asize, bsize,
                     nrows, acodes, bcodes, rowpos, bad);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}
