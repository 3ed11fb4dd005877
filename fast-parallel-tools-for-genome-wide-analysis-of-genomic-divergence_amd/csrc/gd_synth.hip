/*
 * gd_synth.hip -- device generator of the seeded synthetic SNP tracks; produces
 * exactly the arrays of gdscan/synth.py (SURVEY.md 8(d) workload, bench inputs).
 */
#include <hip/hip_runtime.h>
#include "gd_common.h"
#include "../../include/gdscan.h"

#define TAG_GAP 0x11ULL
#define TAG_FREQ 0x22ULL
#define TAG_NOISE 0x100ULL
#define TAG_ISLAND 0x33ULL
#define TAG_GENO 0x1000000ULL
#define TAG_MISS 0x2000000ULL
#define N_ISLANDS 5
#define ISLAND_SNPS 200
#define SYN_BLOCK 1024

__device__ __forceinline__ uint64_t h3(uint64_t seed, uint64_t c, uint64_t s, uint64_t tag) {
  return gd_mix64(gd_mix64(gd_mix64(seed ^ c) ^ s) ^ tag);
}
__device__ __forceinline__ double unit53(uint64_t h) { return (double)(h >> 11) * 0x1p-53; }

/* pass 1: per-block sums of the gaps */
__global__ void __launch_bounds__(256) k_syn_gapsum(int c, int nsnp, uint64_t seed, int64_t *bsum) {
  __shared__ int64_t sh[256];
  const int base = blockIdx.x * SYN_BLOCK;
  int64_t acc = 0;
  for (int i = threadIdx.x; i < SYN_BLOCK; i += 256) {
    const int s = base + i;
    if (s < nsnp) acc += 1 + (int64_t)(h3(seed, c, s, TAG_GAP) % 99ULL);
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = sh[0];
}

/* pass 2: exclusive scan of the block sums (one block, sequential over chunks) */
__global__ void k_syn_scan(int nblk, int64_t *bsum) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int64_t run = 0;
    for (int b = 0; b < nblk; ++b) {
      const int64_t v = bsum[b];
      bsum[b] = run;
      run += v;
    }
  }
}

/* pass 3: positions + genotypes, one block per SYN_BLOCK SNPs */
__global__ void __launch_bounds__(256) k_syn_fill(int c, int nsnp, int asize, int bsize, uint64_t seed,
                                                  const double *qtab, const int64_t *bsum, double *avals,
                                                  double *bvals, int32_t *apos, int32_t *bpos) {
  __shared__ int32_t sh_pos[SYN_BLOCK];
  __shared__ double sh_qa[SYN_BLOCK], sh_qb[SYN_BLOCK];
  const int base = blockIdx.x * SYN_BLOCK;
  const int cnt = min(SYN_BLOCK, nsnp - base);
  if (threadIdx.x == 0) {
    int64_t run = bsum[blockIdx.x];
    for (int i = 0; i < cnt; ++i) {
      run += 1 + (int64_t)(h3(seed, c, base + i, TAG_GAP) % 99ULL);
      sh_pos[i] = (int32_t)run;
    }
  }
  const int span = max(1, nsnp - ISLAND_SNPS);
  for (int i = threadIdx.x; i < cnt; i += 256) {
    const uint64_t s = (uint64_t)(base + i);
    const double qa = qtab[h3(seed, c, s, TAG_FREQ) >> 52];
    double acc = 0.0;
    for (int t = 0; t < 12; ++t) acc = acc + unit53(h3(seed, c, s, TAG_NOISE + t));
    double qb = qa + 0.2 * (acc - 6.0);
    qb = fmin(fmax(qb, 0.0), 1.0);
    for (int k = 0; k < N_ISLANDS; ++k) {
      const uint64_t st = h3(seed, c, (uint64_t)k, TAG_ISLAND) % (uint64_t)span;
      if (s >= st && s < st + ISLAND_SNPS) qb = 1.0 - qa;
    }
    sh_qa[i] = qa;
    sh_qb[i] = qb;
  }
  __syncthreads();
  for (int pop = 0; pop < 2; ++pop) {
    const int size = pop ? bsize : asize;
    double *vals = pop ? bvals : avals;
    int32_t *pos = pop ? bpos : apos;
    const int64_t e0 = (int64_t)base * size;
    const int ne = cnt * size;
    for (int e = threadIdx.x; e < ne; e += 256) {
      const int i = e / size, j = e - i * size;
      const uint64_t s = (uint64_t)(base + i);
      const double q = pop ? sh_qb[i] : sh_qa[i];
      const uint64_t tg = TAG_GENO + ((uint64_t)pop << 20) + (uint64_t)j;
      const uint64_t tm = TAG_MISS + ((uint64_t)pop << 20) + (uint64_t)j;
      const double u = unit53(h3(seed, c, s, tg));
      const double t1 = q * q;
      const double t2 = t1 + (2.0 * q) * (1.0 - q);
      double v = (u < t1) ? -3.0 : ((u < t2) ? 0.0 : 3.0);
      if (h3(seed, c, s, tm) % 50ULL == 0) v = -10000.0;
      vals[e0 + e] = v;
      pos[e0 + e] = sh_pos[i];
    }
  }
}

int gd_synth_launch(int chrom, int nsnp, int asize, int bsize, uint64_t seed, const double *qtab, double *avals,
                    double *bvals, int32_t *apos, int32_t *bpos, hipStream_t s) {
  const int nblk = (nsnp + SYN_BLOCK - 1) / SYN_BLOCK;
  int64_t *bsum = nullptr;
  if (hipMallocAsync((void **)&bsum, sizeof(int64_t) * nblk, s) != hipSuccess) return GD_ERR_HIP;
  hipLaunchKernelGGL(k_syn_gapsum, dim3(nblk), dim3(256), 0, s, chrom, nsnp, seed, bsum);
  hipLaunchKernelGGL(k_syn_scan, dim3(1), dim3(64), 0, s, nblk, bsum);
  hipLaunchKernelGGL(k_syn_fill, dim3(nblk), dim3(256), 0, s, chrom, nsnp, asize, bsize, seed, qtab, bsum, avals,
                     bvals, apos, bpos);
  const hipError_t e = hipGetLastError();
  (void)hipFreeAsync(bsum, s);
  return e == hipSuccess ? GD_OK : GD_ERR_HIP;
}
