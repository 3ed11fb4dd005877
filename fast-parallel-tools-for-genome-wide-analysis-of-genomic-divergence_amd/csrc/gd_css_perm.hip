/*
 * gd_css_perm.hip -- the CSS permutation test (significance_treshold, css.c:675-752)
 * on the MDS coordinates the score kernels leave in xbuf.
 *
 * One workgroup of NWV waves per window (windows pulled from a work counter: the
 * early exit makes their cost uneven), 64 * NWV permutations per pass, one per lane:
 *  1. draws: lane t of wave v (permutation q = 64 v + t of the pass) starts at draw
 *     q (m - 1) of the pass via an affine LCG jump and applies its Fisher-Yates swaps
 *     to an identity column sigma_q of its wave's LDS byte matrix (a rejected draw,
 *     probability ~m/2^31, sends the pass through the serial generator, which records
 *     each permutation's start state).
 *  2. tracks: F_q = F_{q-1} o sigma_q, 64 steps per wave, the waves in turn (the
 *     carry F between them in LDS); F is held one element per lane and gathered with
 *     ds_bpermute; F_q overwrites the dead column sigma_q.
 *  3. score of every lane's F_q: the between-group sum over the smaller group G as
 *     sum_{x in G} R_x - 2 sum_{x<y in G} S_xy (R = row sums of S), read from the
 *     packed lower triangle of S in LDS, plus the consecutive within-group pairs
 *     (Q8).  The observed score is the same function of the identity tracks, so
 *     ties are decided identically for observed and permuted scores.
 *  4. hits are counted in permutation order (one ballot per wave), so the early exit
 *     stops exactly where the serial loop would.
 * The tracks are reset to the identity per window and every window draws from its
 * own nrand48 stream (deviation 1).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/gdscan.h"
#include "gd_common.h"
#include "gd_internal.h"

/* A copy of the lane id the compiler cannot see through: lane-derived addresses are
 * rebuilt inside each phase instead of being hoisted out of the window and pass
 * loops as ~100 live VGPRs. */
#define PERM_OPAQUE(x) asm volatile("" : "+v"(x))

#ifdef GD_PERM_PROFILE
/* diagnostics build only: shader-clock cycles per phase summed over workgroups (thread 0) */
#include <cstdio>
__device__ unsigned long long g_perm_prof[8];
#define PERM_PROF_INIT uint64_t prof_t = __builtin_readcyclecounter()
#define PERM_PROF(ph)                                                  \
  do {                                                                 \
    if (threadIdx.x == 0) {                                            \
      const uint64_t t_ = __builtin_readcyclecounter();               \
      atomicAdd(&g_perm_prof[ph], (unsigned long long)(t_ - prof_t)); \
      prof_t = t_;                                                     \
    }                                                                  \
  } while (0)
#else
#define PERM_PROF_INIT
#define PERM_PROF(ph)
#endif

namespace {

__device__ __forceinline__ int perm_chrom_of(const gd_chrom_dev *ch, int nchrom, int64_t w) {
  int lo = 0, hi = nchrom - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ch[mid].w_base <= w)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

/* calc_dist (css.c:573-587) of points i, j of X (m x 2, row-major) */
__device__ __forceinline__ double perm_xdist(const double *X, int i, int j) {
  const double dx = X[2 * i] - X[2 * j], dy = X[2 * i + 1] - X[2 * j + 1];
  return sqrt(dx * dx + dy * dy);
}

/* waves per workgroup: the LDS (S triangle + per-wave byte matrices) sets it */
template <int MP>
struct PermShape {
  static constexpr int TRI = MP * (MP + 1) / 2 + 1; /* packed triangle + padding row + zero */
  static constexpr int HALF = MP / 2;               /* largest smaller-group size */
#ifndef PERM_NWV_LARGE
#define PERM_NWV_LARGE 2 /* waves per workgroup above 64 individuals */
#endif
  static constexpr int NWV = MP <= 64 ? 4 : PERM_NWV_LARGE;
  static constexpr int NT = 64 * NWV;
};

/* packed lower triangle with one zero row appended: pair (x, y), x != y, at
 * T(max) + min, T(h) = h(h-1)/2; index MP is a padding individual with S = 0, and
 * the pair (MP, MP) lands on the extra zero entry at the end */
__device__ __forceinline__ uint32_t tri8(uint32_t x) { return (x * (x - 1u) >> 1) << 3; }

/* S(x, y) for two individuals given their tri8 forms */
__device__ __forceinline__ double s_pair(const double *S, uint32_t x, uint32_t tx, uint32_t y, uint32_t ty) {
  const uint32_t off = x > y ? tx + (y << 3) : ty + (x << 3);
  return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(S) + off);
}

/* css() of the track array in column `lane` of sig (byte k at sig[k*64 + lane]).
 * The consecutive within-group pairs (css.c:627-642) are summed first, in track
 * order; the smaller group G is collected as a bit set on the way and then written
 * back over the head of the column in ascending order (the column is dead after
 * the score).  With the members ascending, pair (u < v) sits at T(x_v) + x_u with no
 * compare, and the between-group term becomes a function of the SET G alone, so
 * every permutation that keeps the groups' sets gets the observed value bit for bit.
 * Pairs are visited in 8x8 blocks of members (runtime block loops, unrolled blocks),
 * which bounds both the code and the loads in flight. */
template <int MP>
__device__ __forceinline__ double perm_score(const double *S, const double *R, uint8_t *sig, int lane, int a, int b,
                                             double inva, double invb) {
  constexpr int NB = (PermShape<MP>::HALF + 7) / 8;
  const int m = a + b;
  const int g = a <= b ? a : b, off = a <= b ? 0 : a;
  PERM_OPAQUE(lane);
  uint8_t *col = sig + lane;
  const char *Sb = reinterpret_cast<const char *>(S);
  /* consecutive pairs inside each group, and G as a bit set */
  double wa = 0.0, wb = 0.0;
  uint64_t lo = 0, hi = 0;
  auto add_member = [&](uint32_t x) {
    lo |= x < 64 ? 1ull << (x & 63u) : 0ull;
    if constexpr (MP > 64) hi |= x >= 64 ? 1ull << (x & 63u) : 0ull;
  };
  uint32_t prev = col[0], tprev = tri8(prev);
  if (off == 0 && g > 0) add_member(prev);
#pragma unroll 4
  for (int k = 1; k < m; ++k) {
    const uint32_t cur = col[k * 64], tcur = tri8(cur);
    const double e = s_pair(S, prev, tprev, cur, tcur);
    if (k < a) wa += e;
    if (k > a) wb += e;
    if (k >= off && k < off + g) add_member(cur);
    prev = cur;
    tprev = tcur;
  }
  /* the members, ascending, over bytes 0 .. g-1 of the column */
#pragma unroll 4
  for (int k = 0; k < g; ++k) {
    uint32_t x;
    if (MP <= 64 || lo != 0) {
      x = (uint32_t)__builtin_ctzll(lo);
      lo &= lo - 1;
    } else {
      x = 64u + (uint32_t)__builtin_ctzll(hi);
      hi &= hi - 1;
    }
    col[k * 64] = (uint8_t)x;
  }
  /* member k of G, padded with the zero individual MP (the largest index) */
  auto member = [&](int k) -> uint32_t { return k < g ? (uint32_t)col[k * 64] : (uint32_t)MP; };
  auto s_at = [&](uint32_t off8) { return *reinterpret_cast<const double *>(Sb + off8); };
  double sr = 0.0, q0 = 0.0, q1 = 0.0, q2 = 0.0, q3 = 0.0;
#pragma unroll 1
  for (int K = 0; K < NB; ++K) {
    uint32_t xk8[8], tk[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t x = member(8 * K + u);
      sr += R[x];
      xk8[u] = x << 3;
      tk[u] = tri8(x);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int v = u + 1; v < 8; ++v) {
        const double e = s_at(tk[v] + xk8[u]); /* x_u < x_v */
        if ((u + v) & 1)
          q0 += e;
        else
          q1 += e;
      }
      asm volatile("" ::: "memory"); /* a bounded number of gathers in flight */
    }
#pragma unroll 1
    for (int L = K + 1; L < NB; ++L) {
      uint32_t tl[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) tl[v] = tri8(member(8 * L + v));
#pragma unroll
      for (int u = 0; u < 8; ++u) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          const double e = s_at(tl[v] + xk8[u]); /* every member of block K < every member of block L */
          if (v & 1)
            q3 += e;
          else
            q2 += e;
        }
        asm volatile("" ::: "memory");
      }
    }
  }
  const double bet = sr - 2.0 * ((q0 + q1) + (q2 + q3));
  return bet / (double)(a * b) - (double)(a + b) * (wa * inva + wb * invb);
}

/* every lane's column of one wave's byte matrix := identity (rows k < m; row k is
 * 64 bytes of k) */
__device__ __forceinline__ void sig_identity(uint8_t *sig, int m, int lane) {
  PERM_OPAQUE(lane);
  for (int q = lane; q < m * 16; q += 64)
    *reinterpret_cast<uint32_t *>(sig + (q >> 4) * 64 + (q & 15) * 4) = (uint32_t)(q >> 4) * 0x01010101u;
}

/* Fisher-Yates swaps of random_shuffle (css.c:700-706) on the lane's column, draws
 * from state x (no rejection: the caller checks); returns true if a draw would have
 * been rejected */
__device__ __forceinline__ bool fy_fast(uint8_t *col, uint64_t x, int m, const gd_randint *rdt) {
  bool rej = false;
  for (int s = 0; s < m - 1; ++s) {
    const int n = m - s;
    x = gd_lcg_next(x);
    const uint32_t r = gd_lcg_value(x);
    const gd_randint rd = rdt[n];
    rej |= r > rd.limit;
    const int j = (int)gd_randint_mod(&rd, r);
    const uint8_t u = col[(n - 1) * 64], v = col[j * 64];
    col[(n - 1) * 64] = v;
    col[j * 64] = u;
  }
  return rej;
}

/* the same with random_int_nrand48's redraw loop (css.c:675-690) */
__device__ __forceinline__ void fy_exact(uint8_t *col, uint64_t x, int m, const gd_randint *rdt) {
  for (int s = 0; s < m - 1; ++s) {
    const int n = m - s;
    const gd_randint rd = rdt[n];
    uint32_t r;
    do {
      x = gd_lcg_next(x);
      r = gd_lcg_value(x);
    } while (r > rd.limit);
    const int j = (int)gd_randint_mod(&rd, r);
    const uint8_t u = col[(n - 1) * 64], v = col[j * 64];
    col[(n - 1) * 64] = v;
    col[j * 64] = u;
  }
}

}  // namespace

#ifdef PERM_WAVES_PER_SIMD /* diagnostic: register-allocation target */
#define PERM_WPE __attribute__((amdgpu_waves_per_eu(PERM_WAVES_PER_SIMD, PERM_WAVES_PER_SIMD)))
#else
#define PERM_WPE
#endif
template <int MP>
__global__ void __launch_bounds__(PermShape<MP>::NT) PERM_WPE
    k_css_perm(const gd_chrom_dev *ch, int nchrom, const double *xbuf, const uint8_t *status, int64_t wtotal,
               int treshold, int runs, double *pvals, unsigned *wq) {
  constexpr int TRI = PermShape<MP>::TRI, NWV = PermShape<MP>::NWV, NT = PermShape<MP>::NT, P = 64 * NWV;
  constexpr int SIG = MP * 64; /* one wave's byte matrix */
  __shared__ double s_S[TRI];
  __shared__ double s_R[MP + 1];
  __shared__ __attribute__((aligned(16))) uint8_t s_sig[NWV * SIG > 16 * MP ? NWV * SIG : 16 * MP];
  __shared__ gd_randint s_rd[MP + 1];
  __shared__ uint64_t s_st[P + 1];
  __shared__ uint64_t s_hit[NWV];
  __shared__ uint8_t s_car[MP > 64 ? 128 : 64];
  __shared__ int64_t s_w;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int n = tid; n <= MP; n += NT) s_rd[n] = gd_randint_make(n < 1 ? 1u : (uint32_t)n);
  double *s_x = reinterpret_cast<double *>(s_sig); /* X staging, dead before the draws */
  uint8_t *my_sig = s_sig + wave * SIG;

  PERM_PROF_INIT;
  for (;;) {
    __syncthreads();
    if (tid == 0) s_w = (int64_t)atomicAdd(wq, 1u);
    __syncthreads();
    const int64_t w = s_w;
    if (w >= wtotal) break;
    if (!status[w]) continue;
    const int c = perm_chrom_of(ch, nchrom, w);
    const gd_chrom_dev &d = ch[c];
    const int a = d.asize, b = d.bsize, m = a + b, m1 = m - 1;
    const int64_t wl = w - d.w_base;

    /* S (packed triangle, zero rows for individuals >= m) and its row sums */
    int ln = tid;
    PERM_OPAQUE(ln);
    for (int e = ln; e < 2 * m; e += NT) s_x[e] = xbuf[w * 2 * MP + e];
    __syncthreads();
#pragma unroll 1
    for (int h = 1; h <= MP; ++h) {
      for (int l = ln; l < h; l += NT)
        s_S[h * (h - 1) / 2 + l] = (h < m && l < m) ? perm_xdist(s_x, h, l) : 0.0;
    }
    if (tid == 0) s_S[TRI - 1] = 0.0;
    __syncthreads();
    for (int r = ln; r <= MP; r += NT) {
      double acc = 0.0;
      if (r < m) {
        const uint32_t tr = tri8((uint32_t)r);
        for (int j = 0; j < m; ++j)
          if (j != r) acc += s_pair(s_S, (uint32_t)r, tr, (uint32_t)j, tri8((uint32_t)j));
      }
      s_R[r] = acc;
    }
    if (tid < m) s_car[tid] = (uint8_t)tid; /* tracks := identity */
    __syncthreads();

    const double inva = a > 1 ? 1.0 / (double)(a * a * (a - 1)) : 0.0;
    const double invb = b > 1 ? 1.0 / (double)(b * b * (b - 1)) : 0.0;
    sig_identity(my_sig, m, lane);
    __syncthreads();
    const double obs = perm_score<MP>(s_S, s_R, my_sig, lane, a, b, inva, invb);
    PERM_PROF(0);

    uint64_t base = gd_window_state(d.seed, GD_STREAM_CSS, wl);
    const gd_affine Jq = gd_lcg_jump((uint64_t)tid * (uint64_t)m1), JP = gd_lcg_jump((uint64_t)P * (uint64_t)m1);
    int hits = 0, nsc = 0;
    bool done = !(treshold > 0 && runs > 0);
    while (!done) {
      /* 1. draws and Fisher-Yates swaps on sigma_q, q = tid */
      __syncthreads();
      sig_identity(my_sig, m, lane);
      __syncthreads();
      int lq = lane;
      PERM_OPAQUE(lq);
      uint8_t *col = my_sig + lq;
      const bool rej = fy_fast(col, gd_affine_apply(Jq, base), m, s_rd);
      if (__syncthreads_or(rej)) {
        /* exact serial stream: the start state of every permutation of the pass */
        if (tid == 0) {
          uint64_t y = base;
          for (int q = 0; q < P; ++q) {
            s_st[q] = y;
            for (int s = 0; s < m1; ++s) {
              const gd_randint rd = s_rd[m - s];
              do y = gd_lcg_next(y);
              while (gd_lcg_value(y) > rd.limit);
            }
          }
          s_st[P] = y;
        }
        __syncthreads();
        sig_identity(my_sig, m, lane);
        __syncthreads();
        fy_exact(col, s_st[tid], m, s_rd);
        base = s_st[P];
      } else {
        base = gd_affine_apply(JP, base);
      }
      __syncthreads();
      PERM_PROF(1);

      /* 2. F_q = F_{q-1} o sigma_q, one wave after the other; lane i owns rows i and i + 64 */
      for (int v = 0; v < NWV; ++v) {
        if (wave == v) {
          uint32_t pf0[16], pf1[16];
          int li = lane;
          PERM_OPAQUE(li);
          const bool r0 = li < m, r1 = MP > 64 && li + 64 < m;
          /* above 64 individuals lane i carries F(i) and F(i + 64) as the low two bytes of
           * one word, so one ds_bpermute per row fetches whichever of the two is wanted */
          uint32_t car = (uint32_t)s_car[li] | (MP > 64 ? (uint32_t)s_car[li + 64] << 8 : 0u);
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            pf0[q] = r0 ? *reinterpret_cast<const uint32_t *>(my_sig + li * 64 + 4 * q) : 0u;
            pf1[q] = r1 ? *reinterpret_cast<const uint32_t *>(my_sig + (li + 64) * 64 + 4 * q) : 0u;
          }
#pragma unroll
          for (int t = 0; t < 64; ++t) {
            const uint32_t s0 = (pf0[t >> 2] >> (8 * (t & 3))) & 0xFFu;
            uint32_t n0, n1 = 0;
            if constexpr (MP > 64) {
              const uint32_t s1 = (pf1[t >> 2] >> (8 * (t & 3))) & 0xFFu;
              const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((s0 & 63u) << 2), (int)car);
              const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((s1 & 63u) << 2), (int)car);
              n0 = (s0 < 64 ? a0 : a0 >> 8) & 0xFFu;
              n1 = (s1 < 64 ? a1 : a1 >> 8) & 0xFFu;
              if (r1) my_sig[(li + 64) * 64 + t] = (uint8_t)n1;
            } else {
              n0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(s0 << 2), (int)car);
            }
            if (r0) my_sig[li * 64 + t] = (uint8_t)n0;
            car = n0 | (n1 << 8);
          }
          if (r0) s_car[li] = (uint8_t)car;
          if (r1) s_car[li + 64] = (uint8_t)(car >> 8);
        }
        __syncthreads();
      }

      PERM_PROF(2);
      /* 3. scores of the P permuted track arrays, 4. in-order hit count */
      const double sc = perm_score<MP>(s_S, s_R, my_sig, lane, a, b, inva, invb);
#ifdef GD_PERM_PROFILE
      __syncthreads();
      PERM_PROF(3);
#endif
      const int valid = min(P, runs - nsc);
      const uint64_t H = __ballot(tid < valid && sc >= obs);
      if (lane == 0) s_hit[wave] = H;
      __syncthreads();
      for (int v = 0; v < NWV && !done; ++v) {
        const uint64_t Hv = s_hit[v];
        const int vv = min(64, max(0, valid - 64 * v)); /* valid permutations of wave v */
        const int need = treshold - hits;
        if (__popcll(Hv) >= need) {
          uint64_t h = Hv;
          for (int k = 1; k < need; ++k) h &= h - 1;
          nsc += __ffsll((unsigned long long)h); /* position of the need-th hit, + 1 */
          hits = treshold;
          done = true;
        } else {
          hits += __popcll(Hv);
          nsc += vv;
          done = nsc >= runs;
        }
      }
    }
    PERM_PROF(4);
    if (tid == 0) pvals[d.w_out + wl] = (hits + 1) * 1.0 / (nsc + 1);
  }
}

template <int MP>
static int launch_perm(const gd_chrom_dev *d_ch, int nchrom, const double *xbuf, const uint8_t *status, int64_t wtotal,
                       int treshold, int runs, double *p, unsigned *wq, hipStream_t s) {
  const unsigned grid = (unsigned)std::min<int64_t>(wtotal, 256 * 16);
  hipLaunchKernelGGL(k_css_perm<MP>, dim3(grid), dim3(PermShape<MP>::NT), 0, s, d_ch, nchrom, xbuf, status, wtotal,
                     treshold, runs, p, wq);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}

int gd_css_perm_launch(int mp, const gd_chrom_dev *d_ch, int nchrom, const double *xbuf, const uint8_t *status,
                       int64_t wtotal, int treshold, int runs, double *p, unsigned *wq, hipStream_t s) {
#ifdef GD_PERM_PROFILE
  {
    static const unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_perm_prof), z, sizeof z, 0, hipMemcpyHostToDevice, s);
  }
  struct Dump {
    hipStream_t s;
    ~Dump() {
      unsigned long long h[8];
      (void)hipStreamSynchronize(s);
      (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_perm_prof), sizeof h);
      fprintf(stderr, "perm-prof cycles: setup %llu draws %llu compose %llu score %llu hits %llu\n", h[0], h[1], h[2],
              h[3], h[4]);
    }
  } dump{s};
#endif
  switch (mp) {
    case 24: return launch_perm<24>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 40: return launch_perm<40>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 64: return launch_perm<64>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 80: return launch_perm<80>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 96: return launch_perm<96>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
    case 128: return launch_perm<128>(d_ch, nchrom, xbuf, status, wtotal, treshold, runs, p, wq, s);
  }
  return GD_ERR_SIZE;
}
