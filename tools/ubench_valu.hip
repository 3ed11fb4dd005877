// Microbenchmark: VALU throughput of the ops an nrand48 bootstrap loop can use
// (gfx950).  Exact instructions via inline asm, 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N_IT 2048
#define CH 8
template <int OP>
__global__ void k(unsigned *out, unsigned seed) {
  unsigned a[CH];
  double d[CH];
  unsigned long long u[CH];
  const unsigned c = seed * 0x9E3779B9u | 1u;
  const double cd = 1.0000001;
  const unsigned c2 = c ^ 0x5A5A5A5Au;
  const unsigned long long sm = 0x5555555555555555ull ^ seed;
  for (int i = 0; i < CH; ++i) { a[i] = seed + threadIdx.x * 7 + i; d[i] = a[i]; u[i] = a[i]; }
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 4) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(cd));
      if (OP == 5) asm volatile("v_med3_i32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 6) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(cd));
      if (OP == 7) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 8) asm volatile("v_alignbit_b32 %0, %0, %1, 17" : "+v"(a[i]) : "v"(c));
      if (OP == 9) asm volatile("v_floor_f64 %0, %0" : "+v"(d[i]));
      if (OP == 10) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[i]) : "v"(a[i]));
      if (OP == 11) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(a[i]));
      if (OP == 12) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 13) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 14) asm volatile("v_max3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 15) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 16) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 17) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(u[i]) : "v"(a[i]), "v"(c) : "vcc");
      if (OP == 18) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(c));
      if (OP == 19) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 20) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 21) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 22) asm volatile("v_fract_f64 %0, %0" : "+v"(d[i]));
      if (OP == 23) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(u[i]));
      if (OP == 24) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(u[i]) : "v"(a[i]), "v"(c) : "vcc");
      if (OP == 25) asm volatile("v_bfe_u32 %0, %0, 3, 17" : "+v"(a[i]));
      if (OP == 26) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[i]));
      if (OP == 27) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 28) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(u[i]) : "v"(u[0]));
      if (OP == 29) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(c));
      if (OP == 30) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(c2));
      if (OP == 31) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 32) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 33) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(c2));
      if (OP == 34) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 35) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(c2));
      if (OP == 36) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a[i]));
      if (OP == 37) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 38) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 39) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(c), "v"(c2));
      if (OP == 40) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "s"(sm));
      if (OP == 41) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 42) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 43) asm volatile("v_max_f64 %0, %0, %1" : "+v"(d[i]) : "v"(cd));
      if (OP == 44) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(cd));
      if (OP == 45) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(a[i]) : "v"(a[(i + 1) % CH]));
      if (OP == 46) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(c2));
      if (OP == 47) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(c) : "vcc");
      if (OP == 48) asm volatile("v_mad_u32_u16 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(c2));
      if (OP == 49) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 50) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 51) asm volatile("v_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 52) asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a[i]), "v"(c) : "vcc");
      if (OP == 53) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 54) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c2));
      if (OP == 55) asm volatile("v_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 56) asm volatile("v_med3_u16 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(c2));
      if (OP == 57) asm volatile("v_med3_i16 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(c2));
      if (OP == 58) asm volatile("v_max_u16 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 59) asm volatile("v_min_u16 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 60) asm volatile("v_max_u16_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1" : "+v"(a[i]) : "v"(c));
      if (OP == 61) asm volatile("v_max_u32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if (OP == 62) asm volatile("v_min_i16 %0, %0, %1" : "+v"(a[i]) : "v"(c));
    }
  }
  unsigned s = 0;
  for (int i = 0; i < CH; ++i) s += a[i] + (unsigned)d[i] + (unsigned)u[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int OP>
float run(unsigned *o) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(256 * 8), dim3(256), 0, 0, o, 1u);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(256 * 8), dim3(256), 0, 0, o, 1u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  double ops = 5.0 * 256 * 8 * 256 * (double)N_IT * CH;
  return (float)(ops / (ms * 1e-3) / 1e12);
}
int main() {
  unsigned *o;
  (void)hipMalloc(&o, 256 * 8 * 256 * 4);
  printf("v_add_u32        %.1f Tlane-op/s\n", run<0>(o));
  printf("v_mul_lo_u32     %.1f\n", run<1>(o));
  printf("v_mul_hi_u32     %.1f\n", run<2>(o));
  printf("v_mul_u32_u24    %.1f\n", run<3>(o));
  printf("v_fma_f64        %.1f\n", run<4>(o));
  printf("v_med3_i32       %.1f\n", run<5>(o));
  printf("v_mul_f64        %.1f\n", run<6>(o));
  printf("v_mul_hi_u32_u24 %.1f\n", run<7>(o));
  printf("v_alignbit_b32   %.1f\n", run<8>(o));
  printf("v_floor_f64      %.1f\n", run<9>(o));
  printf("v_cvt_f64_u32    %.1f\n", run<10>(o));
  printf("v_lshrrev_b32    %.1f\n", run<11>(o));
  printf("v_sub_u32        %.1f\n", run<12>(o));
  printf("v_max_i32        %.1f\n", run<13>(o));
  printf("v_max3_u32       %.1f\n", run<14>(o));
  printf("v_add3_u32       %.1f\n", run<15>(o));
  printf("v_lshl_add_u32   %.1f\n", run<16>(o));
  printf("v_mad_u64_u32    %.1f\n", run<17>(o));
  printf("v_cndmask_b32    %.1f\n", run<18>(o));
  printf("v_and_b32        %.1f\n", run<19>(o));
  printf("v_mad_u32_u24    %.1f\n", run<20>(o));
  printf("v_pk_min_u16     %.1f\n", run<21>(o));
  printf("v_fract_f64      %.1f\n", run<22>(o));
  printf("v_lshlrev_b64    %.1f\n", run<23>(o));
  printf("v_mad_u64_u32 0  %.1f\n", run<24>(o));
  printf("v_bfe_u32        %.1f\n", run<25>(o));
  printf("v_cvt_f32_u32    %.1f\n", run<26>(o));
  printf("v_mul_f32        %.1f\n", run<27>(o));
  printf("v_pk_mul_f32     %.1f\n", run<28>(o));
  printf("v_mul_lo_u32 s   %.1f\n", run<29>(o));
  printf("v_med3_f32       %.1f\n", run<30>(o));
  printf("v_max_f32        %.1f\n", run<31>(o));
  printf("v_min_f32        %.1f\n", run<32>(o));
  printf("v_max3_f32       %.1f\n", run<33>(o));
  printf("v_add_f32        %.1f\n", run<34>(o));
  printf("v_fma_f32        %.1f\n", run<35>(o));
  printf("v_lshlrev_b32    %.1f\n", run<36>(o));
  printf("v_or_b32         %.1f\n", run<37>(o));
  printf("v_xor_b32        %.1f\n", run<38>(o));
  printf("v_bfi_b32        %.1f\n", run<39>(o));
  printf("v_cndmask_b32 sgpr%.1f\n", run<40>(o));
  printf("v_max_u32        %.1f\n", run<41>(o));
  printf("v_min_u32        %.1f\n", run<42>(o));
  printf("v_max_f64        %.1f\n", run<43>(o));
  printf("v_add_f64        %.1f\n", run<44>(o));
  printf("v_mov_b32_dpp    %.1f\n", run<45>(o));
  printf("v_perm_b32       %.1f\n", run<46>(o));
  printf("v_add_co_u32     %.1f\n", run<47>(o));
  printf("v_mad_u32_u16    %.1f\n", run<48>(o));
  printf("v_pk_max_u16     %.1f\n", run<49>(o));
  printf("v_pk_add_u16     %.1f\n", run<50>(o));
  printf("v_add_u16        %.1f\n", run<51>(o));
  printf("v_cmp_gt_u32     %.1f\n", run<52>(o));
  printf("v_mul_u32_u24 e32%.1f\n", run<53>(o));
  printf("v_mul_hi_u32 x2  %.1f\n", run<54>(o));
  printf("v_max_i16        %.1f\n", run<55>(o));
  printf("v_med3_u16       %.1f\n", run<56>(o));
  printf("v_med3_i16       %.1f\n", run<57>(o));
  printf("v_max_u16        %.1f\n", run<58>(o));
  printf("v_min_u16        %.1f\n", run<59>(o));
  printf("v_max_u16 sdwa   %.1f\n", run<60>(o));
  printf("v_max_u32 e32 rep%.1f\n", run<61>(o));
  printf("v_min_i16        %.1f\n", run<62>(o));
  return 0;
}
