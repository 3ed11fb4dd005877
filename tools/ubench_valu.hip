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
  return 0;
}
