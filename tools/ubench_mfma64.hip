// Microbenchmark: FP64 MFMA (v_mfma_f64_16x16x4_f64) issue rate on gfx950 vs FP64 VALU FMA,
// 4 independent accumulators per wave, one or more waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
#define N_IT 4096
__global__ void k_mfma(double *out, double a0) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = a0 + threadIdx.x, b = a0 * 0.5;
  for (int it = 0; it < N_IT; ++it) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + s.z + s.w;
}
__global__ void k_valu(double *out, double a0) {
  double c[8];
  for (int i = 0; i < 8; ++i) c[i] = a0 + i + threadIdx.x;
  const double m = 1.0000001, k = 1e-9;
  for (int it = 0; it < N_IT; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c[i]) : "v"(m), "v"(k));
  double s = 0;
  for (int i = 0; i < 8; ++i) s += c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <class K>
void run(const char *name, K kern, int waves_per_simd, double flop_per_wave_it) {
  double *o;
  (void)hipMalloc(&o, 1 << 26);
  const int blocks = 256 * 4 * waves_per_simd;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, o, 1.0);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, o, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 3.0 * blocks * (double)N_IT * flop_per_wave_it;
  printf("%-28s waves/SIMD %d: %.1f TFLOP/s\n", name, waves_per_simd, flops / (ms * 1e-3) / 1e12);
  (void)hipFree(o);
}
int main() {
  for (int w : {1, 2, 4}) run("mfma_f64_16x16x4 (4 acc)", k_mfma, w, 4 * 16 * 16 * 4 * 2.0);
  for (int w : {1, 2, 4}) run("v_fma_f64 (8 chains)", k_valu, w, 8 * 64 * 2.0);
  return 0;
}
