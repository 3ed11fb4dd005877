/* gd_fet_fast.hip -- placeholder: route every window to the general path */
#include <hip/hip_runtime.h>
#include "gd_internal.h"
#include "../../include/gdscan.h"

__global__ void k_all_windows(int32_t *list, unsigned *count, int64_t wtotal) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < wtotal) list[i] = (int32_t)i;
  if (i == 0) *count = (unsigned)wtotal;
}

int gd_fet_window_fast_launch(const gd_chrom_dev *ch, int nchrom, int64_t wtotal, const int32_t *lo_a,
                              const int32_t *hi_a, const int32_t *lo_b, const double *snp_score, double perc,
                              double *scores, double *stddev, unsigned *flags, int32_t *slow_list,
                              unsigned *slow_count, hipStream_t s) {
  hipLaunchKernelGGL(k_all_windows, dim3((wtotal + 255) / 256), dim3(256), 0, s, slow_list, slow_count, wtotal);
  return hipGetLastError() == hipSuccess ? GD_OK : GD_ERR_HIP;
}
