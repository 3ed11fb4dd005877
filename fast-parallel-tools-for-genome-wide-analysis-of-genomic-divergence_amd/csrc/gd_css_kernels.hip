/* gd_css_kernels.hip -- CSS pipeline (pending) */
#include <hip/hip_runtime.h>
#include <vector>
#include "gd_internal.h"
#include "../../include/gdscan.h"
struct gd_ctx;
int gd_css_pipeline(gd_ctx *ctx, const gd_chrom_dev *d_ch, const std::vector<gd_chrom_dev> &h_ch, int64_t wtotal,
                    const double *avals, const double *bvals, int wsize, int wstep, int treshold, int runs,
                    double *scores, double *p, hipStream_t s) {
  return GD_ERR_ARG;
}
