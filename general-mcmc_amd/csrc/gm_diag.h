// gm_diag.h — device split-R-hat / ESS stages (diag_kernels.hip).
#pragma once
#include "gm_internal.h"

namespace gm {
struct DiagScratch {
  void* part = nullptr;
  size_t part_bytes = 0;
  DiagScratch() = default;
  DiagScratch(const DiagScratch&) = delete;
  DiagScratch& operator=(const DiagScratch&) = delete;
  ~DiagScratch() {
    if (part) (void)hipFree(part);
  }
};
// Per-split-chain means / within variances ([P][2C] each, f64) and the
// autocovariance summed over this process's split chains ([h][P], f64).
int diag_series(gm_dtype dt, const void* x, long long C, long long N, long long P, long long sc,
                long long sd, long long sp, double* cm, double* s2, double* acov_sum,
                DiagScratch& ws, hipStream_t st);
// From R ranks' cm/s2 ([R][P][K/R], K split chains in all) and acov sums ([R][h][P]).
int diag_final(const double* cm, const double* s2, const double* acov, long long K, int R, int h,
               long long P, float* rhat_dev, float* ess_dev, hipStream_t st);
}  // namespace gm
