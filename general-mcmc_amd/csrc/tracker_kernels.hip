// tracker_kernels.hip — run_progress statistics on the device.
//
// ChainTracker (stats.rs:24-131): the per-step update is fused into the
// MH / NUTS kernels (gm_track.h); here are its initialisation and the
// collect_rhat over all chains' stats (stats.rs:139-193) that the progress
// display reads (core.rs:317-327).
// MultiChainTracker (stats.rs:199-339): HMC::run_progress steps it with the
// current positions at each sync point (hmc.rs:270-290); update, the
// acceptance EMA fold over chains, and rhat.
// Every reduction over chains runs in chain order in f32, as the reference's
// ndarray sum_axis(Axis(0)) and fold do, so results equal the oracle's
// restatement bit for bit.
#include "gm_internal.h"

namespace gm {

template <class T>
__global__ void ct_init_kernel(long long C, int D, const T* __restrict__ q, TrackLaunch t) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < C * D) {
    t.last[k] = (float)q[k];
    t.mean[k] = 0.0f;
    t.msq[k] = 0.0f;
  }
  if (k < C) t.p[k] = -1.0f;  // stats.rs:73
}

// one thread per parameter; thread 0 of block 0 also averages p_accept
__global__ void ct_rhat_kernel(long long C, int D, unsigned long long n_steps, TrackLaunch t,
                               float* __restrict__ rhat, float* __restrict__ p_mean) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const float n = (float)n_steps, nc = (float)C;
  if (p == 0 && p_mean) {
    float s = 0.0f;
    for (long long c = 0; c < C; ++c) s += t.p[c];
    *p_mean = s / nc;
  }
  if (p >= D) return;
  float nsum = 0.0f;
  for (long long c = 0; c < C; ++c) nsum += n;  // sum of the chains' n (stats.rs:186)
  const float navg = nsum / nc;
  float within = 0.0f, gmean = 0.0f, between = 0.0f;
  for (long long c = 0; c < C; ++c) {
    const float m = t.mean[c * D + p];
    within += (t.msq[c * D + p] - m * m) * n / (n - 1.0f);  // sm2 (stats.rs:128)
  }
  within /= nc;
  for (long long c = 0; c < C; ++c) gmean += t.mean[c * D + p];
  gmean /= nc;
  for (long long c = 0; c < C; ++c) {
    const float d = t.mean[c * D + p] - gmean;
    between += d * d;
  }
  between /= (float)(C * (long long)D - 1);  // diffs.len() - 1 (stats.rs:184)
  const float var = between + within * ((navg - 1.0f) / navg);
  rhat[p] = __builtin_sqrtf(var / within);
}

// MultiChainTracker::step: one block per chain row
template <class T>
__global__ void mct_update_kernel(long long C, int P, const T* __restrict__ x, float* __restrict__ mean,
                                  float* __restrict__ msq, float* __restrict__ last, int* __restrict__ flags,
                                  unsigned long long n_after) {
  const long long c = blockIdx.x;
  const float n = (float)n_after, nm1 = n - 1.0f;
  int diff = 0;
  for (int j = threadIdx.x; j < P; j += blockDim.x) {
    const long long k = c * P + j;
    const float xf = (float)x[k];
    mean[k] = (mean[k] * nm1 + xf) / n;
    msq[k] = (n_after == 1) ? xf * xf : (msq[k] * nm1 + xf * xf) / n;
    diff |= xf != last[k];
    last[k] = xf;
  }
  diff = __syncthreads_or(diff);
  if (threadIdx.x == 0) flags[c] = diff;
}
// the acceptance EMA folds over the rows in order (stats.rs:260-265)
__global__ void mct_fold_kernel(long long C, const int* __restrict__ flags, float* __restrict__ p) {
  float v = *p;
  for (long long c = 0; c < C; ++c) v = (1.0f - 0.01f) * v + 0.01f * (flags[c] ? 1.0f : 0.0f);
  *p = v;
}
// MultiChainTracker::rhat (stats.rs:311-338)
__global__ void mct_rhat_kernel(long long C, int P, unsigned long long n_steps, const float* __restrict__ mean,
                                const float* __restrict__ msq, float* __restrict__ rhat) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const float n = (float)n_steps, nc = (float)C;
  const float fac = n / (nc - 1.0f);
  float mc = 0.0f;
  for (long long c = 0; c < C; ++c) mc += mean[c * P + p];
  mc /= nc;
  float between = 0.0f, within = 0.0f;
  for (long long c = 0; c < C; ++c) {
    const float d = mean[c * P + p] - mc;
    between += d * d;
  }
  between *= fac;
  for (long long c = 0; c < C; ++c) {
    const float m = mean[c * P + p];
    within += (msq[c * P + p] - m * m) * n / (n - 1.0f);
  }
  within /= nc;
  const float v = within * ((n - 1.0f) / n) + between * (1.0f / n);
  rhat[p] = __builtin_sqrtf(v / within);
}

hipError_t launch_ct_init(gm_dtype dt, long long C, int D, const void* q, const TrackLaunch& t,
                          hipStream_t st) {
  const long long n = C * D > C ? C * D : C;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  if (dt == GM_F32)
    hipLaunchKernelGGL(ct_init_kernel<float>, dim3(blocks), dim3(256), 0, st, C, D, (const float*)q, t);
  else
    hipLaunchKernelGGL(ct_init_kernel<double>, dim3(blocks), dim3(256), 0, st, C, D, (const double*)q, t);
  return hipGetLastError();
}
hipError_t launch_ct_rhat(long long C, int D, unsigned long long n, const TrackLaunch& t, float* rhat,
                          float* p_mean, hipStream_t st) {
  hipLaunchKernelGGL(ct_rhat_kernel, dim3((D + 63) / 64), dim3(64), 0, st, C, D, n, t, rhat, p_mean);
  return hipGetLastError();
}
hipError_t launch_mct_step(gm_dtype dt, long long C, int P, const void* x, float* mean, float* msq,
                           float* last, int* flags, float* p_accept, unsigned long long n_after,
                           hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(mct_update_kernel<float>, dim3((unsigned)C), dim3(256), 0, st, C, P, (const float*)x,
                       mean, msq, last, flags, n_after);
  else
    hipLaunchKernelGGL(mct_update_kernel<double>, dim3((unsigned)C), dim3(256), 0, st, C, P,
                       (const double*)x, mean, msq, last, flags, n_after);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(mct_fold_kernel, dim3(1), dim3(1), 0, st, C, (const int*)flags, p_accept);
  return hipGetLastError();
}
hipError_t launch_mct_rhat(long long C, int P, unsigned long long n, const float* mean, const float* msq,
                           float* rhat, hipStream_t st) {
  hipLaunchKernelGGL(mct_rhat_kernel, dim3((P + 63) / 64), dim3(64), 0, st, C, P, n, mean, msq, rhat);
  return hipGetLastError();
}

}  // namespace gm
