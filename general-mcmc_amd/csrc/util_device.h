// util_device.h — batched log-density + gradient of a target (device code
// only; compiled ahead of time by util_kernels.hip and at run time for user
// targets by gm_jit.cpp).
#pragma once
#include "gm_device.h"

namespace gm {

template <class T, int LPC, int E, class TG>
__global__ __launch_bounds__(256) void logp_grad_kernel(long long n, int D, const T* __restrict__ x,
                                                        T* __restrict__ logp, T* __restrict__ grad,
                                                        TG tg_) {
  const long long gtid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long c = gtid / LPC;
  const int lane = (int)(gtid % LPC);
  const auto tg = tg_.template bind<LPC, E>(lane);  // per-lane target view
  if (c >= n) return;
  T q[E], g[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    q[e] = (i < D) ? x[c * D + i] : (T)0;
  }
  const T lp = tg.template eval<LPC, E, true>(q, g, lane);
  if (grad) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      if (i < D) grad[c * D + i] = g[e];
    }
  }
  if (lane == 0 && logp) logp[c] = lp;
}

}  // namespace gm
