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

// One leapfrog of every chain with the state in HBM (the reference's
// BatchedGenericHMC::leapfrog loop body, batched_hmc.rs:166-190, as one
// kernel): p += g*(eps/2); q += p*eps; (logp, g) = target(q); p += g*(eps/2),
// the kicks and the drift as the fused hmc_kernel's fused multiply-adds, so
// the same bits as that kernel (the composed tier-2 ops round the product and
// the sum separately, as the reference's add_scaled_assign).
// Per chain-leapfrog it moves exactly SURVEY.md's B_alg = (6D+1)*sizeof(T)
// bytes: the per-leapfrog design the HBM roofline is defined for.
template <class T, int LPC, int E, class TG>
__global__ __launch_bounds__(256) void leapfrog_hbm_kernel(long long n, int D, T* __restrict__ qs,
                                                           T* __restrict__ ps, T* __restrict__ gs,
                                                           T* __restrict__ logp, T eps, TG tg_) {
  const long long gtid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long c = gtid / LPC;
  const int lane = (int)(gtid % LPC);
  const auto tg = tg_.template bind<LPC, E>(lane);  // per-lane target view
  if (c >= n) return;
  const T half = (T)0.5 * eps;
  T q[E], p[E], g[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    q[e] = (i < D) ? qs[c * D + i] : (T)0;
    p[e] = (i < D) ? ps[c * D + i] : (T)0;
    g[e] = (i < D) ? gs[c * D + i] : (T)0;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = gfma(g[e], half, p[e]);
#pragma unroll
  for (int e = 0; e < E; ++e) q[e] = gfma(p[e], eps, q[e]);
  const T lp = tg.template eval<LPC, E, true>(q, g, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = gfma(g[e], half, p[e]);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    if (i < D) {
      qs[c * D + i] = q[e];
      ps[c * D + i] = p[e];
      gs[c * D + i] = g[e];
    }
  }
  if (lane == 0 && logp) logp[c] = lp;
}

}  // namespace gm
