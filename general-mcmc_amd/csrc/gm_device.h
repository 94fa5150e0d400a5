// gm_device.h — lane-group primitives and built-in targets for the gfx950
// sampling kernels.
//
// Layout: a chain is owned by a group of LPC consecutive lanes of one
// wavefront (LPC in {1,2,...,64}); lane l of the group holds coordinates
// [l*E, (l+1)*E) of the chain in registers. Coordinates >= D are padding and
// stay exactly 0.
//
// Reduction order (the engine's defined summation order, mirrored by the CPU
// oracle): each lane sums its E terms left to right, then an xor butterfly
// over offsets 1,2,4,...,LPC/2. Addition is commutative in IEEE arithmetic, so
// every lane of the group ends with the identical total.
#pragma once
#include "gm_rng.h"

namespace gm {

template <int LPC, class T> __device__ __forceinline__ T group_sum(T v) {
#pragma unroll
  for (int off = 1; off < LPC; off <<= 1) v = v + __shfl_xor(v, off, LPC);
  return v;
}
// lane l of the group receives lane l+1's value (last lane: own value)
template <int LPC, class T> __device__ __forceinline__ T from_next(T v) {
  if constexpr (LPC == 1) return v;
  else return __shfl_down(v, 1, LPC);
}
// lane l of the group receives lane l-1's value (first lane: own value)
template <int LPC, class T> __device__ __forceinline__ T from_prev(T v) {
  if constexpr (LPC == 1) return v;
  else return __shfl_up(v, 1, LPC);
}

// ---------------------------------------------------------------------------
// Rosenbrock: logp = -sum_{i<=D-2} [ b*(x_{i+1}-x_i^2)^2 + (a-x_i)^2 ]
// RosenbrockND (distributions.rs:544-554) is a=1, b=100; Rosenbrock2D
// (distributions.rs:502-515) is D=2 with free a,b. Gradient (analytic form of
// what autodiff computes, hmc.rs:42-61):
//   g_i = [i<=D-2] ( (4b x_i) t_i + 2 (a - x_i) ) - [i>=1] (2b t_{i-1}),
//   t_i = x_{i+1} - x_i^2.
template <class T> struct RosenbrockT {
  T a, b, b2, b4;  // b2 = 2b, b4 = 4b (rounded once, host side)
  int D;
  template <int LPC, int E, bool LOGP>
  __device__ __forceinline__ T eval(const T (&x)[E], T (&g)[E], int lane) const {
    T t[E];
    const T nx = from_next<LPC>(x[0]);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const T xn = (e + 1 < E) ? x[(e + 1 < E) ? e + 1 : e] : nx;
      t[e] = xn - x[e] * x[e];
    }
    const T tp = from_prev<LPC>(t[E - 1]);
    T part = (T)0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      const T tprev = (e > 0) ? t[(e > 0) ? e - 1 : 0] : tp;
      const T am = a - x[e];
      T gi;
      if (i <= D - 2) {
        gi = (b4 * x[e]) * t[e] + (T)2 * am;
        if (i >= 1) gi = gi - b2 * tprev;
      } else if (i == D - 1 && i >= 1) {
        gi = -(b2 * tprev);
      } else {
        gi = (T)0;
      }
      g[e] = gi;
      if (LOGP) {
        const T s = (i <= D - 2) ? (b * (t[e] * t[e]) + am * am) : (T)0;
        part = (e == 0) ? s : part + s;
      }
    }
    if (LOGP) return -group_sum<LPC>(part);
    return (T)0;
  }
};

// IsotropicGaussian as a target (distributions.rs:398-406):
//   logp = (-0.5 * sum x^2) / (std*std),  g = (-x) / (std*std)
template <class T> struct IsoGaussT {
  T var;  // std*std
  int D;
  template <int LPC, int E, bool LOGP>
  __device__ __forceinline__ T eval(const T (&x)[E], T (&g)[E], int lane) const {
    T part = (T)0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      g[e] = (i < D) ? (-x[e]) / var : (T)0;
      if (LOGP) {
        const T s = (i < D) ? x[e] * x[e] : (T)0;
        part = (e == 0) ? s : part + s;
      }
    }
    if (LOGP) return ((T)-0.5 * group_sum<LPC>(part)) / var;
    return (T)0;
  }
};

// Dense Gaussian (DiffableGaussian2D generalised, distributions.rs:257-292):
//   d = x - mu; w_k = sum_j P_kj d_j (j ascending); logp = nc - 0.5*sum_k w_k d_k;
//   g = -w   (= -0.5 (P + P^T) d for symmetric P, the autodiff result)
template <class T> struct GaussT {
  const T* mu;    // [D] device
  const T* prec;  // [D*D] device row-major
  T nc;
  int D;
  template <int LPC, int E, bool LOGP>
  __device__ __forceinline__ T eval(const T (&x)[E], T (&g)[E], int lane) const {
    T d[E], w[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      d[e] = (i < D) ? x[e] - mu[i] : (T)0;
    }
    for (int j = 0; j < D; ++j) {
      T dj;
      // coordinate j lives in lane j/E, slot j%E of this chain's group
      const int src = j / E, slot = j % E;
      T mine = d[0];
#pragma unroll
      for (int e = 1; e < E; ++e) mine = (slot == e) ? d[e] : mine;
      if constexpr (LPC == 1) dj = mine;
      else dj = __shfl(mine, src, LPC);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        const T pij = (i < D) ? prec[(long long)i * D + j] : (T)0;
        w[e] = (j == 0) ? pij * dj : w[e] + pij * dj;
      }
    }
    T part = (T)0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      g[e] = (i < D) ? -w[e] : (T)0;
      if (LOGP) {
        const T s = (i < D) ? w[e] * d[e] : (T)0;
        part = (e == 0) ? s : part + s;
      }
    }
    if (LOGP) return nc - group_sum<LPC>(part) * (T)0.5;
    return (T)0;
  }
};

}  // namespace gm
