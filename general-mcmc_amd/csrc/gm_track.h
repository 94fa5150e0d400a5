// gm_track.h — ChainTracker (stats.rs:24-131) fused into the sampling
// kernels: run_progress steps every chain's tracker after every transition
// (core.rs:146-163 for ChainRunner / MH, generic_nuts.rs:688-704 for NUTS).
// A chain's running mean, mean of squares and last state stay in VGPRs for
// the whole launch; the acceptance EMA is per chain. All f32, in the
// reference's operation order.
#pragma once
#include "gm_device.h"
#include "gm_launch.h"

namespace gm {

template <int LPC, int E> struct ChainTrack {
  float m[E], q[E], l[E];
  float p;
  __device__ __forceinline__ void load(const TrackLaunch& t, long long c, int lane, int D) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      const long long k = c * D + i;
      m[e] = (i < D) ? t.mean[k] : 0.0f;
      q[e] = (i < D) ? t.msq[k] : 0.0f;
      l[e] = (i < D) ? t.last[k] : 0.0f;
    }
    p = t.p[c];
  }
  // ChainTracker::step with n = the count after the increment
  template <class T>
  __device__ __forceinline__ void step(const T (&x)[E], unsigned long long n_after, int lane, int D) {
    const float n = (float)n_after;
    const float nm1 = n - 1.0f;
    int diff = 0, d0 = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      if (i < D) {
        const float xf = (float)x[e];  // to_f32 (stats.rs:94)
        m[e] = (m[e] * nm1 + xf) / n;
        q[e] = (n_after == 1) ? xf * xf : (q[e] * nm1 + xf * xf) / n;
        const int dd = xf != l[e];  // ArrayView::ne: any element differs (NaN differs)
        diff |= dd;
        if (i == 0) d0 = dd;
        l[e] = xf;
      }
    }
    const bool any = group_sum<LPC>(diff) != 0;
    const bool first = group_sum<LPC>(d0) != 0;
    const float p_start = (p >= 0.0f) ? p : (first ? 1.0f : 0.0f);  // stats.rs:108-113
    p = (1.0f - 0.01f) * p_start + 0.01f * (any ? 1.0f : 0.0f);     // ALPHA = 0.01
  }
  // the vectors alone (a kernel short of registers keeps them in memory
  // between transitions: load_vec, step, store_vec; p stays in a register)
  __device__ __forceinline__ void load_vec(const TrackLaunch& t, long long c, int lane, int D) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      const long long k = c * D + i;
      m[e] = (i < D) ? t.mean[k] : 0.0f;
      q[e] = (i < D) ? t.msq[k] : 0.0f;
      l[e] = (i < D) ? t.last[k] : 0.0f;
    }
  }
  __device__ __forceinline__ void store_vec(const TrackLaunch& t, long long c, int lane, int D) const {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      if (i < D) {
        const long long k = c * D + i;
        t.mean[k] = m[e];
        t.msq[k] = q[e];
        t.last[k] = l[e];
      }
    }
  }
  __device__ __forceinline__ void store(const TrackLaunch& t, long long c, int lane, int D) const {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      if (i < D) {
        const long long k = c * D + i;
        t.mean[k] = m[e];
        t.msq[k] = q[e];
        t.last[k] = l[e];
      }
    }
    if (lane == 0) t.p[c] = p;
  }
};

}  // namespace gm
