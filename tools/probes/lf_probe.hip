// Cost of the HMC leapfrog body (gm_device.h RosenbrockLane, 64 lanes x 1)
// versus waves per SIMD, and of its parts: variant 0 = as in the kernel,
// 1 = the two DPP lane shifts replaced by plain VALU ops (same count),
// 2 = no coordinate masks. Prints ns per leapfrog per wave slot.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../general-mcmc_amd/csrc/gm_device.h"

using namespace gm;

template <int V>
__global__ __launch_bounds__(256) void lf(float* out, int iters, float eps) {
  const int lane = threadIdx.x & 63;
  RosenbrockT<float> tg;
  tg.a = 1.f; tg.b = 100.f; tg.b2 = 200.f; tg.b4 = 400.f; tg.D = (V == 2) ? 1 << 20 : 64;
  auto t = tg.template bind<64, 1>(lane);
  if (V == 2) { t.ms[0] = ~0u; t.mp[0] = ~0u; }
  float q[1] = {0.01f * (float)(threadIdx.x + blockIdx.x)}, p[1] = {0.3f}, g[1] = {0.f};
  const float half = 0.5f * eps;
  float gh = 0.f;
  for (int it = 0; it < iters; ++it) {
    p[0] = p[0] + gh;
    q[0] = q[0] + p[0] * eps;
    if constexpr (V == 1) {
      // same instruction count without cross-lane moves
      const float x = q[0], nx = x * 1.0001f, px = x * 0.9999f;
      const float tt = nx - x * x, tp = x - px * px;
      const float A = keep((t.b4 * x) * tt + 2.f * (t.a - x), t.ms[0]);
      const float B = keep(t.b2 * tp, t.mp[0]);
      g[0] = A - B;
    } else {
      t.template eval<64, 1, false>(q, g, lane);
    }
    gh = g[0] * half;
    p[0] = p[0] + gh;
  }
  out[blockIdx.x * 256 + threadIdx.x] = q[0] + p[0];
}

template <int V> float run(int wps, int iters) {
  float* o;
  const int blocks = 256 * wps;  // 256 CUs x 4 SIMDs x wps waves (4 waves per block)
  (void)hipMalloc(&o, blocks * 256 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(lf<V>, dim3(blocks), dim3(256), 0, 0, o, 100, 1e-4f);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(lf<V>, dim3(blocks), dim3(256), 0, 0, o, iters, 1e-4f);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipFree(o);
  return ms * 1e6f / iters / wps;  // ns per leapfrog per wave slot
}

int main() {
  const int iters = 20000;
  const char* names[3] = {"kernel body", "no DPP", "no masks"};
  for (int v = 0; v < 3; ++v)
    for (int w : {1, 2, 4, 8}) {
      float ns = v == 0 ? run<0>(w, iters) : v == 1 ? run<1>(w, iters) : run<2>(w, iters);
      printf("%-12s waves/SIMD=%d : %.2f ns per leapfrog per wave (%.1f cycles at 2.17 GHz)\n", names[v], w,
             ns, ns * 2.17f);
    }
  return 0;
}
