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

// Variant 3: 32 lanes x 2 coordinates per chain, the two coordinates of a
// lane as one float2 so that the elementwise math issues as v_pk_* ops.
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void lf_pk(float* out, int iters, float eps) {
  const int lane = threadIdx.x & 31;
  const int i0 = 2 * lane;
  const float a = 1.f, b2 = 200.f, b4 = 400.f;
  const f2 b4m = {i0 <= 62 ? b4 : 0.f, i0 + 1 <= 62 ? b4 : 0.f};
  const f2 c2m = {i0 <= 62 ? 2.f : 0.f, i0 + 1 <= 62 ? 2.f : 0.f};
  const f2 b2m = {i0 >= 1 ? b2 : 0.f, b2};
  f2 q = {0.01f * (float)(threadIdx.x + blockIdx.x), 0.02f}, p = {0.3f, 0.2f}, gh = {0.f, 0.f};
  const f2 half = {0.5f * eps, 0.5f * eps}, ev = {eps, eps}, av = {a, a};
  for (int it = 0; it < iters; ++it) {
    p = p + gh;
    q = q + p * ev;
    const f2 xx = q * q;
    // x_{i+1} for the second slot is the next lane's first coordinate,
    // x_{i-1}^2 for the first slot is the previous lane's second square
    // wave-wide shifts; the lanes at the 32-lane chain boundary read the
    // other chain, so select 0 there (as a two-chains-per-wave kernel must)
    float nx = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, q.x), 0x130, 0xf, 0xf, true));
    float pxx = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, xx.y), 0x138, 0xf, 0xf, true));
    nx = (lane == 31) ? 0.f : nx;
    pxx = (lane == 0) ? 0.f : pxx;
    const f2 xn = {q.y, nx}, xp2 = {pxx, xx.x};
    const f2 t = xn - xx, tp = q - xp2;
    const f2 am = av - q;
    const f2 A = (b4m * q) * t + c2m * am;
    const f2 B = b2m * tp;
    const f2 g = A - B;
    gh = g * half;
    p = p + gh;
  }
  out[blockIdx.x * 256 + threadIdx.x] = q.x + q.y + p.x + p.y;
}

float run_pk(int wps, int iters) {
  float* o;
  const int blocks = 256 * wps;
  (void)hipMalloc(&o, blocks * 256 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(lf_pk, dim3(blocks), dim3(256), 0, 0, o, 100, 1e-4f);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(lf_pk, dim3(blocks), dim3(256), 0, 0, o, iters, 1e-4f);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipFree(o);
  return ms * 1e6f / iters / wps / 2;  // two chains per wave: ns per chain-leapfrog slot
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
  for (int rep = 0; rep < 2; ++rep)
  for (int v : {0, 2})
    for (int w : {2, 4, 8}) {
      float ns = v == 0 ? run<0>(w, iters) : v == 1 ? run<1>(w, iters) : run<2>(w, iters);
      printf("%-12s waves/SIMD=%d : %.2f ns per leapfrog per wave (%.1f cycles at 2.17 GHz)\n", names[v], w,
             ns, ns * 2.17f);
    }
  for (int rep = 0; rep < 2; ++rep)
  for (int w : {2, 4, 8}) {
    const float ns = run_pk(w, iters);
    printf("%-12s waves/SIMD=%d : %.2f ns per chain-leapfrog (2 chains per wave) (%.1f cycles)\n", "packed E=2", w,
           ns, ns * 2.17f);
  }
  return 0;
}
