// copy_probe.hip — HBM copy rate of 16-byte-word copy kernels over 1 GiB
// (read + write bytes / event time, median of 20): grid-stride vs one pass,
// words in flight per thread, non-temporal hints.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
typedef unsigned v4u __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_stride(const v4u* __restrict__ s, v4u* __restrict__ d, long long n) {
  const long long stride = (long long)gridDim.x * 256 * U;
  for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
    v4u w[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < n) w[u] = NT ? __builtin_nontemporal_load(&s[i + u * 256]) : s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < n) {
        if (NT) __builtin_nontemporal_store(w[u], &d[i + u * 256]);
        else d[i + u * 256] = w[u];
      }
  }
}
int main() {
  const long long bytes = 1ll << 30, n = bytes / 16;
  v4u *s, *d;
  if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
  hipMemset(s, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto bench = [&](const char* name, auto kern, long long blocks) {
    std::vector<float> t;
    for (int r = 0; r < 25; ++r) {
      hipEventRecord(a);
      hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, 0, s, d, n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 5) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-36s blocks=%-8lld %.0f GB/s\n", name, blocks, 2.0 * bytes / (t[t.size() / 2] * 1e-3) / 1e9);
  };
  bench("stride U4 (engine's copy16)", copy_stride<4, false>, 8192);
  bench("stride U4 32/CU x2", copy_stride<4, false>, 16384);
  bench("stride U8", copy_stride<8, false>, 8192);
  bench("one pass U4", copy_stride<4, false>, n / 1024);
  bench("one pass U1", copy_stride<1, false>, n / 256);
  bench("stride U4 nontemporal", copy_stride<4, true>, 8192);
  bench("one pass U4 nontemporal", copy_stride<4, true>, n / 1024);
  bench("stride U2 2048 blocks", copy_stride<2, false>, 2048);
  return 0;
}
