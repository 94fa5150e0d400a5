// place_probe.hip — where does the dispatcher put the waves of a
// 1024 x 256-thread grid (the bench's hmc_kernel launch shape)?
// Each wave records XCC, SE, SH, CU, SIMD and its start/end s_memtime while
// it runs a fixed dependent VALU chain. Optional dynamic LDS pad (argv[2]).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(256) void probe(unsigned* rec, int iters) {
  extern __shared__ float pad[];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float x = threadIdx.x * 1e-3f, y = 1.0f;
  for (int i = 0; i < iters; ++i) {
    x = x * 0.999f + y;
    y = y * 0.5f + x * 1e-6f;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {
    const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    rec[w * 6 + 0] = hw;
    rec[w * 6 + 1] = xcc;
    rec[w * 6 + 2] = (unsigned)t0;
    rec[w * 6 + 3] = (unsigned)(t0 >> 32);
    rec[w * 6 + 4] = (unsigned)t1;
    rec[w * 6 + 5] = (x + y == 12345.f) ? 1u : (unsigned)(t1 >> 32);
  }
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1024;
  const size_t lds = argc > 2 ? atol(argv[2]) : 0;
  const int iters = argc > 3 ? atoi(argv[3]) : 200000;
  const int waves = blocks * 4;
  unsigned* d;
  hipMalloc(&d, waves * 6 * 4);
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), lds, 0, d, 1000);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), lds, 0, d, iters);
  hipDeviceSynchronize();
  std::vector<unsigned> h(waves * 6);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  std::map<unsigned, int> per_cu, per_simd;
  unsigned long long tmin = ~0ull, tmax = 0;
  for (int w = 0; w < waves; ++w) {
    const unsigned hw = h[w * 6], xcc = h[w * 6 + 1] & 15;
    const unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7, simd = (hw >> 4) & 3;
    const unsigned key = (xcc << 16) | (se << 8) | (sh << 4) | cu;
    per_cu[key]++;
    per_simd[(key << 2) | simd]++;
    unsigned long long t0 = h[w * 6 + 2] | ((unsigned long long)h[w * 6 + 3] << 32);
    unsigned long long t1 = h[w * 6 + 4] | ((unsigned long long)h[w * 6 + 5] << 32);
    tmin = std::min(tmin, t0);
    tmax = std::max(tmax, t1);
  }
  std::map<int, int> hist_cu, hist_simd;
  for (auto& kv : per_cu) hist_cu[kv.second]++;
  for (auto& kv : per_simd) hist_simd[kv.second]++;
  printf("blocks %d lds %zu: %zu CUs used, %zu SIMDs used, span %llu memtime ticks\n", blocks, lds,
         per_cu.size(), per_simd.size(), tmax - tmin);
  printf("  waves per CU histogram:");
  for (auto& kv : hist_cu) printf(" %d:%d", kv.first, kv.second);
  printf("\n  waves per SIMD histogram:");
  for (auto& kv : hist_simd) printf(" %d:%d", kv.first, kv.second);
  printf("\n");
  return 0;
}
