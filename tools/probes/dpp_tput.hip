// Issue throughput (SIMD cycles per wave-instruction) of plain VALU adds and
// of DPP-fed adds (wave_shl:1), with independent chains (8 per wave) and
// 8 waves per SIMD, so that latency is hidden and only issue cost remains.
// Mixes: all plain, all DPP, 1 DPP per 8, 2 DPP per 16 (the leapfrog's ratio).
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ float shl(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}
template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, long long* cyc, int iters) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = threadIdx.x * 1e-3f + j;
  const float c = 1e-7f;
  __syncthreads();
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bool dpp = MODE == 1 || (MODE == 2 && j == 0 && r == 0) || (MODE == 3 && j == 0);
        v[j] = (dpp ? shl(v[j]) : v[j]) + c;
      }
    }
  }
  long long t1 = clock64();
  float s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int MODE> void run(const char* name) {
  // 256 CUs x 8 blocks of 256 threads = 8 waves per SIMD
  const int blocks = 256 * 8, threads = 256, iters = 2048;
  float* o; long long* c;
  (void)hipMalloc(&o, blocks * threads * 4); (void)hipMalloc(&c, blocks * 8);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, o, c, iters);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, o, c, iters);
  long long* h = new long long[blocks];
  (void)hipMemcpy(h, c, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int b = 0; b < blocks; ++b) m += (double)h[b];
  m /= blocks;
  // per SIMD: 8 waves issue 16 instrs per iteration each
  printf("%-16s : %.2f SIMD cycles per wave-instruction (8 waves/SIMD)\n", name, m / (iters * 16.0 * 8.0));
  delete[] h;
  (void)hipFree(o); (void)hipFree(c);
}
int main() {
  run<0>("plain add");
  run<1>("all dpp add");
  run<2>("1 dpp in 16");
  run<3>("2 dpp in 16");
  return 0;
}
