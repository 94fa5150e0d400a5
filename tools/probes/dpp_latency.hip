// Dependent-chain latency (cycles per instruction) of plain VALU adds and of
// DPP-fed adds (wave_shl:1, row_shl:1, quad_perm), one wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ void k(float* out, long long* cyc, int iters) {
  float v = threadIdx.x * 1e-3f;
  const float c = 1e-7f;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (MODE == 0) v = v + c;
      if constexpr (MODE == 1) v = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true)) + c;
      if constexpr (MODE == 2) v = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x101, 0xf, 0xf, true)) + c;
      if constexpr (MODE == 3) v = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xf, 0xf, true)) + c;
      if constexpr (MODE == 4) v = v * v + c;
    }
  }
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int MODE> void run(const char* name, int blocks, int threads) {
  float* o; long long* c; int iters = 4096;
  (void)hipMalloc(&o, blocks * threads * 4); (void)hipMalloc(&c, blocks * 8);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, o, c, iters);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, o, c, iters);
  long long h[1]; (void)hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
  printf("%-10s blocks=%4d threads=%4d : %.2f cycles per dependent instr\n", name, blocks, threads,
         (double)h[0] / (iters * 16.0));
  (void)hipFree(o); (void)hipFree(c);
}
int main() {
  for (int th : {64, 256, 1024}) {
    run<0>("add", 256, th); run<1>("wave_shl", 256, th); run<2>("row_shl", 256, th);
    run<3>("quad_perm", 256, th); run<4>("mul+add", 256, th);
  }
  return 0;
}
