// Cross-row lane exchange on gfx950: correctness of the candidate l^16 / l^32
// reduction stages and their dependent latency (cycles per stage).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ float sw32_builtin(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
  return __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
}
__device__ __forceinline__ float sw16_builtin(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
  return __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
}
// explicit: a = v, b = v; swap; a + b
__device__ __forceinline__ float sw32_asm(float v) {
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  return a + b;
}
__device__ __forceinline__ float sw16_asm(float v) {
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  return a + b;
}
__device__ __forceinline__ float shfl16(float v) { return v + __shfl_xor(v, 16, 64); }
__device__ __forceinline__ float shfl32(float v) { return v + __shfl_xor(v, 32, 64); }

__global__ void check(const float* in, float* out) {
  const int l = threadIdx.x;
  const float v = in[blockIdx.x * 64 + l];
  float* o = out + blockIdx.x * 64 * 6;
  o[0 * 64 + l] = shfl16(v);
  o[1 * 64 + l] = shfl32(v);
  o[2 * 64 + l] = sw16_builtin(v);
  o[3 * 64 + l] = sw32_builtin(v);
  o[4 * 64 + l] = sw16_asm(v);
  o[5 * 64 + l] = sw32_asm(v);
}

template <int M>
__global__ void lat(const float* in, float* out, long long* cyc, int n) {
  float v = in[threadIdx.x];
  const float c = in[64];
  __syncthreads();
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    if constexpr (M == 0) v = shfl16(v) * c;
    if constexpr (M == 1) v = sw16_builtin(v) * c;
    if constexpr (M == 2) v = sw16_asm(v) * c;
    if constexpr (M == 3) v = v * c + c;
  }
  long long t1 = clock64();
  out[threadIdx.x] = v;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void mul_lat(const uint32_t* in, uint32_t* out, long long* cyc, int n, int wide) {
  uint32_t a = in[threadIdx.x], b = in[threadIdx.x + 64];
  long long t0 = clock64();
  if (wide) {
    for (int i = 0; i < n; ++i) {
      uint64_t p = (uint64_t)a * 0xD2511F53u;
      a = (uint32_t)p ^ (uint32_t)(p >> 32) ^ b;
    }
  } else {
    for (int i = 0; i < n; ++i) {
      uint32_t lo = a * 0xD2511F53u, hi = __umulhi(a, 0xD2511F53u);
      a = lo ^ hi ^ b;
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  const int B = 64;
  float *hin = (float*)malloc(B * 64 * 4), *hout = (float*)malloc(B * 64 * 6 * 4);
  srand(1);
  for (int i = 0; i < B * 64; ++i) hin[i] = (float)rand() / RAND_MAX - 0.5f;
  float *din, *dout;
  hipMalloc(&din, B * 64 * 4);
  hipMalloc(&dout, B * 64 * 6 * 4);
  hipMemcpy(din, hin, B * 64 * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check, dim3(B), dim3(64), 0, 0, din, dout);
  hipMemcpy(hout, dout, B * 64 * 6 * 4, hipMemcpyDeviceToHost);
  int bad[6] = {0};
  for (int b = 0; b < B; ++b)
    for (int l = 0; l < 64; ++l) {
      const float* v = hin + b * 64;
      const float e16 = v[l] + v[l ^ 16], e32 = v[l] + v[l ^ 32];
      const float* o = hout + b * 64 * 6;
      bad[0] += o[0 * 64 + l] != e16;
      bad[1] += o[1 * 64 + l] != e32;
      bad[2] += o[2 * 64 + l] != e16;
      bad[3] += o[3 * 64 + l] != e32;
      bad[4] += o[4 * 64 + l] != e16;
      bad[5] += o[5 * 64 + l] != e32;
    }
  printf("mismatches: shfl16 %d shfl32 %d builtin16 %d builtin32 %d asm16 %d asm32 %d (of %d)\n",
         bad[0], bad[1], bad[2], bad[3], bad[4], bad[5], B * 64);
  long long* dc;
  hipMalloc(&dc, 8);
  const int n = 4096;
  const char* names[4] = {"shfl_xor16+mul", "builtin swap16+mul", "asm swap16(+2 nops)+mul", "fma-like mul+add"};
  for (int m = 0; m < 4; ++m) {
    long long c = 0;
    for (int rep = 0; rep < 3; ++rep) {
      if (m == 0) hipLaunchKernelGGL(lat<0>, dim3(1), dim3(64), 0, 0, din, dout, dc, n);
      if (m == 1) hipLaunchKernelGGL(lat<1>, dim3(1), dim3(64), 0, 0, din, dout, dc, n);
      if (m == 2) hipLaunchKernelGGL(lat<2>, dim3(1), dim3(64), 0, 0, din, dout, dc, n);
      if (m == 3) hipLaunchKernelGGL(lat<3>, dim3(1), dim3(64), 0, 0, din, dout, dc, n);
      hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    }
    printf("%-28s %.2f cycles per iteration\n", names[m], (double)c / n);
  }
  uint32_t* du;
  hipMalloc(&du, 128 * 4);
  hipMemcpy(du, hin, 128 * 4, hipMemcpyHostToDevice);
  for (int w = 0; w < 2; ++w) {
    long long c = 0;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(mul_lat, dim3(1), dim3(64), 0, 0, du, du, dc, n, w);
      hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    }
    printf("%-28s %.2f cycles per iteration\n", w ? "mad_u64_u32 + 2 xor" : "mul_lo+mul_hi + 2 xor", (double)c / n);
  }
  return 0;
}
