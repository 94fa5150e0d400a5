// issue_f64_probe.hip — SIMD cycles per wave64 instruction (throughput) for the
// f64 and 64-bit integer operations of the samplers' RNG and polynomials, with
// VGPR vs SGPR operands, 8 independent chains per wave, 1/2/4/8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
template <int M>
__global__ __launch_bounds__(256) void k(double* out, int iters, double sc) {
  double v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
  double vc = sc * threadIdx.x;
  unsigned u0 = threadIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3, u4 = u0 + 4, u5 = u0 + 5, u6 = u0 + 6, u7 = u0 + 7;
  unsigned uc = threadIdx.x * 7u;
  const unsigned su = __builtin_amdgcn_readfirstlane(iters) * 2654435761u;
  for (int i = 0; i < iters; ++i) {
#define FV(j) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(v##j) : "v"(vc));
#define FS(j) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(v##j) : "s"(sc));
#define AV(j) asm volatile("v_add_f64 %0, %0, %1" : "+v"(v##j) : "v"(vc));
#define AS(j) asm volatile("v_add_f64 %0, %0, %1" : "+v"(v##j) : "s"(sc));
#define XV(j) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u##j) : "v"(uc));
#define XS(j) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(u##j) : "s"(su));
#define MV(j) { unsigned long long t; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(t) : "v"(u##j), "v"(uc) : "vcc"); u##j = (unsigned)(t >> 32) ^ (unsigned)t; }
#define MS(j) { unsigned long long t; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(t) : "v"(u##j), "s"(su) : "vcc"); u##j = (unsigned)(t >> 32) ^ (unsigned)t; }
    if constexpr (M == 0) { R8(FV) R8(FV) }
    if constexpr (M == 1) { R8(FS) R8(FS) }
    if constexpr (M == 2) { R8(AV) R8(AV) }
    if constexpr (M == 3) { R8(AS) R8(AS) }
    if constexpr (M == 4) { R8(XV) R8(XV) }
    if constexpr (M == 5) { R8(XS) R8(XS) }
    if constexpr (M == 6) { R8(MV) R8(MV) }
    if constexpr (M == 7) { R8(MS) R8(MS) }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + (u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7);
}
template <int M> void run(const char* name, int per_iter) {
  const int iters = 20000;
  double* o;
  (void)hipMalloc(&o, 256 * 8 * 256 * 8);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int w : {1, 2, 4, 8}) {
    const int blocks = 256 * w;
    hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, o, 200, 1e-7);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, o, iters, 1e-7);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double cyc = ms * 1e-3 * 2.4e9;  // nominal clock; ratios matter
    printf("%-26s waves/SIMD=%d : %.2f SIMD cycles per wave-instr (@2.4GHz)\n", name, w, cyc / ((double)iters * per_iter * w));
  }
  (void)hipFree(o);
}
int main() {
  run<0>("v_fma_f64 v,v,v", 16);
  run<1>("v_fma_f64 v,s,s", 16);
  run<2>("v_add_f64 v,v", 16);
  run<3>("v_add_f64 v,s", 16);
  run<4>("v_xor_b32 v,v", 16);
  run<5>("v_xor_b32 s,v", 16);
  run<6>("v_mad_u64_u32 v,v (+2 ops)", 48);
  run<7>("v_mad_u64_u32 v,s (+2 ops)", 48);
  return 0;
}
