// issue_probe.hip — SIMD cycles per wave64 VALU instruction (throughput) at
// 2/4/8 waves per SIMD, independent chains, exact instructions via inline asm.
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
template <int M>
__global__ __launch_bounds__(256) void k(float* out, int iters, float sc) {
  float v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
  float vc = sc * threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#define OPV(j) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v##j) : "v"(vc));
#define OPS(j) asm volatile("v_add_f32 %0, %1, %0" : "+v"(v##j) : "s"(sc));
#define OPM(j) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v##j) : "v"(vc));
#define OPD(j) asm volatile("v_add_f32_dpp %0, %0, %1 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v##j) : "v"(vc));
#define OPR(j) asm volatile("v_add_f32_dpp %0, %0, %1 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v##j) : "v"(vc));
#define OPX(j) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(v##j) : "v"(vc));
    if constexpr (M == 0) { R8(OPV) R8(OPV) }
    if constexpr (M == 1) { R8(OPS) R8(OPS) }
    if constexpr (M == 2) { R8(OPM) R8(OPM) }
    if constexpr (M == 3) { R8(OPD) R8(OPD) }
    if constexpr (M == 4) { R8(OPR) R8(OPR) }
    if constexpr (M == 5) { R8(OPV) OPD(0) OPV(1) OPV(2) OPV(3) OPV(4) OPV(5) OPV(6) OPD(7) }
    if constexpr (M == 6) { R8(OPX) R8(OPX) }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
}
template <int M> void run(const char* name) {
  const int iters = 20000;
  float* o;
  (void)hipMalloc(&o, 256 * 8 * 256 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int w : {1, 2, 4, 8}) {
    const int blocks = 256 * w;
    hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, o, 200, 1e-7f);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, o, iters, 1e-7f);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double cyc = ms * 1e-3 * 2.1e9;  // nominal-ish clock; ratios matter
    printf("%-22s waves/SIMD=%d : %.2f SIMD cycles per wave-instr (@2.1GHz)\n", name, w, cyc / (iters * 16.0 * w));
  }
  (void)hipFree(o);
}
int main() {
  run<0>("v_add v,v");
  run<1>("v_add s,v");
  run<2>("v_mul v,v");
  run<3>("v_add_dpp wave_shl");
  run<4>("v_add_dpp row_shl");
  run<5>("14 add + 2 dpp");
  run<6>("v_sub v,v");
  return 0;
}
