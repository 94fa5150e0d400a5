// bank_probe.hip — does a VGPR bank conflict between the two source operands
// of a wave64 VALU instruction cost issue cycles on gfx950? 16 instructions
// per iteration on 8 accumulators (v32..v39); the second operand is in a
// different bank (mode 0), the same bank (mode 1), or an SGPR (mode 2).
#include <hip/hip_runtime.h>
#include <cstdio>
#define S_(x) #x
#define S(x) S_(x)
#define D0(j, c) "v_add_f32 v" S(j) ", v" S(j) ", v" S(c) "\n"
template <int M>
__global__ __launch_bounds__(256) void k(float* out, int iters, float sc) {
  asm volatile(
      "v_mov_b32 v32, 1.0\n v_mov_b32 v33, 1.0\n v_mov_b32 v34, 1.0\n v_mov_b32 v35, 1.0\n"
      "v_mov_b32 v36, 1.0\n v_mov_b32 v37, 1.0\n v_mov_b32 v38, 1.0\n v_mov_b32 v39, 1.0\n"
      "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n" ::
          : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43");
  for (int i = 0; i < iters; ++i) {
    if constexpr (M == 0)
      asm volatile(D0(32, 41) D0(33, 42) D0(34, 43) D0(35, 40) D0(36, 41) D0(37, 42) D0(38, 43) D0(39, 40)
                   D0(32, 41) D0(33, 42) D0(34, 43) D0(35, 40) D0(36, 41) D0(37, 42) D0(38, 43) D0(39, 40) ::
                       : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
    if constexpr (M == 1)
      asm volatile(D0(32, 40) D0(33, 41) D0(34, 42) D0(35, 43) D0(36, 40) D0(37, 41) D0(38, 42) D0(39, 43)
                   D0(32, 40) D0(33, 41) D0(34, 42) D0(35, 43) D0(36, 40) D0(37, 41) D0(38, 42) D0(39, 43) ::
                       : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
    if constexpr (M == 2)
      asm volatile(
          "v_add_f32 v32, %0, v32\n v_add_f32 v33, %0, v33\n v_add_f32 v34, %0, v34\n v_add_f32 v35, %0, v35\n"
          "v_add_f32 v36, %0, v36\n v_add_f32 v37, %0, v37\n v_add_f32 v38, %0, v38\n v_add_f32 v39, %0, v39\n"
          "v_add_f32 v32, %0, v32\n v_add_f32 v33, %0, v33\n v_add_f32 v34, %0, v34\n v_add_f32 v35, %0, v35\n"
          "v_add_f32 v36, %0, v36\n v_add_f32 v37, %0, v37\n v_add_f32 v38, %0, v38\n v_add_f32 v39, %0, v39\n" ::"s"(sc)
          : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
    if constexpr (M == 3)  // literal operand
      asm volatile(
          "v_add_f32 v32, 0x3f8ccccd, v32\n v_add_f32 v33, 0x3f8ccccd, v33\n v_add_f32 v34, 0x3f8ccccd, v34\n v_add_f32 v35, 0x3f8ccccd, v35\n"
          "v_add_f32 v36, 0x3f8ccccd, v36\n v_add_f32 v37, 0x3f8ccccd, v37\n v_add_f32 v38, 0x3f8ccccd, v38\n v_add_f32 v39, 0x3f8ccccd, v39\n"
          "v_add_f32 v32, 0x3f8ccccd, v32\n v_add_f32 v33, 0x3f8ccccd, v33\n v_add_f32 v34, 0x3f8ccccd, v34\n v_add_f32 v35, 0x3f8ccccd, v35\n"
          "v_add_f32 v36, 0x3f8ccccd, v36\n v_add_f32 v37, 0x3f8ccccd, v37\n v_add_f32 v38, 0x3f8ccccd, v38\n v_add_f32 v39, 0x3f8ccccd, v39\n" ::
              : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
    if constexpr (M == 4)  // inline constant operand
      asm volatile(
          "v_add_f32 v32, 1.0, v32\n v_add_f32 v33, 1.0, v33\n v_add_f32 v34, 1.0, v34\n v_add_f32 v35, 1.0, v35\n"
          "v_add_f32 v36, 1.0, v36\n v_add_f32 v37, 1.0, v37\n v_add_f32 v38, 1.0, v38\n v_add_f32 v39, 1.0, v39\n"
          "v_add_f32 v32, 1.0, v32\n v_add_f32 v33, 1.0, v33\n v_add_f32 v34, 1.0, v34\n v_add_f32 v35, 1.0, v35\n"
          "v_add_f32 v36, 1.0, v36\n v_add_f32 v37, 1.0, v37\n v_add_f32 v38, 1.0, v38\n v_add_f32 v39, 1.0, v39\n" ::
              : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
    if constexpr (M == 5)  // v_mad_u64_u32, VGPR multiplier
      asm volatile(
          "v_mad_u64_u32 v[32:33], s[0:1], v40, v41, v[32:33]\n v_mad_u64_u32 v[34:35], s[0:1], v40, v41, v[34:35]\n"
          "v_mad_u64_u32 v[36:37], s[0:1], v40, v41, v[36:37]\n v_mad_u64_u32 v[38:39], s[0:1], v40, v41, v[38:39]\n"
          "v_mad_u64_u32 v[32:33], s[0:1], v40, v41, v[32:33]\n v_mad_u64_u32 v[34:35], s[0:1], v40, v41, v[34:35]\n"
          "v_mad_u64_u32 v[36:37], s[0:1], v40, v41, v[36:37]\n v_mad_u64_u32 v[38:39], s[0:1], v40, v41, v[38:39]\n"
          "v_mad_u64_u32 v[32:33], s[0:1], v40, v41, v[32:33]\n v_mad_u64_u32 v[34:35], s[0:1], v40, v41, v[34:35]\n"
          "v_mad_u64_u32 v[36:37], s[0:1], v40, v41, v[36:37]\n v_mad_u64_u32 v[38:39], s[0:1], v40, v41, v[38:39]\n"
          "v_mad_u64_u32 v[32:33], s[0:1], v40, v41, v[32:33]\n v_mad_u64_u32 v[34:35], s[0:1], v40, v41, v[34:35]\n"
          "v_mad_u64_u32 v[36:37], s[0:1], v40, v41, v[36:37]\n v_mad_u64_u32 v[38:39], s[0:1], v40, v41, v[38:39]\n" ::
              : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "s0", "s1");
    if constexpr (M == 6)  // v_mad_u64_u32, SGPR multiplier
      asm volatile(
          "v_mad_u64_u32 v[32:33], s[0:1], %0, v41, v[32:33]\n v_mad_u64_u32 v[34:35], s[0:1], %0, v41, v[34:35]\n"
          "v_mad_u64_u32 v[36:37], s[0:1], %0, v41, v[36:37]\n v_mad_u64_u32 v[38:39], s[0:1], %0, v41, v[38:39]\n"
          "v_mad_u64_u32 v[32:33], s[0:1], %0, v41, v[32:33]\n v_mad_u64_u32 v[34:35], s[0:1], %0, v41, v[34:35]\n"
          "v_mad_u64_u32 v[36:37], s[0:1], %0, v41, v[36:37]\n v_mad_u64_u32 v[38:39], s[0:1], %0, v41, v[38:39]\n"
          "v_mad_u64_u32 v[32:33], s[0:1], %0, v41, v[32:33]\n v_mad_u64_u32 v[34:35], s[0:1], %0, v41, v[34:35]\n"
          "v_mad_u64_u32 v[36:37], s[0:1], %0, v41, v[36:37]\n v_mad_u64_u32 v[38:39], s[0:1], %0, v41, v[38:39]\n"
          "v_mad_u64_u32 v[32:33], s[0:1], %0, v41, v[32:33]\n v_mad_u64_u32 v[34:35], s[0:1], %0, v41, v[34:35]\n"
          "v_mad_u64_u32 v[36:37], s[0:1], %0, v41, v[36:37]\n v_mad_u64_u32 v[38:39], s[0:1], %0, v41, v[38:39]\n" ::"s"(__float_as_uint(sc))
              : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "s0", "s1");
    if constexpr (M == 7)  // v_xor3 with SGPR key
      asm volatile(
          "v_xor_b32 v32, %0, v32\n v_xor_b32 v33, %0, v33\n v_xor_b32 v34, %0, v34\n v_xor_b32 v35, %0, v35\n"
          "v_xor_b32 v36, %0, v36\n v_xor_b32 v37, %0, v37\n v_xor_b32 v38, %0, v38\n v_xor_b32 v39, %0, v39\n"
          "v_xor_b32 v32, %0, v32\n v_xor_b32 v33, %0, v33\n v_xor_b32 v34, %0, v34\n v_xor_b32 v35, %0, v35\n"
          "v_xor_b32 v36, %0, v36\n v_xor_b32 v37, %0, v37\n v_xor_b32 v38, %0, v38\n v_xor_b32 v39, %0, v39\n" ::"s"(__float_as_uint(sc))
              : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
    if constexpr (M == 8)  // v_xor3 all VGPR
      asm volatile(
          "v_xor_b32 v32, v40, v32\n v_xor_b32 v33, v40, v33\n v_xor_b32 v34, v40, v34\n v_xor_b32 v35, v40, v35\n"
          "v_xor_b32 v36, v40, v36\n v_xor_b32 v37, v40, v37\n v_xor_b32 v38, v40, v38\n v_xor_b32 v39, v40, v39\n"
          "v_xor_b32 v32, v40, v32\n v_xor_b32 v33, v40, v33\n v_xor_b32 v34, v40, v34\n v_xor_b32 v35, v40, v35\n"
          "v_xor_b32 v36, v40, v36\n v_xor_b32 v37, v40, v37\n v_xor_b32 v38, v40, v38\n v_xor_b32 v39, v40, v39\n" ::
              : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
  }
  float r;
  asm volatile("v_add_f32 %0, v32, v39" : "=v"(r));
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
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
    printf("%-14s waves/SIMD=%d : %.3f ns per wave-instr per SIMD\n", name, w, ms * 1e6 / (iters * 16.0 * w));
  }
  (void)hipFree(o);
}
int main() {
  for (int r = 0; r < 2; ++r) {
    run<0>("diff bank");
    run<1>("same bank");
    run<2>("sgpr operand");
    run<3>("literal operand");
    run<4>("inline constant");
    run<5>("mad_u64 vgpr");
    run<6>("mad_u64 sgpr");
    run<7>("xor sgpr");
    run<8>("xor vgpr");
  }
  return 0;
}
