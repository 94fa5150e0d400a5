// gemv_mfma_probe.hip — A/B of the dense-Gaussian gradient's batched GEMV
// (w = P d per chain, D = 32, f64; BASELINE configs[2], NUTS cfg3) on the
// vector ALU against the matrix cores, at cfg3's 8192 chains.
//
//  valu: the NUTS kernel's form. 16 lanes x 2 coordinates per chain (4 chains
//        per wave, 2048 waves), P staged in LDS with row stride 32, d published
//        per chain in LDS and read as a broadcast, w_i = fma chain over j.
//  mfma: v_mfma_f64_16x16x4f64 with the chain as the N dimension: 16 chains
//        per wave (lane l <-> chain l % 16, 8 coordinates per lane), P held in
//        registers as the 16 A fragments (2 output tiles x 8 K-steps), d as the
//        B fragment straight from registers (the K order is permuted so that a
//        lane's outputs are its next inputs: no shuffles), 512 waves.
// Each kernel applies the GEMV R times per chain (d <- 0.001 w + d), so the
// time is R dependent GEMVs of every chain; reported per GEMV of all chains.
//
//   hipcc --offload-arch=gfx950 -O3 -o gemv_mfma_probe gemv_mfma_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int D = 32;
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gemv_valu(const double* __restrict__ P, double* __restrict__ x, long long C,
                                                 int R) {
  __shared__ double sp[D * D];
  __shared__ double sd[256 * 2];
  for (int k = threadIdx.x; k < D * D; k += 256) sp[k] = P[k];  // P^T: sp[j*32 + i] = P_ij (symmetric here)
  __syncthreads();
  const long long gt = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long c = gt / 16;
  const int lane = threadIdx.x % 16;
  if (c >= C) return;
  double d[2] = {x[c * D + lane * 2], x[c * D + lane * 2 + 1]};
  double* my = sd + (threadIdx.x / 16) * 32;
  for (int r = 0; r < R; ++r) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    my[lane * 2] = d[0];
    my[lane * 2 + 1] = d[1];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double w0 = 0, w1 = 0;
#pragma unroll 4
    for (int j = 0; j < D; ++j) {
      const double dj = my[j];
      w0 = __builtin_fma(sp[j * D + lane * 2], dj, w0);
      w1 = __builtin_fma(sp[j * D + lane * 2 + 1], dj, w1);
    }
    d[0] = __builtin_fma(0.001, w0, d[0]);
    d[1] = __builtin_fma(0.001, w1, d[1]);
  }
  x[c * D + lane * 2] = d[0];
  x[c * D + lane * 2 + 1] = d[1];
}

// lane l: chain l%16, group g = l/16 holds coordinates c(g, s) = 16*(s/4) + g + 4*(s%4), s = 0..7:
// the f64 16x16x4 C/D map (col = lane&15, row = (lane>>4) + 4*reg) puts output
// row g + 4i of tile mt in lane group g, so a lane's outputs are its next inputs
__device__ __forceinline__ int cidx(int g, int s) { return 16 * (s / 4) + g + 4 * (s % 4); }

__global__ __launch_bounds__(256) void gemv_mfma(const double* __restrict__ P, double* __restrict__ x, long long C,
                                                 int R) {
  const long long wv = ((long long)blockIdx.x * 256 + threadIdx.x) / 64;
  const int l = threadIdx.x % 64, n = l % 16, g = l / 16;
  const long long c = wv * 16 + n;
  if (wv * 16 >= C) return;
  const bool live = c < C;
  // A fragments: tile mt (outputs 16mt..16mt+15), step s: A[m][k] = P[16mt+m][c(k, s)], lane holds m = l%16, k = l/16
  double A[2][8];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int s = 0; s < 8; ++s) A[mt][s] = P[(16 * mt + n) * D + cidx(g, s)];
  double d[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) d[s] = live ? x[c * D + cidx(g, s)] : 0.0;
  for (int r = 0; r < R; ++r) {
    d4 acc[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      acc[mt] = d4{0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < 8; ++s) acc[mt] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[mt][s], d[s], acc[mt], 0, 0, 0);
    }
    // D[row][n] of tile mt at lane l, reg i: row = g + 4i -> coordinate 16mt + g + 4i = c(g, 4mt + i)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) d[4 * mt + i] = __builtin_fma(0.001, acc[mt][i], d[4 * mt + i]);
  }
  if (live)
#pragma unroll
    for (int s = 0; s < 8; ++s) x[c * D + cidx(g, s)] = d[s];
}

#define CK(e)                                                                     \
  do {                                                                            \
    hipError_t _e = (e);                                                          \
    if (_e != hipSuccess) {                                                       \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

int main(int argc, char** argv) {
  const long long C = argc > 1 ? atoll(argv[1]) : 8192;
  const int R = argc > 2 ? atoi(argv[2]) : 200;
  std::vector<double> P(D * D), x0(C * D);
  srand(42);
  for (int i = 0; i < D; ++i)
    for (int j = 0; j <= i; ++j) {
      const double v = (i == j) ? 1.0 + (rand() % 100) / 100.0 : ((rand() % 200) - 100) / 1000.0;
      P[i * D + j] = P[j * D + i] = v;
    }
  for (auto& v : x0) v = ((rand() % 2000) - 1000) / 1000.0;
  double *dP, *dx1, *dx2;
  CK(hipMalloc(&dP, sizeof(double) * D * D));
  CK(hipMalloc(&dx1, sizeof(double) * C * D));
  CK(hipMalloc(&dx2, sizeof(double) * C * D));
  CK(hipMemcpy(dP, P.data(), sizeof(double) * D * D, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned bv = (unsigned)((C * 16 + 255) / 256), bm = (unsigned)(((C + 15) / 16 * 64 + 255) / 256);
  float best_v = 1e30f, best_m = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemcpy(dx1, x0.data(), sizeof(double) * C * D, hipMemcpyHostToDevice));
    CK(hipMemcpy(dx2, x0.data(), sizeof(double) * C * D, hipMemcpyHostToDevice));
    float t;
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(gemv_valu, dim3(bv), dim3(256), 0, 0, dP, dx1, C, R);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t, a, b));
    best_v = t < best_v ? t : best_v;
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(gemv_mfma, dim3(bm), dim3(256), 0, 0, dP, dx2, C, R);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t, a, b));
    best_m = t < best_m ? t : best_m;
  }
  std::vector<double> r1(C * D), r2(C * D);
  CK(hipMemcpy(r1.data(), dx1, sizeof(double) * C * D, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r2.data(), dx2, sizeof(double) * C * D, hipMemcpyDeviceToHost));
  double md = 0;
  for (long long i = 0; i < C * D; ++i) md = fmax(md, fabs(r1[i] - r2[i]) / (1e-300 + fabs(r1[i])));
  const double gf = 2.0 * D * D * C * R / 1e9;
  printf("{\"chains\": %lld, \"rounds\": %d, \"valu_us_per_gemv\": %.4f, \"mfma_us_per_gemv\": %.4f, "
         "\"valu_tflops\": %.2f, \"mfma_tflops\": %.2f, \"mfma_over_valu_time\": %.3f, \"max_rel_diff\": %.3e}\n",
         C, R, best_v * 1e3 / R, best_m * 1e3 / R, gf / best_v * 1e3 / 1e3, gf / best_m * 1e3 / 1e3, best_m / best_v, md);
  return 0;
}
