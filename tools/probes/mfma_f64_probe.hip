// mfma_f64_probe.hip — what the f64 matrix instructions compute, exactly, on
// gfx950, and what they cost: the basis for putting the dense-Gaussian GEMV
// (NUTS cfg3) on the matrix cores bit-exactly.
//
//  1. lane maps of v_mfma_f64_4x4x4_4b_f64 and v_mfma_f64_16x16x4_f64: every
//     candidate (A, B, D) map is checked against small-integer data (exact);
//  2. rounding: D against, per output, (a) the k-ascending fma chain from C,
//     (b) the k-descending chain, (c) rounded products summed left to right,
//     on random doubles with spread exponents and cancellation;
//  3. cost: cycles per instruction, dependent chain (latency) and 4
//     independent accumulators (issue), one wave per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 -o bin/mfma_f64_probe mfma_f64_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k4(const double* a, const double* b, const double* c, double* d, int T) {
  const int l = threadIdx.x;
  for (int t = 0; t < T; ++t)
    d[t * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[t * 64 + l], b[t * 64 + l], c[t * 256 + l], 0, 0, 0);
}
__global__ void k16(const double* a, const double* b, const double* c, double* d, int T) {
  const int l = threadIdx.x;
  for (int t = 0; t < T; ++t) {
    d4 acc = {c[t * 256 + l * 4], c[t * 256 + l * 4 + 1], c[t * 256 + l * 4 + 2], c[t * 256 + l * 4 + 3]};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t * 64 + l], b[t * 64 + l], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[t * 256 + l * 4 + r] = acc[r];
  }
}

// one-hot decode of the 4x4x4_4b maps: A = e_la, B[l] = l + 1, C = 0
__global__ void k4hot(double* d) {
  const int l = threadIdx.x;
  for (int la = 0; la < 64; ++la)
    d[la * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(l == la ? 1.0 : 0.0, (double)(l + 1), 0.0, 0, 0, 0);
}
__global__ void k4hotc(double* d) {  // C one-hot, A = B = 0: where C[l] lands in D
  const int l = threadIdx.x;
  for (int lc = 0; lc < 64; ++lc) d[lc * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(0.0, 0.0, l == lc ? 1.0 : 0.0, 0, 0, 0);
}

// timing: R rounds of N dependent (chains = 1) or 4 independent chains
template <int CH>
__global__ void t4(double* out, int R, long long* cyc) {
  double a = 1.0 + threadIdx.x * 1e-3, b = 0.5;
  double acc[CH];
  for (int i = 0; i < CH; ++i) acc[i] = i;
  const long long t0 = clock64();
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  const long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < CH; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int CH>
__global__ void t16(double* out, int R, long long* cyc) {
  double a = 1.0 + threadIdx.x * 1e-3, b = 0.5;
  d4 acc[CH];
  for (int i = 0; i < CH; ++i) acc[i] = d4{(double)i, 0, 0, 0};
  const long long t0 = clock64();
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  const long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < CH; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

#define CK(e)                                                                          \
  do {                                                                                 \
    hipError_t _e = (e);                                                               \
    if (_e != hipSuccess) {                                                            \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

// host model of one 4x4 block product / one 16x16x4 product for a given k order
enum Mode { FMA_ASC, FMA_DESC, ROUNDED_SUM };
static double dot4(const double* a, const double* b, double c, Mode m) {
  if (m == FMA_ASC) {
    for (int k = 0; k < 4; ++k) c = std::fma(a[k], b[k], c);
    return c;
  }
  if (m == FMA_DESC) {
    for (int k = 3; k >= 0; --k) c = std::fma(a[k], b[k], c);
    return c;
  }
  for (int k = 0; k < 4; ++k) c = c + a[k] * b[k];
  return c;
}

// 4x4x4_4b candidate maps: within block b = l/16, i = l%16; sel bit 0: A[m=i%4][k=i/4] (0) or A[m=i/4][k=i%4] (1);
// bit 1: B[k=i/4][n=i%4] (0) or B[k=i%4][n=i/4] (1); bit 2: D[m=i/4][n=i%4] (0) or D[m=i%4][n=i/4] (1)
// sel 8: the map decoded from the one-hot runs below: lane l = 16r + 4*blk + q holds A[m=q][k=r],
// B[k=r][n=q], C/D[m=r][n=q] of block blk
static void model4(const double* a, const double* b, const double* c, double* d, int sel, Mode mode) {
  if (sel == 8) {
    for (int blk = 0; blk < 4; ++blk) {
      double A[4][4], B[4][4], Cm[4][4];
      for (int r = 0; r < 4; ++r)
        for (int q = 0; q < 4; ++q) {
          const int l = 16 * r + 4 * blk + q;
          A[q][r] = a[l];
          B[r][q] = b[l];
          Cm[r][q] = c[l];
        }
      for (int r = 0; r < 4; ++r)
        for (int q = 0; q < 4; ++q) {
          double ar[4], br[4];
          for (int k = 0; k < 4; ++k) { ar[k] = A[r][k]; br[k] = B[k][q]; }
          d[16 * r + 4 * blk + q] = dot4(ar, br, Cm[r][q], mode);
        }
    }
    return;
  }
  for (int blk = 0; blk < 4; ++blk) {
    double A[4][4], B[4][4], Cm[4][4];
    for (int i = 0; i < 16; ++i) {
      const int l = blk * 16 + i;
      if (sel & 1) A[i / 4][i % 4] = a[l]; else A[i % 4][i / 4] = a[l];
      if (sel & 2) B[i % 4][i / 4] = b[l]; else B[i / 4][i % 4] = b[l];
      if (sel & 4) Cm[i % 4][i / 4] = c[l]; else Cm[i / 4][i % 4] = c[l];
    }
    for (int i = 0; i < 16; ++i) {
      const int l = blk * 16 + i;
      const int m = (sel & 4) ? i % 4 : i / 4, n = (sel & 4) ? i / 4 : i % 4;
      double ar[4], br[4];
      for (int k = 0; k < 4; ++k) { ar[k] = A[m][k]; br[k] = B[k][n]; }
      d[l] = dot4(ar, br, Cm[m][n], mode);
    }
  }
}
// 16x16x4 (guide): A[m=l%16][k=l/16], B[k=l/16][n=l%16], C/D lane l reg r: row (l>>4)+4r, col l&15;
// sel bit 2 flips D to row 4*(l>>4)+r (the non-f64 map) for contrast
static void model16(const double* a, const double* b, const double* c, double* d, int sel, Mode mode) {
  double A[16][4], B[4][16], Cm[16][16];
  for (int l = 0; l < 64; ++l) {
    A[l % 16][l / 16] = a[l];
    B[l / 16][l % 16] = b[l];
    for (int r = 0; r < 4; ++r) {
      const int row = (sel & 4) ? 4 * (l >> 4) + r : (l >> 4) + 4 * r;
      Cm[row][l & 15] = c[l * 4 + r];
    }
  }
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int row = (sel & 4) ? 4 * (l >> 4) + r : (l >> 4) + 4 * r, col = l & 15;
      double ar[4], br[4];
      for (int k = 0; k < 4; ++k) { ar[k] = A[row][k]; br[k] = B[k][col]; }
      d[l * 4 + r] = dot4(ar, br, Cm[row][col], mode);
    }
}

static bool same(double x, double y) { return std::memcmp(&x, &y, 8) == 0; }

int main() {
  const int T = 2000;
  std::mt19937_64 rng(7);
  std::vector<double> a(T * 64), b(T * 64), c(T * 256), d4v(T * 64), d16(T * 256);
  double *da, *db, *dc, *dd;
  CK(hipMalloc(&da, 8 * a.size()));
  CK(hipMalloc(&db, 8 * b.size()));
  CK(hipMalloc(&dc, 8 * c.size()));
  CK(hipMalloc(&dd, 8 * c.size()));
  printf("{");
  for (int phase = 0; phase < 2; ++phase) {  // 0: small integers (maps), 1: spread doubles (rounding)
    std::uniform_int_distribution<int> si(-8, 8), ex(-30, 30);
    std::uniform_real_distribution<double> u(1.0, 2.0);
    auto draw = [&](int t) -> double {
      if (phase == 0) return (double)si(rng);
      const double v = std::ldexp(u(rng), ex(rng)) * ((rng() & 1) ? 1 : -1);
      return (t % 3 == 0) ? std::ldexp(std::nearbyint(std::ldexp(v, 20)), -20) : v;  // some exact-ish values
    };
    for (size_t i = 0; i < a.size(); ++i) a[i] = draw((int)i);
    for (size_t i = 0; i < b.size(); ++i) b[i] = draw((int)i + 1);
    for (size_t i = 0; i < c.size(); ++i) c[i] = draw((int)i + 2);
    CK(hipMemcpy(da, a.data(), 8 * a.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), 8 * b.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dc, c.data(), 8 * c.size(), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k4, dim3(1), dim3(64), 0, 0, da, db, dc, dd, T);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(d4v.data(), dd, 8 * d4v.size(), hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, da, db, dc, dd, T);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(d16.data(), dd, 8 * d16.size(), hipMemcpyDeviceToHost));
    const char* mname[3] = {"fma_k_ascending", "fma_k_descending", "rounded_products_summed"};
    printf("%s\"%s\": {\"mfma_4x4x4_4b\": {", phase ? ", " : "", phase ? "rounding_spread_doubles" : "maps_small_integers");
    for (int sel = 0; sel < 9; ++sel)
      for (int mo = 0; mo < 3; ++mo) {
        if (phase == 0 && mo > 0) continue;
        long long bad = 0;
        std::vector<double> m(64);
        for (int t = 0; t < T; ++t) {
          // c for the 4x4 form: the first 64 of each t's 256
          model4(&a[t * 64], &b[t * 64], &c[t * 256], m.data(), sel, (Mode)mo);
          for (int l = 0; l < 64; ++l) bad += !same(m[l], d4v[t * 64 + l]);
        }
        printf("%s\"sel%d_%s\": %lld", (sel || mo) ? ", " : "", sel, mname[mo], bad);
      }
    printf("}, \"mfma_16x16x4\": {");
    for (int sel = 0; sel < 8; sel += 4)
      for (int mo = 0; mo < 3; ++mo) {
        if (phase == 0 && mo > 0) continue;
        long long bad = 0;
        std::vector<double> m(256);
        for (int t = 0; t < T; ++t) {
          model16(&a[t * 64], &b[t * 64], &c[t * 256], m.data(), sel, (Mode)mo);
          for (int l = 0; l < 256; ++l) bad += !same(m[l], d16[t * 256 + l]);
        }
        printf("%s\"sel%d_%s\": %lld", (sel || mo) ? ", " : "", sel, mname[mo], bad);
      }
    printf("}, \"outputs_per_form\": [%d, %d]}", T * 64, T * 256);
  }
  {
    std::vector<double> h(64 * 64);
    hipLaunchKernelGGL(k4hot, dim3(1), dim3(64), 0, 0, dd);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), dd, 8 * h.size(), hipMemcpyDeviceToHost));
    printf(", \"onehot_A_4x4x4\": [");
    for (int la = 0; la < 64; ++la) {
      printf("%s\"%d:", la ? ", " : "", la);
      for (int l = 0; l < 64; ++l)
        if (h[la * 64 + l] != 0) printf(" %d<-B%d", l, (int)h[la * 64 + l] - 1);
      printf("\"");
    }
    printf("]");
    hipLaunchKernelGGL(k4hotc, dim3(1), dim3(64), 0, 0, dd);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), dd, 8 * h.size(), hipMemcpyDeviceToHost));
    printf(", \"onehot_C_4x4x4\": \"");
    for (int lc = 0; lc < 64; ++lc)
      for (int l = 0; l < 64; ++l)
        if (h[lc * 64 + l] != 0) printf(" C%d->D%d", lc, l);
    printf("\"");
  }
  // timing, one wave per SIMD (1024 waves of 64 on 256 CUs x 4 SIMDs) and one wave alone
  double* dout;
  long long* dcyc;
  CK(hipMalloc(&dout, 8 * 2048 * 64));
  CK(hipMalloc(&dcyc, 8 * 2048));
  const int R = 4096;
  auto run = [&](int which, int blocks, int per) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (which) {
        case 0: hipLaunchKernelGGL(t4<1>, dim3(blocks), dim3(64), 0, 0, dout, R, dcyc); break;
        case 1: hipLaunchKernelGGL(t4<4>, dim3(blocks), dim3(64), 0, 0, dout, R, dcyc); break;
        case 2: hipLaunchKernelGGL(t4<8>, dim3(blocks), dim3(64), 0, 0, dout, R, dcyc); break;
        case 3: hipLaunchKernelGGL(t16<1>, dim3(blocks), dim3(64), 0, 0, dout, R, dcyc); break;
        default: hipLaunchKernelGGL(t16<4>, dim3(blocks), dim3(64), 0, 0, dout, R, dcyc); break;
      }
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
    }
    std::vector<long long> cy(blocks);
    CK(hipMemcpy(cy.data(), dcyc, 8 * blocks, hipMemcpyDeviceToHost));
    double s = 0;
    for (long long v : cy) s += (double)v;
    return s / blocks / ((double)R * per);
  };
  printf(", \"cycles_per_mfma\": {\"f64_4x4x4_4b_dependent\": %.2f, \"f64_4x4x4_4b_4chains\": %.2f, "
         "\"f64_4x4x4_4b_8chains\": %.2f, \"f64_16x16x4_dependent\": %.2f, \"f64_16x16x4_4chains\": %.2f, "
         "\"f64_4x4x4_4b_4chains_2waves_per_simd\": %.2f, \"note\": \"clock64 cycles per instruction per wave\"}}\n",
         run(0, 1024, 1), run(1, 1024, 4), run(2, 1024, 8), run(3, 1024, 1), run(4, 1024, 4), run(1, 2048, 4));
  return 0;
}
