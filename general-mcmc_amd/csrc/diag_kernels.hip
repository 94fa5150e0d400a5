// diag_kernels.hip — split-R-hat / ESS on the device (stats.rs:419-573).
//
// split_rhat_mean_ess (stats.rs:439-450): the sample is cast to f32
// (stats.rs:443), each chain is split into its first and last h = N/2 draws
// (splitcat, :419-425), and per parameter
//   cm_k = mean_t y_kt, s2_k = sum_t (y_kt - cm_k)^2 / h            (withinvar :456-504)
//   B = sum_k (cm_k - mean cm)^2 * (h / (2C-1)),  W = mean_k s2_k,
//   V = (h-1)/h W + B/h,  R-hat = sqrt(W / V)                       (rhat :452-454)
//   acov_k[l] = sum_{t<h-l} y~_t y~_{t+l} / h                       (autocov_bf :659-681)
//   rho_l = 1 - (W - mean_k acov_k[l]) / V, Geyer initial monotone sum (ess :523-573)
//   ESS = 2C h / tau,  tau = -1 + 2 sum P_i.
// Inputs are rounded to f32 as the reference does; sums are carried in f64
// (the reference's f32 ndarray sums are what the 1e-3 tolerance absorbs).
//
// Three stages so that the multi-GPU path can all-gather the middle products:
//   series_kernel: per split chain k and parameter p -> cm, s2, and acov
//                  summed over the block's chains (partials per chain group)
//   acov_reduce_kernel: partials -> acov_sum[l][p] in fixed group order
//   final_kernel: per parameter, over all (gathered) chains -> R-hat, ESS
#include <hip/hip_runtime.h>

#include "gm_diag.h"

namespace gm {

template <class T>
__device__ __forceinline__ float load_f32(const T* base, long long idx) {
  return (float)base[idx];
}

// blockDim.x = PT * KB: PT parameters (fastest) x KB split chains.
// Dynamic LDS: h * blockDim.x floats (the block's series, t-major) when use_lds.
template <class T>
__global__ void series_kernel(const T* __restrict__ x, long long C, long long N, long long P,
                              long long sc, long long sd, long long sp, int h, int PT, int KB,
                              int use_lds, double* __restrict__ cm, double* __restrict__ s2,
                              double* __restrict__ acov_part /* [G][h][P] */) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int pt = tid % PT, kb = tid / PT;
  const long long nPB = (P + PT - 1) / PT;
  const long long p = (long long)(blockIdx.x % nPB) * PT + pt;
  const long long g = blockIdx.x / nPB;  // chain group
  const long long k = g * KB + kb; // split-chain index in [0, 2C)
  const bool valid = (p < P) && (k < 2 * C);
  const long long chain = valid ? (k < C ? k : k - C) : 0;
  const long long t0 = (k < C) ? 0 : N - h;
  const T* __restrict__ base = x + chain * sc + (valid ? p : 0) * sp;
  const int nth = blockDim.x;
  // pass 1: load to LDS (or not) and the mean
  double sum = 0.0;
  for (int t = 0; t < h; ++t) {
    const float y = valid ? load_f32(base, (t0 + t) * sd) : 0.0f;
    if (use_lds) lds[t * nth + tid] = y;
    sum += (double)y;
  }
  const double mean = valid ? sum / (double)h : 0.0;
  auto Y = [&](int t) -> double {
    const float y = use_lds ? lds[t * nth + tid] : (valid ? load_f32(base, (t0 + t) * sd) : 0.0f);
    return (double)y - mean;
  };
  double sq = 0.0;
  for (int t = 0; t < h; ++t) {
    const double d = Y(t);
    sq += d * d;
  }
  if (valid) {
    cm[k * P + p] = mean;
    s2[k * P + p] = sq / (double)h;
  }
  __syncthreads();  // all series loaded before LDS is reused below
  // autocovariance, summed over the KB chains of this block for each (l, p)
  double* red = (double*)(lds + (use_lds ? (long long)h * nth : 0));
  for (int l = 0; l < h; ++l) {
    double acc = 0.0;
    for (int t = 0; t + l < h; ++t) acc += Y(t) * Y(t + l);
    acc = valid ? acc / (double)h : 0.0;
    // reduce over kb for the same pt (fixed tree order)
    red[tid] = acc;
    __syncthreads();
    for (int w = KB / 2; w >= 1; w >>= 1) {
      if (kb < w) red[tid] = red[tid] + red[tid + w * PT];
      __syncthreads();
    }
    if (kb == 0 && p < P) acov_part[(g * h + l) * P + p] = red[tid];
    __syncthreads();
  }
}

__global__ void acov_reduce_kernel(const double* __restrict__ part, long long G, int h, long long P,
                                   double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)h * P) return;
  double s = 0.0;
  for (long long g = 0; g < G; ++g) s += part[g * h * P + i];
  out[i] = s;
}

// One block (256 threads) per parameter. cm/s2 are [R][2*Cr][P] (R ranks'
// blocks back to back), acov is [R][h][P].
__global__ void final_kernel(const double* __restrict__ cm, const double* __restrict__ s2,
                             const double* __restrict__ acov, long long K /* total split chains */,
                             int R, int h, long long P, float* __restrict__ rhat,
                             float* __restrict__ ess) {
  __shared__ double red[256];
  __shared__ double sh_mean;
  const long long p = blockIdx.x;
  const int tid = threadIdx.x;
  // mean of chain means
  double a = 0.0;
  for (long long k = tid; k < K; k += 256) a += cm[k * P + p];
  red[tid] = a;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) sh_mean = red[0] / (double)K;
  __syncthreads();
  const double mbar = sh_mean;
  __syncthreads();
  double b = 0.0, w2 = 0.0;
  for (long long k = tid; k < K; k += 256) {
    const double d = cm[k * P + p] - mbar;
    b += d * d;
  }
  red[tid] = b;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  const double Bsum = red[0];
  __syncthreads();
  for (long long k = tid; k < K; k += 256) w2 += s2[k * P + p];
  red[tid] = w2;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  const double Wsum = red[0];
  if (tid == 0) {
    const double n = (double)h;
    const double B = Bsum * (n / (double)(K - 1));
    const double W = Wsum / (double)K;
    const double V = ((n - 1.0) / n) * W + B / n;
    rhat[p] = (float)sqrt(W / V);
    // Geyer initial monotone sequence over rho_l (stats.rs:550-567)
    auto rho = [&](int l) -> double {
      double s = 0.0;
      for (int r = 0; r < R; ++r) s += acov[((long long)r * h + l) * P + p];
      const double abar = s / (double)K;
      return 1.0 - (W - abar) / V;
    };
    double mn = (h >= 2) ? rho(0) + rho(1) : 0.0;
    double out = 0.0;
    for (int i = 0; 2 * i + 1 < h; ++i) {
      double pt = rho(2 * i) + rho(2 * i + 1);
      if (pt <= 0.0) break;
      if (pt > mn) pt = mn;
      mn = pt;
      out += pt;
    }
    const double tau = -1.0 + 2.0 * out;
    ess[p] = (float)((1.0 / tau) * (double)K * n);
  }
}

int diag_series(gm_dtype dt, const void* x, long long C, long long N, long long P, long long sc,
                long long sd, long long sp, double* cm, double* s2, double* acov_sum,
                DiagScratch& ws, hipStream_t st) {
  const int h = (int)(N / 2);
  if (h < 1) {
    set_error("split diagnostics need at least 2 draws");
    return GM_EINVAL;
  }
  int PT = 1;
  while (PT < P && PT < 16) PT <<= 1;
  int nth;
  int use_lds = 1;
  if ((long long)h * 256 * 4 + 256 * 8 <= 150 * 1024) nth = 256;
  else if ((long long)h * 128 * 4 + 128 * 8 <= 150 * 1024) nth = 128;
  else if ((long long)h * 64 * 4 + 64 * 8 <= 150 * 1024) nth = 64;
  else {
    nth = 256;
    use_lds = 0;
  }
  if (nth < PT) nth = PT;
  const int KB = nth / PT;
  const long long G = (2 * C + KB - 1) / KB;
  const size_t part_bytes = (size_t)G * h * P * sizeof(double);
  if (ws.part_bytes < part_bytes) {
    if (ws.part) hipFree(ws.part);
    ws.part = nullptr;
    ws.part_bytes = 0;
    if (hipMalloc(&ws.part, part_bytes) != hipSuccess) {
      set_error("diagnostics scratch allocation failed");
      return GM_ENOMEM;
    }
    ws.part_bytes = part_bytes;
  }
  const size_t lds = (use_lds ? (size_t)h * nth * 4 : 0) + (size_t)nth * 8;
  const long long nblk = ((P + PT - 1) / PT) * G;
  if (nblk > 0x7fffffffLL) {
    set_error("diagnostics: problem too large for one launch");
    return GM_EINVAL;
  }
  dim3 grid((unsigned)nblk);
  if (dt == GM_F32)
    hipLaunchKernelGGL(series_kernel<float>, grid, dim3(nth), lds, st, (const float*)x, C, N, P, sc,
                       sd, sp, h, PT, KB, use_lds, cm, s2, (double*)ws.part);
  else
    hipLaunchKernelGGL(series_kernel<double>, grid, dim3(nth), lds, st, (const double*)x, C, N, P,
                       sc, sd, sp, h, PT, KB, use_lds, cm, s2, (double*)ws.part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("series kernel failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  const long long n = (long long)h * P;
  hipLaunchKernelGGL(acov_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (const double*)ws.part, G, h, P, acov_sum);
  e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("acov reduce failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  return GM_OK;
}

int diag_final(const double* cm, const double* s2, const double* acov, long long K, int R, int h,
               long long P, float* rhat_dev, float* ess_dev, hipStream_t st) {
  hipLaunchKernelGGL(final_kernel, dim3((unsigned)P), dim3(256), 0, st, cm, s2, acov, K, R, h, P,
                     rhat_dev, ess_dev);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("final diagnostics kernel failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  return GM_OK;
}

}  // namespace gm
