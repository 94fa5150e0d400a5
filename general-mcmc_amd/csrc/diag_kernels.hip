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
//   series_gram_kernel (h <= 64; MFMA) / series_lag_kernel (h > 64):
//                  per split chain k and parameter p -> cm, s2 ([P][2C]), and
//                  acov summed over a chain group's split chains ([G][h][P])
//   acov_reduce_kernel: partials -> acov_sum[l][p] in fixed group order
//   final_kernel: per parameter, over all (gathered) chains -> R-hat, ESS
#include <hip/hip_runtime.h>

#include "gm_diag.h"

namespace gm {

template <class T>
__device__ __forceinline__ float load_f32(const T* base, long long idx) {
  return (float)base[idx];
}

// Fallback for series too long for series_lag_kernel's LDS staging
// (h beyond ~35,000 draws per split chain): the direct per-thread form.
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
    cm[p * 2 * C + k] = mean;
    s2[p * 2 * C + k] = sq / (double)h;
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

// ---------------------------------------------------------------------------
// series_lag_kernel: the same products for h > 64 (long runs), one wave per
// parameter. Block = LT_PT waves = LT_PT consecutive parameters x one chain
// group; the block walks the group's split chains: it stages a split chain's
// h draws of its LT_PT parameters in LDS (rounded to f32 as the reference
// does), each wave centres its parameter's series (mean and within-variance
// by wave reduction, written to cm/s2), and then accumulates the lagged
// products of a block of 512 lags over all t: lane l owns lags
// L0 + 8l + j (j < 8) and keeps the 8 values y~[t + L0 + 8l + j] as a sliding
// register window, so one step of t costs one broadcast read of y~[t], one
// new window read and 8 f64 fma. Series are stored skewed (element i at
// i + i/8) so that the window reads of a wave (8 elements apart) hit distinct
// banks, and zero-padded past h so that no lane tests bounds. The group's sums
// stay in registers across its chains; acov_part[g][l][p] = sum / h. Lags
// beyond 512 take further passes over the group (h > 512 only).
constexpr int LT_PT = 8;                // parameters (waves) per block, at most
constexpr int LT_T = LT_PT * 64;        // threads per block, at most
constexpr int LT_LAGS = 512;            // lags per pass (64 lanes x 8)
__host__ __device__ constexpr int lt_skew(int i) { return i + (i >> 3); }
__host__ __device__ constexpr int lt_stride(int h) { return lt_skew(h + LT_LAGS + 8) + 1; }

template <class T>
__global__ __launch_bounds__(LT_T) void series_lag_kernel(const T* __restrict__ x, long long C, long long N,
                                                          long long P, long long sc, long long sd, long long sp,
                                                          int h, int PT, long long nPT, long long KPG,
                                                          double* __restrict__ cm, double* __restrict__ s2,
                                                          double* __restrict__ acov_part /* [G][h][P] */) {
  extern __shared__ float ys[];  // [PT][stride] skewed series
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nt = PT * 64;
  const long long pt0 = (long long)(blockIdx.x % nPT) * PT;
  const long long g = blockIdx.x / nPT;
  const long long p = pt0 + w;
  const bool pvalid = p < P;
  const int stride = lt_stride(h);
  float* my = ys + w * stride;
  const long long k0 = g * KPG, k1 = (k0 + KPG < 2 * C) ? k0 + KPG : 2 * C;
  // zero the padding once (the series part is rewritten for every chain)
  for (int i = h + lane; i < h + LT_LAGS + 8; i += 64) my[lt_skew(i)] = 0.0f;
  for (int L0 = 0; L0 < h; L0 += LT_LAGS) {
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.0;
    for (long long k = k0; k < k1; ++k) {
      const long long chain = k < C ? k : k - C;
      const long long t0 = k < C ? 0 : N - h;
      __syncthreads();  // the previous series is no longer read
      // stage: consecutive threads take consecutive parameters of one draw
      for (int i = tid; i < h * PT; i += nt) {
        const int t = i / PT, q = i - t * PT;
        const long long pq = pt0 + q;
        ys[q * stride + lt_skew(t)] = pq < P ? load_f32(x + chain * sc + pq * sp, (t0 + t) * sd) : 0.0f;
      }
      __syncthreads();
      // centre (in f64, rounded back to f32 in LDS) and, on the first pass,
      // the split chain's mean and within-variance
      double sum = 0.0;
      for (int t = lane; t < h; t += 64) sum += (double)my[lt_skew(t)];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
      const double mean = sum / (double)h;
      double sq = 0.0;
      for (int t = lane; t < h; t += 64) {
        const double d = (double)my[lt_skew(t)] - mean;
        sq += d * d;
        my[lt_skew(t)] = (float)d;
      }
      if (L0 == 0) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) sq += __shfl_xor(sq, o);
        if (pvalid && lane == 0) {
          cm[p * 2 * C + k] = mean;
          s2[p * 2 * C + k] = sq / (double)h;
        }
      }
      // this wave's own series: its writes above are visible to its reads below
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int base = L0 + 8 * lane;  // this lane's first lag
      double win[8];
#pragma unroll
      for (int j = 0; j < 7; ++j) win[j] = (double)my[lt_skew(base + j)];
      const int tn = h - L0;  // t past which every lag of this pass reads padding
      int t = 0;
      for (; t + 8 <= tn; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          // window slot (u + 7) % 8 takes y~[t + u + base + 7]
          win[(u + 7) & 7] = (double)my[lt_skew(t + u + base + 7)];
          const double a = (double)my[lt_skew(t + u)];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = __builtin_fma(a, win[(u + j) & 7], acc[j]);
        }
      }
      for (; t < tn; ++t) {  // the tail, window kept in order
        win[7] = (double)my[lt_skew(t + base + 7)];
        const double a = (double)my[lt_skew(t)];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = __builtin_fma(a, win[j], acc[j]);
#pragma unroll
        for (int j = 0; j < 7; ++j) win[j] = win[j + 1];
      }
    }
    if (pvalid) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int l = L0 + 8 * lane + j;
        if (l < h) acov_part[(g * h + l) * P + p] = acc[j] / (double)h;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// series_gram_kernel: the same products for h <= 64 with the autocovariance
// on the matrix cores. For one parameter p, summed over split chains k,
//   sum_k acov_k[l] = (1/h) sum_t G[t][t+l],   G = sum_k y~_k y~_k^T  (h x h)
// so a wave owns one parameter and accumulates the upper-triangle 16x16
// tiles of its Gram matrix G with v_mfma_f64_16x16x4_f64 (K = 4 split chains
// per instruction; A = B = the same fragment, lane l holding y~_{k=l/16}
// [t = 16*tb + l%16]). The lag sums are taken once per block at the end.
//
// Block: 512 threads = 8 waves = 8 parameters (GT_PT) x one chain group;
// chains are processed in chunks of GT_KC, staged in LDS as f32 (the
// reference's cast, stats.rs:443) laid out [split][param][t] with an odd row
// stride so the fragment reads are bank-conflict free. Grid: XCD-aware, all
// parameter tiles of one chain group run on the same XCD (blockIdx % 8), so
// each sample cache line is fetched into one L2 only.
constexpr int GT_KC = 8;   // chains per chunk (16 split series = 4 MFMA k-steps)
constexpr int GT_PT = 8;   // parameters per block (one per wave)
constexpr int GT_T = GT_PT * 64;  // threads per block (two blocks per CU at 128 VGPRs)

using f64x4 = __attribute__((ext_vector_type(4))) double;

template <class T>
__global__ __launch_bounds__(GT_T) void series_gram_kernel(
    const T* __restrict__ x, long long C, long long N, long long P, long long sc, long long sd,
    long long sp, int h, int nPT, long long CPG, double* __restrict__ cm, double* __restrict__ s2,
    double* __restrict__ acov_part /* [G][h][P] */) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const int HS = h | 1;
  float* ys = (float*)lds_raw;                             // [2*KC][PT][HS]
  const int ys_floats = 2 * GT_KC * GT_PT * HS;
  const int scr_off = ((ys_floats * 4 > GT_PT * 2048 ? ys_floats * 4 : GT_PT * 2048) + 15) & ~15;
  double* smean = (double*)(lds_raw + scr_off);            // [2*KC][PT]
  const int b = blockIdx.x;
  const int xcd = b & 7, local = b >> 3;
  const int pt = local % nPT;
  const long long g = (long long)(local / nPT) * 8 + xcd;
  const long long p0 = (long long)pt * GT_PT;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const long long p = p0 + wave;
  const bool pvalid = p < P;
  f64x4 acc[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) acc[i] = (f64x4){0.0, 0.0, 0.0, 0.0};
  const long long cbeg = g * CPG;
  const long long cend = (cbeg + CPG < C) ? cbeg + CPG : C;
  for (long long c0 = cbeg; c0 < cend; c0 += GT_KC) {
    __syncthreads();  // the previous chunk's fragments have been read
    {
      // A thread keeps one (chain, parameter) pair and walks the draws: rows
      // r = r0 + RS*it of the 2h kept draws, at most 2*64/RS = 16 per thread
      // (h <= 64), unrolled so that eight loads are in flight together.
      constexpr int RS = GT_T / (GT_PT * GT_KC);
      const int lpp = tid % GT_PT, lc = (tid / GT_PT) % GT_KC, r0 = tid / (GT_PT * GT_KC);
      const long long chain = c0 + lc, gp = p0 + lpp;
      const bool ok = chain < cend && gp < P;
      const T* src = x + (ok ? chain * sc + gp * sp : 0);
      float* dst = ys + (lc * GT_PT + lpp) * HS;
#pragma unroll 8
      for (int it = 0; it < 2 * 64 / RS; ++it) {
        const int r = r0 + it * RS;
        if (r < 2 * h) {
          const int half = r >= h, t = half ? r - h : r;
          const long long tt = half ? N - h + t : t;
          dst[half * GT_KC * GT_PT * HS + t] = ok ? (float)src[tt * sd] : 0.0f;
        }
      }
    }
    __syncthreads();
    if (tid < 2 * GT_KC * GT_PT) {  // one thread per split series: mean, within variance
      const int pp = tid % GT_PT, c = (tid / GT_PT) % GT_KC, half = tid / (GT_PT * GT_KC);
      const float* row = ys + ((half * GT_KC + c) * GT_PT + pp) * HS;
      double sum = 0.0;
      for (int t = 0; t < h; ++t) sum += (double)row[t];
      const long long chain = c0 + c, gp = p0 + pp;
      const bool valid = chain < cend && gp < P;
      const double mean = valid ? sum / (double)h : 0.0;
      double sq = 0.0;
      for (int t = 0; t < h; ++t) {
        const double dv = (double)row[t] - mean;
        sq += dv * dv;
      }
      if (valid) {
        const long long k = half ? C + chain : chain;
        cm[gp * 2 * C + k] = mean;
        s2[gp * 2 * C + k] = sq / (double)h;
      }
      smean[(half * GT_KC + c) * GT_PT + pp] = mean;
    }
    __syncthreads();
    if (pvalid) {
#pragma unroll
      for (int ks = 0; ks < 2 * GT_KC / 4; ++ks) {
        const int k = ks * 4 + (lane >> 4);  // split series of the chunk (= half*KC + c)
        const float* row = ys + (k * GT_PT + wave) * HS;
        const double m = smean[k * GT_PT + wave];
        double f[4];
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) {
          const int t = tb * 16 + (lane & 15);
          f[tb] = (t < h) ? (double)row[t] - m : 0.0;
        }
        int ti = 0;
#pragma unroll
        for (int tb = 0; tb < 4; ++tb)
#pragma unroll
          for (int tb2 = tb; tb2 < 4; ++tb2, ++ti)
            if (tb2 * 16 < h) acc[ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(f[tb], f[tb2], acc[ti], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // LDS is reused as per-wave tile scratch below
  double* scr = (double*)lds_raw + wave * 256;
  double S = 0.0;  // lane = lag
  int ti = 0;
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int tb2 = tb; tb2 < 4; ++tb2, ++ti) {
      if (tb2 * 16 >= h) continue;
      // C/D map of the f64 MFMA: col = lane%16, row = lane/16 + 4*r
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[ti][r];
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int dlt = lane - 16 * (tb2 - tb);  // t' - t = lane  <=>  col = row + dlt
      if (dlt >= -15 && dlt <= 15) {
        for (int row = 0; row < 16; ++row) {
          const int col = row + dlt;
          if (col >= 0 && col < 16 && tb2 * 16 + col < h) S += scr[row * 16 + col];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  if (pvalid && lane < h) acov_part[(g * h + lane) * P + p] = S / (double)h;
}

__global__ void acov_reduce_kernel(const double* __restrict__ part, long long G, int h, long long P,
                                   double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)h * P) return;
  double s = 0.0;
  for (long long g = 0; g < G; ++g) s += part[g * h * P + i];
  out[i] = s;
}

// One block (1024 threads) per parameter. cm/s2 are [R][P][Kl] (each
// rank's block parameter-major, so a parameter's split chains are contiguous;
// Kl = K / R), acov is [R][h][P]. Block sums use a fixed tree order.
constexpr int FIN_T = 1024;
__device__ __forceinline__ double block_sum(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int w = FIN_T / 2; w >= 1; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}
__global__ __launch_bounds__(FIN_T) void final_kernel(const double* __restrict__ cm,
                                                      const double* __restrict__ s2,
                                                      const double* __restrict__ acov,
                                                      long long K /* total split chains */, int R,
                                                      int h, long long P, float* __restrict__ rhat,
                                                      float* __restrict__ ess) {
  __shared__ double red[FIN_T];
  const long long p = blockIdx.x;
  const int tid = threadIdx.x;
  const long long Kl = K / R;
  double a = 0.0, w2 = 0.0;
  for (int r = 0; r < R; ++r) {
    const double* c = cm + ((long long)r * P + p) * Kl;
    const double* v = s2 + ((long long)r * P + p) * Kl;
    for (long long k = tid; k < Kl; k += FIN_T) {
      a += c[k];
      w2 += v[k];
    }
  }
  const double mbar = block_sum(a, red) / (double)K;
  const double Wsum = block_sum(w2, red);
  double b = 0.0;
  for (int r = 0; r < R; ++r) {
    const double* c = cm + ((long long)r * P + p) * Kl;
    for (long long k = tid; k < Kl; k += FIN_T) {
      const double d = c[k] - mbar;
      b += d * d;
    }
  }
  const double Bsum = block_sum(b, red);
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
  auto ensure_part = [&](size_t part_bytes) -> int {
    if (ws.part_bytes >= part_bytes) return GM_OK;
    if (ws.part) hipFree(ws.part);
    ws.part = nullptr;
    ws.part_bytes = 0;
    if (hipMalloc(&ws.part, part_bytes) != hipSuccess) {
      set_error("diagnostics scratch allocation failed");
      return GM_ENOMEM;
    }
    ws.part_bytes = part_bytes;
    return GM_OK;
  };
  long long G;
  hipError_t e;
  if (h <= 64) {
    // matrix-core path: ~512 blocks of 8 waves, chain groups a multiple of 8
    const long long nPT = (P + GT_PT - 1) / GT_PT;
    const long long chunks = (C + GT_KC - 1) / GT_KC;
    G = (512 + nPT - 1) / nPT;
    if (G > chunks) G = chunks;
    G = (G + 7) / 8 * 8;
    long long CPG = (C + G - 1) / G;
    CPG = (CPG + GT_KC - 1) / GT_KC * GT_KC;
    if (nPT * G > 0x7fffffffLL) {
      set_error("diagnostics: problem too large for one launch");
      return GM_EINVAL;
    }
    int rc = ensure_part((size_t)G * h * P * sizeof(double));
    if (rc) return rc;
    const int HS = h | 1;
    const size_t ys_bytes = (size_t)2 * GT_KC * GT_PT * HS * 4;
    const size_t lds = ((ys_bytes > GT_PT * 2048 ? ys_bytes : GT_PT * 2048) + 15) / 16 * 16 +
                       (size_t)2 * GT_KC * GT_PT * sizeof(double);
    dim3 grid((unsigned)(nPT * G));
    if (dt == GM_F32)
      hipLaunchKernelGGL(series_gram_kernel<float>, grid, dim3(GT_T), lds, st, (const float*)x, C, N,
                         P, sc, sd, sp, h, (int)nPT, CPG, cm, s2, (double*)ws.part);
    else
      hipLaunchKernelGGL(series_gram_kernel<double>, grid, dim3(GT_T), lds, st, (const double*)x,
                         C, N, P, sc, sd, sp, h, (int)nPT, CPG, cm, s2, (double*)ws.part);
    e = hipGetLastError();
  } else if ((size_t)lt_stride(h) * sizeof(float) <= 150 * 1024) {
    // long series: ~512 blocks of PT waves (PT parameters, as many as the
    // LDS staging allows, at most LT_PT) over chain groups of split chains
    int PT = (int)((150 * 1024) / ((size_t)lt_stride(h) * sizeof(float)));
    if (PT > LT_PT) PT = LT_PT;
    const long long nPT = (P + PT - 1) / PT;
    G = (512 + nPT - 1) / nPT;
    if (G > 2 * C) G = 2 * C;
    const long long KPG = (2 * C + G - 1) / G;
    G = (2 * C + KPG - 1) / KPG;
    if (nPT * G > 0x7fffffffLL) {
      set_error("diagnostics: problem too large for one launch");
      return GM_EINVAL;
    }
    int rc = ensure_part((size_t)G * h * P * sizeof(double));
    if (rc) return rc;
    const size_t lds = (size_t)PT * lt_stride(h) * sizeof(float);
    dim3 grid((unsigned)(nPT * G));
    if (dt == GM_F32)
      hipLaunchKernelGGL(series_lag_kernel<float>, grid, dim3(PT * 64), lds, st, (const float*)x, C, N, P, sc,
                         sd, sp, h, PT, nPT, KPG, cm, s2, (double*)ws.part);
    else
      hipLaunchKernelGGL(series_lag_kernel<double>, grid, dim3(PT * 64), lds, st, (const double*)x, C, N, P,
                         sc, sd, sp, h, PT, nPT, KPG, cm, s2, (double*)ws.part);
    e = hipGetLastError();
  } else {  // very long series: the direct per-thread kernel
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
    G = (2 * C + KB - 1) / KB;
    int rc = ensure_part((size_t)G * h * P * sizeof(double));
    if (rc) return rc;
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

    e = hipGetLastError();
  }
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
  hipLaunchKernelGGL(final_kernel, dim3((unsigned)P), dim3(FIN_T), 0, st, cm, s2, acov, K, R, h, P,
                     rhat_dev, ess_dev);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("final diagnostics kernel failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  return GM_OK;
}

}  // namespace gm
