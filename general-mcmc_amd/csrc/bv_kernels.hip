// bv_kernels.hip — the granular BatchVector operations on [n_chains, dim]
// device matrices (euclidean.rs:447-534, the `impl BatchVector for
// Tensor<B, 2>`), for callers that drive the reference's step loop
// (batched_hmc.rs:129-190) op by op instead of through the fused kernel.
//
// Each op is the same arithmetic as the fused HMC kernel's corresponding
// stage: the random fills read the same Philox streams (TAG_MOM / TAG_ACC,
// keyed by global chain id and step), the per-chain reductions use the
// canonical lane-group order of the layout given, and the scalar forms
// round exactly as the kernel does. A step composed of these ops therefore
// equals the fused kernel's step bit for bit (tests/test_gpu_bv.py).
#include "gm_layouts.h"

namespace gm {

template <class F> hipError_t dispatch_layout(gm_dtype dt, const Layout& lay, F&& f) {
#define GM_TRY_LAYOUT_ONLY(L_, E_)                                   \
  if (lay.lanes == L_ && lay.elems == E_) {                          \
    if (dt == GM_F32) return f.template operator()<float, L_, E_>(); \
    return f.template operator()<double, L_, E_>();                  \
  }
  GM_LAYOUT_LIST(GM_TRY_LAYOUT_ONLY)
#undef GM_TRY_LAYOUT_ONLY
  return hipErrorInvalidValue;
}

static unsigned grid_for(long long threads) { return (unsigned)((threads + 255) / 256); }

// kinetic_energy (euclidean.rs:464-472): 0.5 * sum_j p_j^2 per chain
template <class T, int LPC, int E>
__global__ __launch_bounds__(256) void bv_kinetic_kernel(long long C, int D, const T* __restrict__ p,
                                                         T* __restrict__ ke) {
  const long long gtid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long c = gtid / LPC;
  const int lane = (int)(gtid % LPC);
  if (c >= C) return;  // whole lane groups leave together
  T kp = (T)0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    const T v = (i < D) ? p[c * D + i] : (T)0;
    const T sq = v * v;
    kp = (e == 0) ? sq : kp + sq;
  }
  const T k = group_sum<LPC>(kp) * (T)0.5;
  if (lane == 0) ke[c] = k;
}

// masked_assign (euclidean.rs:474-482): x[c,:] = other[c,:] where mask[c]
template <class T>
__global__ void bv_masked_assign_kernel(long long C, int D, T* __restrict__ x, const T* __restrict__ o,
                                        const uint8_t* __restrict__ mask) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= C * D) return;
  if (mask[k / D]) x[k] = o[k];
}

// add_scaled_assign (euclidean.rs:392-394): x = x + other * alpha (two roundings)
template <class T>
__global__ void bv_axpy_kernel(long long n, T* __restrict__ x, const T* __restrict__ o, T alpha) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) x[k] = x[k] + o[k] * alpha;
}

// scale_assign (euclidean.rs:396-398): x = x * alpha; fill_zero (:370-374) as a fill
template <class T>
__global__ void bv_scale_kernel(long long n, T* __restrict__ x, T alpha) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) x[k] = x[k] * alpha;
}
template <class T>
__global__ void bv_fill_kernel(long long n, T* __restrict__ x, T v) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) x[k] = v;
}
// dot (euclidean.rs:400-403): sum over every element of a*b, one block:
// thread t sums elements t, t+1024, ... left to right, then a fixed pairwise
// tree over the 1024 partials (deterministic, summed in T)
template <class T>
__global__ __launch_bounds__(1024) void bv_dot_kernel(long long n, const T* __restrict__ a, const T* __restrict__ b,
                                                      double* __restrict__ out) {
  __shared__ T part[1024];
  T s = (T)0;
  for (long long k = threadIdx.x; k < n; k += 1024) s = s + a[k] * b[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] = part[threadIdx.x] + part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (double)part[0];
}

// fill_random_normal (euclidean.rs:484-496): N(0,1) from the momentum stream,
// the HMC kernels' momentum draws (gm_rng.h momenta_of: the f32 table form)
template <class T>
__global__ void bv_normal_kernel(long long C, int D, T* __restrict__ out, uint64_t seed,
                                 uint32_t chain_offset, uint64_t step, uint32_t tag) {
  __shared__ BmLds32 bm32[1];
  if constexpr (sizeof(T) == 4) {
    bm_lds_fill32(bm32[0]);
    __syncthreads();
  }
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= C * D) return;
  const uint32_t c = (uint32_t)(k / D), i = (uint32_t)(k % D);
  T z[Blk<T>::S];
  momenta_of(draw_block(seed, chain_offset + c, step / Blk<T>::S, tag, i), z, bm32[0]);
  out[k] = pick(z, (int)(step % Blk<T>::S));
}

// sample_uniform (euclidean.rs:498-509): one [0,1) uniform per chain
template <class T>
__global__ void bv_uniform_kernel(long long C, T* __restrict__ out, uint64_t seed, uint32_t chain_offset,
                                  uint64_t step, uint32_t tag) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) out[c] = uniform_co<T>(seed, chain_offset + (uint32_t)c, step, tag, 0u);
}

// energy_sub/add/neg/ln (euclidean.rs:511-525) and accept_mask (527-533)
enum : int { BV_SUB = 0, BV_ADD = 1, BV_NEG = 2, BV_LN = 3 };
template <class T>
__global__ void bv_energy_kernel(int op, long long n, const T* __restrict__ a, const T* __restrict__ b,
                                 T* __restrict__ out) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const T x = a[k];
  T r;
  if (op == BV_SUB) r = x - b[k];
  else if (op == BV_ADD) r = x + b[k];
  else if (op == BV_NEG) r = -x;
  else r = glog(x);
  out[k] = r;
}
template <class T>
__global__ void bv_accept_kernel(long long n, const T* __restrict__ la, const T* __restrict__ lnu,
                                 uint8_t* __restrict__ mask) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) mask[k] = (la[k] >= lnu[k]) ? 1 : 0;  // NaN -> false
}

hipError_t launch_bv_kinetic(gm_dtype dt, const Layout& lay, long long C, int D, const void* p, void* ke,
                             hipStream_t st) {
  return dispatch_layout(dt, lay, [&]<class T, int LPC, int E>() -> hipError_t {
    hipLaunchKernelGGL((bv_kinetic_kernel<T, LPC, E>), dim3(grid_for(C * LPC)), dim3(256), 0, st, C, D,
                       (const T*)p, (T*)ke);
    return hipGetLastError();
  });
}
hipError_t launch_bv_masked_assign(gm_dtype dt, long long C, int D, void* x, const void* o,
                                   const uint8_t* mask, hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_masked_assign_kernel<float>, dim3(grid_for(C * D)), dim3(256), 0, st, C, D,
                       (float*)x, (const float*)o, mask);
  else
    hipLaunchKernelGGL(bv_masked_assign_kernel<double>, dim3(grid_for(C * D)), dim3(256), 0, st, C, D,
                       (double*)x, (const double*)o, mask);
  return hipGetLastError();
}
hipError_t launch_bv_axpy(gm_dtype dt, long long n, void* x, const void* o, double alpha, hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_axpy_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, n, (float*)x,
                       (const float*)o, (float)alpha);
  else
    hipLaunchKernelGGL(bv_axpy_kernel<double>, dim3(grid_for(n)), dim3(256), 0, st, n, (double*)x,
                       (const double*)o, alpha);
  return hipGetLastError();
}
hipError_t launch_bv_scale(gm_dtype dt, long long n, void* x, double alpha, hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_scale_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, n, (float*)x, (float)alpha);
  else
    hipLaunchKernelGGL(bv_scale_kernel<double>, dim3(grid_for(n)), dim3(256), 0, st, n, (double*)x, alpha);
  return hipGetLastError();
}
hipError_t launch_bv_fill(gm_dtype dt, long long n, void* x, double v, hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_fill_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, n, (float*)x, (float)v);
  else
    hipLaunchKernelGGL(bv_fill_kernel<double>, dim3(grid_for(n)), dim3(256), 0, st, n, (double*)x, v);
  return hipGetLastError();
}
hipError_t launch_bv_dot(gm_dtype dt, long long n, const void* a, const void* b, double* out, hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_dot_kernel<float>, dim3(1), dim3(1024), 0, st, n, (const float*)a, (const float*)b, out);
  else
    hipLaunchKernelGGL(bv_dot_kernel<double>, dim3(1), dim3(1024), 0, st, n, (const double*)a, (const double*)b,
                       out);
  return hipGetLastError();
}
hipError_t launch_bv_normal(gm_dtype dt, long long C, int D, void* out, uint64_t seed, uint32_t off,
                            uint64_t step, uint32_t tag, hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_normal_kernel<float>, dim3(grid_for(C * D)), dim3(256), 0, st, C, D, (float*)out,
                       seed, off, step, tag);
  else
    hipLaunchKernelGGL(bv_normal_kernel<double>, dim3(grid_for(C * D)), dim3(256), 0, st, C, D,
                       (double*)out, seed, off, step, tag);
  return hipGetLastError();
}
hipError_t launch_bv_uniform(gm_dtype dt, long long C, void* out, uint64_t seed, uint32_t off, uint64_t step,
                             uint32_t tag, hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_uniform_kernel<float>, dim3(grid_for(C)), dim3(256), 0, st, C, (float*)out, seed,
                       off, step, tag);
  else
    hipLaunchKernelGGL(bv_uniform_kernel<double>, dim3(grid_for(C)), dim3(256), 0, st, C, (double*)out,
                       seed, off, step, tag);
  return hipGetLastError();
}
hipError_t launch_bv_energy(gm_dtype dt, int op, long long n, const void* a, const void* b, void* out,
                            hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_energy_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, op, n, (const float*)a,
                       (const float*)b, (float*)out);
  else
    hipLaunchKernelGGL(bv_energy_kernel<double>, dim3(grid_for(n)), dim3(256), 0, st, op, n,
                       (const double*)a, (const double*)b, (double*)out);
  return hipGetLastError();
}
hipError_t launch_bv_accept(gm_dtype dt, long long n, const void* la, const void* lnu, uint8_t* mask,
                            hipStream_t st) {
  if (dt == GM_F32)
    hipLaunchKernelGGL(bv_accept_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, n, (const float*)la,
                       (const float*)lnu, mask);
  else
    hipLaunchKernelGGL(bv_accept_kernel<double>, dim3(grid_for(n)), dim3(256), 0, st, n, (const double*)la,
                       (const double*)lnu, mask);
  return hipGetLastError();
}

}  // namespace gm
