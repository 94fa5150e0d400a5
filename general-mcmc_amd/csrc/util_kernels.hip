// util_kernels.hip — target evaluation (logp_and_grad over a batch of
// points, batched_hmc.rs:18-22 / hmc.rs:42-61) and the sample-layout
// transpose used on egress ([N][C][D] device -> [C][N][D] reference layout,
// hmc.rs:179-180).
#include "util_device.h"
#include "gm_jit.h"
#include "gm_layouts.h"

namespace gm {

// dim > 1024: one point per workgroup (the wide layout of hmc_wide_kernel)
template <class T, int E, class TG>
__global__ __launch_bounds__(gm_wide_max_threads(sizeof(T), E)) void logp_grad_wide_kernel(int D, const T* __restrict__ x,
                                                             T* __restrict__ logp,
                                                             T* __restrict__ grad, TG tg_) {
  __shared__ T xf[2 * GM_WIDE_MAX_WAVES], xl[2 * GM_WIDE_MAX_WAVES], red[GM_WIDE_MAX_WAVES];
  const int tid = threadIdx.x;
  const long long c = blockIdx.x;
  const auto tg = tg_.template bind<64, E>(tid);
  WideCtx<T> cx{tid >> 6, (int)(blockDim.x >> 6), tid & 63, xf, xl, red, 0};
  T q[E], g[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = tid * E + e;
    q[e] = (i < D) ? x[c * D + i] : (T)0;
  }
  const T lp = tg.template eval_wide<E, true>(q, g, cx);
  if (grad) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = tid * E + e;
      if (i < D) grad[c * D + i] = g[e];
    }
  }
  if (tid == 0 && logp) logp[c] = lp;
}

hipError_t launch_logp_grad(gm_dtype dt, const TargetDev& tg, const Layout& lay, long long n,
                            const void* x, void* logp, void* grad, hipStream_t st) {
  if (tg.kind == GM_TARGET_CUSTOM) {  // user target, runtime-compiled (gm_jit.cpp)
    long long nn = n;
    int D = tg.D;
    const void* xx = x;
    void *lp = logp, *gr = grad;
    UserTargetArg ut{tg.params, tg.D};
    void* args[] = {&nn, &D, &xx, &lp, &gr, &ut};
    return jit_launch(JIT_LOGP, dt, tg, (unsigned)((n + 255) / 256), 256, 0, st, args);
  }
  if (layout_is_wide(lay)) {
    if (n == 0) return hipSuccess;
    return dispatch_wide(dt, tg, lay, [&]<class T, int E, class TG>(TG t) -> hipError_t {
      hipLaunchKernelGGL((logp_grad_wide_kernel<T, E, TG>), dim3((unsigned)n), dim3(lay.lanes), 0, st,
                         tg.D, (const T*)x, (T*)logp, (T*)grad, t);
      return hipGetLastError();
    });
  }
  return dispatch(dt, tg, lay, [&]<class T, int LPC, int E, class TG>(TG t) -> hipError_t {
    const long long threads = n * LPC;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    const size_t lds = t.template lds_bytes<LPC, E>();
    hipLaunchKernelGGL((logp_grad_kernel<T, LPC, E, TG>), dim3(blocks), dim3(256), lds, st, n,
                       tg.D, (const T*)x, (T*)logp, (T*)grad, t);
    return hipGetLastError();
  });
}

hipError_t launch_leapfrog_hbm(gm_dtype dt, const TargetDev& tg, const Layout& lay, long long n, void* q,
                               void* p, void* g, void* logp, double eps, hipStream_t st) {
  if (n == 0) return hipSuccess;
  return dispatch(dt, tg, lay, [&]<class T, int LPC, int E, class TG>(TG t) -> hipError_t {
    const long long threads = n * LPC;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    const size_t lds = t.template lds_bytes<LPC, E>();
    hipLaunchKernelGGL((leapfrog_hbm_kernel<T, LPC, E, TG>), dim3(blocks), dim3(256), lds, st, n, tg.D,
                       (T*)q, (T*)p, (T*)g, (T*)logp, (T)eps, t);
    return hipGetLastError();
  });
}

template <class T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                        long long rows, long long C, long long D) {
  const long long total = rows * C * D;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < total;
       k += (long long)gridDim.x * blockDim.x) {
    const long long d = k % D;
    const long long rc = k / D;       // = c*rows + r in dst order
    const long long r = rc % rows;
    const long long c = rc / rows;
    dst[k] = src[(r * C + c) * D + d];
  }
}

// Device-to-device copy in 16-byte words (assign, euclidean.rs:380-382):
// one word per thread in a single pass over the buffer (a grid-stride loop
// only past 2^31 blocks). Measured on 1 GiB (tools/probes/copy_probe.hip,
// profiles/r03/probes/copy_probe.log): 6.15 TB/s, against 5.46 TB/s for
// 4 words per thread over a 8192-block grid-stride loop and 6.03 TB/s for
// the latter with non-temporal hints.
__global__ __launch_bounds__(256) void copy16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                     long long n) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

hipError_t launch_copy16(const void* src, void* dst, long long words, hipStream_t st) {
  if (words <= 0) return hipSuccess;
  long long blocks = (words + 255) / 256;
  if (blocks > 0x7fffffffll) blocks = 0x7fffffffll;
  hipLaunchKernelGGL(copy16_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const uint4*)src, (uint4*)dst,
                     words);
  return hipGetLastError();
}

hipError_t launch_transpose_samples(gm_dtype dt, const void* src, void* dst, long long rows,
                                    long long C, long long D, hipStream_t st) {
  const long long total = rows * C * D;
  if (total == 0) return hipSuccess;
  long long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (dt == GM_F32)
    hipLaunchKernelGGL(transpose_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, st,
                       (const float*)src, (float*)dst, rows, C, D);
  else
    hipLaunchKernelGGL(transpose_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, st,
                       (const double*)src, (double*)dst, rows, C, D);
  return hipGetLastError();
}

}  // namespace gm
