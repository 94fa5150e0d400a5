// gm_internal.h — host-side declarations shared by the C ABI (gmcmc_api.cpp)
// and the kernel translation units. Not part of the public boundary.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/gmcmc.h"
#include "gm_launch.h"

namespace gm {

void set_error(const std::string& msg);

// Device-side view of a target (pointers are device memory).
struct TargetDev {
  int kind = 0;
  int D = 0;
  double a = 1, b = 100, std = 1, norm_const = 0;
  const void* mu = nullptr;    // [D] of the sampler dtype
  const void* prec = nullptr;  // [D*D] of the sampler dtype, transposed (prec[j*D+i] = P_ij)
  const char* src = nullptr;     // CUSTOM: user source (interned, lives for the process)
  const void* params = nullptr;  // CUSTOM: [n_params] of the sampler dtype
};

struct Layout {
  int lanes = 64;
  int elems = 1;
};
bool layout_supported(int lanes, int elems);
// one chain per workgroup of lanes/64 waves (HMC only, dim > 1024)
inline bool layout_is_wide(const Layout& l) { return l.lanes > 64; }
bool wide_layout_supported(int lanes, int elems, gm_dtype dt);
// largest dim of the wide path (f32; f64 is half of it)
constexpr int GM_WIDE_MAX_DIM = 16384;
Layout default_layout(int D, gm_dtype dt, int kind);
Layout nuts_wide_default(int D, gm_dtype dt);
bool nuts_wide_layout_supported(int lanes, int elems);  // nuts_wide.hip

// Events a launcher records around its kernel (either may be null).
struct LaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};

// An AOT kernel launch between its timing events (event records on the
// stream; hipExtLaunchKernel's in-dispatch events measured 8-14 us slower per
// call on the host, profiles/r02/launch_ab.json).
template <class... A>
hipError_t launch_timed(void (*k)(A...), dim3 grid, dim3 block, size_t lds, hipStream_t st, LaunchEvents ev,
                        A... args) {
  hipError_t e = ev.start ? hipEventRecord(ev.start, st) : hipSuccess;
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, grid, block, lds, st, args...);
  e = hipGetLastError();
  if (e == hipSuccess && ev.stop) e = hipEventRecord(ev.stop, st);
  return e;
}
// The same events around a launch path that goes through another API (the
// runtime-compiled user-target kernels).
template <class F>
hipError_t with_events(LaunchEvents ev, hipStream_t st, F&& launch) {
  hipError_t e = ev.start ? hipEventRecord(ev.start, st) : hipSuccess;
  if (e == hipSuccess) e = launch();
  if (e == hipSuccess && ev.stop) e = hipEventRecord(ev.stop, st);
  return e;
}

// ---- HMC -------------------------------------------------------------------
hipError_t launch_hmc(gm_dtype dt, const TargetDev& tg, const Layout& lay, const HmcLaunch& a,
                      hipStream_t st, LaunchEvents ev = {});

// ---- run_progress statistics (gm_track.h, tracker_kernels.hip) -------------
// ChainTracker::new for every chain from the current positions
hipError_t launch_ct_init(gm_dtype dt, long long C, int D, const void* q, const TrackLaunch& t,
                          hipStream_t st);
// ChainTracker::stats of every chain + collect_rhat (stats.rs:122-193) -> rhat[D],
// and the mean acceptance EMA over chains -> p_mean[0]
hipError_t launch_ct_rhat(long long C, int D, unsigned long long n, const TrackLaunch& t, float* rhat,
                          float* p_mean, hipStream_t st);
// MultiChainTracker::step / rhat (stats.rs:199-339) on [C][P] positions
hipError_t launch_mct_step(gm_dtype dt, long long C, int P, const void* x, float* mean, float* msq,
                           float* last, int* flags, float* p_accept, unsigned long long n_after,
                           hipStream_t st);
hipError_t launch_mct_rhat(long long C, int P, unsigned long long n, const float* mean, const float* msq,
                           float* rhat, hipStream_t st);

// ---- MH --------------------------------------------------------------------
hipError_t launch_mh(gm_dtype dt, const TargetDev& tg, const Layout& lay, const MhLaunch& a,
                     hipStream_t st, LaunchEvents ev = {});

// ---- target evaluation -----------------------------------------------------
// one leapfrog of n chains, state in HBM (util_device.h leapfrog_hbm_kernel)
hipError_t launch_leapfrog_hbm(gm_dtype dt, const TargetDev& tg, const Layout& lay, long long n, void* q,
                               void* p, void* g, void* logp, double eps, hipStream_t st);
hipError_t launch_logp_grad(gm_dtype dt, const TargetDev& tg, const Layout& lay, long long n,
                            const void* x, void* logp, void* grad, hipStream_t st);

// ---- granular BatchVector ops (bv_kernels.hip) -------------------------------
hipError_t launch_bv_kinetic(gm_dtype dt, const Layout& lay, long long C, int D, const void* p, void* ke,
                             hipStream_t st);
hipError_t launch_bv_masked_assign(gm_dtype dt, long long C, int D, void* x, const void* o,
                                   const uint8_t* mask, hipStream_t st);
hipError_t launch_bv_axpy(gm_dtype dt, long long n, void* x, const void* o, double alpha, hipStream_t st);
hipError_t launch_bv_scale(gm_dtype dt, long long n, void* x, double alpha, hipStream_t st);
hipError_t launch_bv_fill(gm_dtype dt, long long n, void* x, double v, hipStream_t st);
hipError_t launch_bv_dot(gm_dtype dt, long long n, const void* a, const void* b, double* out, hipStream_t st);
hipError_t launch_bv_normal(gm_dtype dt, long long C, int D, void* out, uint64_t seed, uint32_t off,
                            uint64_t step, uint32_t tag, hipStream_t st);
hipError_t launch_bv_uniform(gm_dtype dt, long long C, void* out, uint64_t seed, uint32_t off, uint64_t step,
                             uint32_t tag, hipStream_t st);
hipError_t launch_bv_energy(gm_dtype dt, int op, long long n, const void* a, const void* b, void* out,
                            hipStream_t st);
hipError_t launch_bv_accept(gm_dtype dt, long long n, const void* la, const void* lnu, uint8_t* mask,
                            hipStream_t st);

// target construction (gmcmc_api.cpp): device copies of mean / precision
int build_target(const gm_target* t, gm_dtype dt, long long dim, TargetDev* out, void** d_mu,
                 void** d_prec);

// ---- utilities -------------------------------------------------------------
// [rows][C][D] -> [C][rows][D]
// dst = src in 16-byte words (both 16-byte aligned), util_kernels.hip
hipError_t launch_copy16(const void* src, void* dst, long long words, hipStream_t st);
hipError_t launch_transpose_samples(gm_dtype dt, const void* src, void* dst, long long rows,
                                    long long C, long long D, hipStream_t st);

// roctx ranges when GMCMC_ROCTX=1 and the roctx library can be opened
// (gmcmc_api.cpp); push returns whether a range was opened
bool roctx_push(const char* name);
void roctx_pop();

}  // namespace gm
