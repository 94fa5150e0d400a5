// gm_jit.h — user-defined targets compiled at run time (hiprtc).
//
// The reference's targets are user code (Target / GradientTarget traits over
// burn autodiff, distributions.rs:67-110). Here a user target is HIP source
// defining
//     template <class T> __device__ T gm_logp_grad(const T* x, T* g, const T* params);
// for one chain's position x[GM_DIM] (GM_DIM is a macro), writing the gradient
// to g and returning the log-density. gm_jit.cpp compiles the engine's own
// sampler kernels (hmc_device.h, mh_device.h, nuts_device.h, util_device.h)
// around it for the one-chain-per-lane layout (lanes 1, elems = dim), with
// the same flags as the ahead-of-time build, and caches the code per process.
#pragma once
#include "gm_internal.h"

namespace gm {

struct JitHeader {
  const char* name;
  const char* text;
};
extern const JitHeader jit_headers[];  // embedded device headers (build/gm_jit_headers.cpp)
extern const int n_jit_headers;

enum JitKernel { JIT_HMC = 0, JIT_MH = 1, JIT_NUTS = 2, JIT_LOGP = 3 };

// Host mirror of the device adapter gm::UserTarget<T> (kernel argument).
struct UserTargetArg {
  const void* params;
  int D;
};

// Launch kernel `which` for the user target of tg (compiling it on first
// use); args are the kernel's arguments in order, the last one the
// UserTargetArg.
hipError_t jit_launch(JitKernel which, gm_dtype dt, const TargetDev& tg, unsigned grid, unsigned block,
                      size_t lds, hipStream_t st, void** args);
// Compile and load (cached) ahead of the first launch, so that a source that
// does not compile fails at sampler creation with the compiler log.
int jit_prepare(JitKernel which, gm_dtype dt, const TargetDev& tg);
// Compile only (validation of a user source); GM_OK or GM_EINVAL with the log.
int jit_compile(JitKernel which, gm_dtype dt, const char* src, int D);

constexpr int GM_CUSTOM_MAX_DIM = 256;

}  // namespace gm
