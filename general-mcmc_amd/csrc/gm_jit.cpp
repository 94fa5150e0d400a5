// gm_jit.cpp — runtime compilation of the sampler kernels around a user
// target (see gm_jit.h). One hiprtc program per (kernel, dtype, dim, source,
// device); the module stays loaded for the life of the process.
#include "gm_jit.h"

#include <hip/hiprtc.h>

#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace gm {

namespace {

const char* kKernelHeader[] = {"hmc_device.h", "mh_device.h", "nuts_device.h", "util_device.h"};
const char* kKernelName[] = {"hmc_kernel", "mh_kernel", "nuts_kernel", "logp_grad_kernel"};

// The adapter between the user's function and the engine's target concept
// (bind / lds_bytes / eval, gm_device.h): one chain per lane, so E = dim and
// no cross-lane work; the user's sums are the chain's sums.
const char* kAdapter = R"GMADAPT(
namespace gm {
template <class T> struct UserTarget {
  const T* params;
  int D;
  template <int LPC, int E> __host__ __device__ size_t lds_bytes() const { return 0; }
  template <int LPC, int E> __device__ __forceinline__ UserTarget bind(int) const { return *this; }
  template <int LPC, int E, bool LOGP>
  __device__ __forceinline__ T eval(const T (&x)[E], T (&g)[E], int) const {
    static_assert(LPC == 1 && E == GM_DIM, "user targets run one chain per lane");
    return gm_logp_grad<T>(x, g, params);
  }
  // one lane per chain: the "part" is the whole log-density
  template <int LPC> static constexpr bool has_part = true;
  template <int LPC, int E>
  __device__ __forceinline__ T eval_part(const T (&x)[E], T (&g)[E], int lane) const {
    return eval<LPC, E, true>(x, g, lane);
  }
  __device__ __forceinline__ T finish(T total) const { return total; }
};
}  // namespace gm
)GMADAPT";

struct Key {
  int which, dt, D, device;
  std::string src;
  bool operator<(const Key& o) const {
    return std::tie(which, dt, D, device, src) < std::tie(o.which, o.dt, o.D, o.device, o.src);
  }
};
std::mutex g_mu;
std::map<Key, hipFunction_t> g_cache;

std::string program_source(JitKernel which, const char* src, int D) {
  std::string s = "#define GM_DIM " + std::to_string(D) + "\n";
  s += std::string("#include \"") + kKernelHeader[which] + "\"\n";
  s += "#line 1 \"user_target\"\n";
  s += src;
  s += "\n";
  s += kAdapter;
  return s;
}

std::string name_expr(JitKernel which, gm_dtype dt, int D) {
  const char* t = dt == GM_F32 ? "float" : "double";
  // the NUTS kernel's last argument: metric handling compiled in (user
  // targets run with or without mass-matrix adaptation from one module)
  return std::string("gm::") + kKernelName[which] + "<" + t + ", 1, " + std::to_string(D) +
         ", gm::UserTarget<" + t + ">" + (which == JIT_NUTS ? ", 2" : "") + " >";
}

// compile; on success fills code and the lowered kernel name
int compile(JitKernel which, gm_dtype dt, const char* src, int D, std::vector<char>* code,
            std::string* lowered) {
  const std::string text = program_source(which, src, D);
  std::vector<const char*> hdr_text(n_jit_headers), hdr_name(n_jit_headers);
  for (int i = 0; i < n_jit_headers; ++i) {
    hdr_text[i] = jit_headers[i].text;
    hdr_name[i] = jit_headers[i].name;
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, text.c_str(), "gm_user_target.hip", n_jit_headers, hdr_text.data(),
                          hdr_name.data()) != HIPRTC_SUCCESS) {
    set_error("hiprtcCreateProgram failed");
    return GM_EINVAL;
  }
  const std::string ne = name_expr(which, dt, D);
  hiprtcAddNameExpression(prog, ne.c_str());
  // the ahead-of-time build's flags (general-mcmc_amd/Makefile): same rounding
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++20", "-ffp-contract=off",
                        "-fno-slp-vectorize"};
  const hiprtcResult r = hiprtcCompileProgram(prog, 5, opts);
  if (r != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    set_error(std::string("user target does not compile (hiprtc): ") + log);
    return GM_EINVAL;
  }
  const char* low = nullptr;
  if (hiprtcGetLoweredName(prog, ne.c_str(), &low) != HIPRTC_SUCCESS || !low) {
    hiprtcDestroyProgram(&prog);
    set_error("hiprtc: kernel name not found");
    return GM_EINVAL;
  }
  *lowered = low;
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code->resize(n);
  hiprtcGetCode(prog, code->data());
  hiprtcDestroyProgram(&prog);
  return GM_OK;
}

int get_function(JitKernel which, gm_dtype dt, const TargetDev& tg, hipFunction_t* fn) {
  int dev = 0;
  hipGetDevice(&dev);
  Key k{(int)which, (int)dt, tg.D, dev, tg.src ? tg.src : ""};
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_cache.find(k);
  if (it != g_cache.end()) {
    *fn = it->second;
    return GM_OK;
  }
  std::vector<char> code;
  std::string lowered;
  int rc = compile(which, dt, k.src.c_str(), tg.D, &code, &lowered);
  if (rc) return rc;
  hipModule_t mod;
  hipError_t e = hipModuleLoadData(&mod, code.data());
  if (e == hipSuccess) e = hipModuleGetFunction(fn, mod, lowered.c_str());
  if (e != hipSuccess) {
    set_error(std::string("loading the user-target kernel failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  g_cache[k] = *fn;
  return GM_OK;
}

}  // namespace

hipError_t jit_launch(JitKernel which, gm_dtype dt, const TargetDev& tg, unsigned grid, unsigned block,
                      size_t lds, hipStream_t st, void** args) {
  hipFunction_t fn;
  if (get_function(which, dt, tg, &fn) != GM_OK) return hipErrorInvalidImage;
  if (grid == 0) return hipSuccess;
  return hipModuleLaunchKernel(fn, grid, 1, 1, block, 1, 1, (unsigned)lds, st, args, nullptr);
}

int jit_prepare(JitKernel which, gm_dtype dt, const TargetDev& tg) {
  hipFunction_t fn;
  return get_function(which, dt, tg, &fn);
}

int jit_compile(JitKernel which, gm_dtype dt, const char* src, int D) {
  std::vector<char> code;
  std::string lowered;
  return compile(which, dt, src, D, &code, &lowered);
}

}  // namespace gm
