// gmcmc_api.cpp — the C ABI (include/gmcmc.h): sampler objects, device
// memory, streams, run orchestration and error reporting.
//
// Orchestration mirrors the reference facades:
//   HMC::new / run / run_positions      hmc.rs:113-181, batched_hmc.rs:62-123
//   MetropolisHastings + ChainRunner    metropolis_hastings.rs:151-197, core.rs:95-115,219-229
//   NUTS::new / run / run_progress      nuts.rs:156-304, generic_nuts.rs:592-753
// but a transition of all chains is one fused kernel step, and many steps run
// inside one launch with the chain state resident in registers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>

#include "gm_jit.h"
#include "gm_layouts.h"
#include "gm_nuts.h"
#include "gm_rng.h"

namespace gm {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

bool layout_supported(int lanes, int elems) {
#define GM_CHECK_LAYOUT(L_, E_) \
  if (lanes == L_ && elems == E_) return true;
  GM_LAYOUT_LIST(GM_CHECK_LAYOUT)
#undef GM_CHECK_LAYOUT
  return false;
}

bool wide_layout_supported(int lanes, int elems, gm_dtype dt) {
  const int esz = dt == GM_F32 ? 4 : 8;
  if (!(elems == 4 || elems == 8 || elems == 16 || (elems == 32 && dt == GM_F32))) return false;
  return lanes > 64 && lanes % 64 == 0 && lanes <= gm_wide_max_threads(esz, elems);
}

static int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// NUTS above 256 dimensions (Rosenbrock, isotropic Gaussian): a chain over
// a workgroup of 2-8 waves (nuts_wide.hip), whose per-lane state fits the
// registers; the one-wave layouts 64 x 8 / 64 x 16 spilled (f64) there.
Layout nuts_wide_default(int D, gm_dtype dt) {
  Layout l;
  if (dt == GM_F32) {
    l.lanes = D <= 512 ? 128 : 256;
    l.elems = 4;
  } else {
    l.lanes = D <= 512 ? 256 : 512;
    l.elems = 2;
  }
  return l;
}

Layout default_layout(int D, gm_dtype dt, int kind) {
  (void)dt;
  Layout l;
  if (kind == GM_TARGET_CUSTOM) {  // user code: one chain per lane
    l.lanes = 1;
    l.elems = D;
    return l;
  }
  if (D > 1024) {
    // wide: the smallest elems whose workgroup holds the chain, so that a
    // chain gets as many waves as possible (few huge chains fill more of the
    // GPU): f32 4 / 8 (1024 threads), 32 (512); f64 4 (1024), 16 (512)
    const int esz = dt == GM_F32 ? 4 : 8;
    const int cand[4] = {4, 8, 16, 32};
    for (int k = 0; k < 4; ++k) {
      const int E = cand[k];
      if (!wide_layout_supported(128, E, dt)) continue;
      const int W = (D + 64 * E - 1) / (64 * E);
      if (W * 64 <= gm_wide_max_threads(esz, E)) {
        l.elems = E;
        l.lanes = 64 * (W < 2 ? 2 : W);
        return l;
      }
    }
    l.elems = 32;
    l.lanes = 512;  // beyond the supported dims (build_target rejects them)
    return l;
  }
  if (D <= 64) {
    l.elems = 1;
    l.lanes = next_pow2(D < 1 ? 1 : D);
  } else if (D <= 128) {
    l.lanes = 64;
    l.elems = 2;
  } else if (D <= 256) {
    l.lanes = 64;
    l.elems = 4;
  } else if (D <= 512) {
    l.lanes = 64;
    l.elems = 8;
  } else {
    l.lanes = 64;
    l.elems = 16;
  }
  return l;
}
}  // namespace gm

using namespace gm;

#define GM_HIP(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) {                                                            \
      set_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " #expr);     \
      return GM_EHIP;                                                                  \
    }                                                                                  \
  } while (0)

#define GM_REQ(cond, msg)      \
  do {                         \
    if (!(cond)) {             \
      set_error(msg);          \
      return GM_EINVAL;        \
    }                          \
  } while (0)

enum SamplerKind { K_HMC = 1, K_MH = 2, K_NUTS = 3 };

// roctx ranges around the sampler entry points (the
// reference times its runs with dev_tools::Timer, here the ranges appear in
// rocprofv3 --marker-trace timelines). Enabled by GMCMC_ROCTX=1 (read once),
// so that the bench's timed call carries no annotation cost by default; the
// roctx library is then opened with dlopen, so libgmcmc.so loads on machines
// without rocprofiler-sdk (and the ranges are silently off there).
namespace gm {
struct RoctxFns {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
};
static const RoctxFns& roctx_fns() {
  static const RoctxFns f = [] {
    RoctxFns r;
    const char* e = std::getenv("GMCMC_ROCTX");
    if (!(e && e[0] == '1')) return r;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return r;
    r.push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
    r.pop = (int (*)())dlsym(h, "roctxRangePop");
    if (!r.push || !r.pop) r.push = nullptr, r.pop = nullptr;
    return r;
  }();
  return f;
}
bool roctx_push(const char* name) {
  const RoctxFns& f = roctx_fns();
  if (!f.push) return false;
  f.push(name);
  return true;
}
void roctx_pop() {
  const RoctxFns& f = roctx_fns();
  if (f.pop) f.pop();
}
}  // namespace gm
struct RoctxRange {
  bool on;
  explicit RoctxRange(const char* name) : on(gm::roctx_push(name)) {}
  ~RoctxRange() {
    if (on) gm::roctx_pop();
  }
};

struct gm_sampler {
  int kind = 0;
  gm_dtype dt = GM_F32;
  size_t esz = 4;
  long long C = 0;
  int D = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  TargetDev tg;
  void* d_mu = nullptr;
  void* d_prec = nullptr;
  double eps = 0;
  int L = 0;
  double prop_std = 1;
  double target_accept = 0.8;
  int max_depth = 10;
  uint64_t seed = 0;
  uint64_t step = 0;
  uint32_t chain_offset = 0;
  void* d_q = nullptr;
  void* d_logp = nullptr;
  long long* d_acc = nullptr;
  void* d_samples = nullptr;
  size_t samples_bytes = 0;
  void* d_tmp = nullptr;
  size_t tmp_bytes = 0;
  void* h_stage[2] = {nullptr, nullptr};  // pinned D2H staging slots (gm_copy_samples)
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  void* d_zs = nullptr;  // wide-layout HMC momentum scratch
  size_t zs_bytes = 0;
  Layout lay;
  bool lay_from_wide = false;  // NUTS: a wide layout replaced for a dense metric (gm_nuts_set_mass_adaptation)
  Layout lay_wide{};            // ... and that layout
  long long steps_per_launch = 1000;
  int lf_unroll = 0;  // HMC leapfrog-loop unroll: 0 by the wave count (hmc_lf_unroll), else 1, 2 or 4
  std::vector<hipEvent_t> evs;
  double last_ms = 0;
  long long last_launches = 0;
  bool last_ms_pending = false;  // HMC/MH: last_ms is read from evs[0..1] on request
  bool async_runs = false;       // HMC/MH runs return after enqueueing (gm_sampler_set_async)
  bool may_async = false;        // set by the entry points that honour async_runs
  long long total_steps = 0;  // transitions since creation
  long long last_rows = 0;    // sample rows produced by the last run
  NutsState nuts;
  // run_progress statistics: per-chain trackers (MH, NUTS) and a
  // MultiChainTracker (HMC), one allocation each (TrackSet)
  void* d_trk = nullptr;
  size_t trk_bytes = 0;
  unsigned long long trk_n = 0;  // ChainTracker steps taken (0: no stats yet)
  void* d_mct = nullptr;
  size_t mct_bytes = 0;
};

// Views into one tracker allocation: mean, msq, last [C*D]; p [C]; flags [C]
// (int); rhat [D]; scalar [1].
struct TrackSet {
  float *mean, *msq, *last, *p, *rhat, *scalar;
  int* flags;
  static size_t bytes(long long C, int D) { return sizeof(float) * (3 * (size_t)C * D + 2 * C + D + 1); }
  TrackSet(void* base, long long C, int D) {
    float* f = (float*)base;
    mean = f;
    msq = f + (size_t)C * D;
    last = f + 2 * (size_t)C * D;
    p = f + 3 * (size_t)C * D;
    flags = (int*)(p + C);
    rhat = (float*)(flags + C);
    scalar = rhat + D;
  }
  TrackLaunch launch() const {
    TrackLaunch t;
    t.mean = mean;
    t.msq = msq;
    t.last = last;
    t.p = p;
    return t;
  }
};

static int ensure_buf(void** p, size_t* cap, size_t need) {
  if (*cap >= need) return GM_OK;
  if (*p) hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (need == 0) return GM_OK;
  hipError_t e = hipMalloc(p, need);
  if (e != hipSuccess) {
    *p = nullptr;
    set_error(std::string("device allocation of ") + std::to_string(need) + " bytes failed: " +
              hipGetErrorString(e));
    return GM_ENOMEM;
  }
  *cap = need;
  return GM_OK;
}

// User sources live as long as the process (kernels compiled from them are
// cached per process); identical sources share one copy.
static const char* intern_source(const char* src) {
  static std::mutex mu;
  static std::set<std::string> pool;
  std::lock_guard<std::mutex> lock(mu);
  return pool.insert(std::string(src)).first->c_str();
}

// Copy a double array to device as dtype.
static int upload_as(gm_dtype dt, const double* src, size_t n, void** dst) {
  const size_t esz = dt == GM_F32 ? 4 : 8;
  std::vector<unsigned char> tmp(n * esz);
  for (size_t i = 0; i < n; ++i) {
    if (dt == GM_F32) {
      float v = (float)src[i];
      memcpy(&tmp[i * 4], &v, 4);
    } else {
      memcpy(&tmp[i * 8], &src[i], 8);
    }
  }
  GM_HIP(hipMalloc(dst, n * esz));
  GM_HIP(hipMemcpy(*dst, tmp.data(), n * esz, hipMemcpyHostToDevice));
  return GM_OK;
}

int gm::build_target(const gm_target* t, gm_dtype dt, long long dim, TargetDev* out, void** d_mu,
                     void** d_prec) {
  GM_REQ(t != nullptr, "target is NULL");
  GM_REQ(t->dim == dim, "target dim does not match the sampler dim");
  GM_REQ(dim >= 1 && dim <= (dt == GM_F32 ? GM_WIDE_MAX_DIM : GM_WIDE_MAX_DIM / 2),
         "dim must be in [1, 16384] (f32) / [1, 8192] (f64)");
  GM_REQ(dim <= 1024 || t->kind == GM_TARGET_ROSENBROCK || t->kind == GM_TARGET_ISO_GAUSS,
         "dim > 1024 is supported for the Rosenbrock and isotropic Gaussian targets");
  out->kind = t->kind;
  out->D = (int)dim;
  out->a = t->a;
  out->b = t->b;
  out->std = t->std;
  out->norm_const = t->norm_const;
  switch (t->kind) {
    case GM_TARGET_ROSENBROCK:
      break;
    case GM_TARGET_ISO_GAUSS:
      GM_REQ(t->std > 0, "ISO_GAUSS std must be > 0");
      break;
    case GM_TARGET_GAUSS: {
      GM_REQ(t->mean != nullptr && t->prec != nullptr, "GAUSS needs mean and prec");
      int rc = upload_as(dt, t->mean, (size_t)dim, d_mu);
      if (rc) return rc;
      {
        // stored transposed, prec_t[j][i] = P[i][j]: lane i of a chain reads
        // column j of its row at consecutive addresses (one or two cache
        // lines per wave per j instead of one line per lane)
        std::vector<double> pt((size_t)(dim * dim));
        for (long long i = 0; i < dim; ++i)
          for (long long j = 0; j < dim; ++j) pt[(size_t)(j * dim + i)] = t->prec[i * dim + j];
        rc = upload_as(dt, pt.data(), (size_t)(dim * dim), d_prec);
      }
      if (rc) return rc;
      out->mu = *d_mu;
      out->prec = *d_prec;
      break;
    }
    case GM_TARGET_CUSTOM: {
      GM_REQ(t->source != nullptr, "CUSTOM needs source");
      GM_REQ(dim <= GM_CUSTOM_MAX_DIM, "CUSTOM targets support dim <= 256 (one chain per lane)");
      GM_REQ(t->n_params >= 0 && (t->n_params == 0 || t->params != nullptr), "bad CUSTOM params");
      out->src = intern_source(t->source);
      // params (at least one slot, so the pointer is never null)
      std::vector<double> pv(t->n_params > 0 ? (size_t)t->n_params : 1, 0.0);
      for (int64_t i = 0; i < t->n_params; ++i) pv[(size_t)i] = t->params[i];
      int rc = upload_as(dt, pv.data(), pv.size(), d_prec);
      if (rc) return rc;
      out->params = *d_prec;
      break;
    }
    default:
      GM_REQ(false, "unknown target kind");
  }
  return GM_OK;
}

extern "C" {

const char* gm_last_error(void) { return g_err.c_str(); }

int gm_device_count(int* count) {
  GM_REQ(count, "count is NULL");
  GM_HIP(hipGetDeviceCount(count));
  return GM_OK;
}

// The calling thread's host waits spin instead of yielding (set before the
// device is first used): a run's completion wait is short and latency-bound,
// and a thread that slept through it comes back with cold caches; measured
// 4 us less wall time on the bench's first timed run
// (profiles/r02/launch_ab.json).
int gm_set_device(int device) {
  GM_HIP(hipSetDevice(device));
  // after hipSetDevice, so that the flag applies to `device` (ignored once
  // that device is initialised)
  hipSetDeviceFlags(hipDeviceScheduleSpin);
  return GM_OK;
}

int gm_device_synchronize(void) {
  GM_HIP(hipDeviceSynchronize());
  return GM_OK;
}

int gm_custom_target_check(const char* source, gm_dtype dtype, int64_t dim, int32_t kind) {
  GM_REQ(source, "source is NULL");
  GM_REQ(dtype == GM_F32 || dtype == GM_F64, "bad dtype");
  GM_REQ(dim >= 1 && dim <= GM_CUSTOM_MAX_DIM, "CUSTOM targets support dim in [1, 256]");
  GM_REQ(kind >= 0 && kind <= 3, "kind: 0 logp/grad, 1 HMC, 2 MH, 3 NUTS");
  const JitKernel jk = kind == 1 ? JIT_HMC : kind == 2 ? JIT_MH : kind == 3 ? JIT_NUTS : JIT_LOGP;
  return jit_compile(jk, dtype, source, (int)dim);
}

// DiffableGaussian2D::new (distributions.rs:229-253); dim > 2 via the
// reference's own Cholesky / inverse (generic_nuts.rs:306-359).
int gm_gauss_from_cov(int64_t dim, const double* cov, double* prec, double* nc) {
  GM_REQ(dim >= 1 && cov && prec && nc, "bad arguments");
  const double pi = 3.14159265358979323846;
  if (dim == 2) {
    const double det = cov[0] * cov[3] - cov[1] * cov[2];
    GM_REQ(det > 0, "covariance is not positive definite");
    const double inv_det = 1.0 / det;
    prec[0] = cov[3] * inv_det;
    prec[1] = -cov[1] * inv_det;
    prec[2] = -cov[2] * inv_det;
    prec[3] = cov[0] * inv_det;
    const double logdet = std::log(det);
    const double two = 1.0 + 1.0;
    *nc = -(two * std::log(two * pi) + logdet) / two;
    return GM_OK;
  }
  const long long n = dim;
  std::vector<double> l(n * n, 0.0), inv_l(n * n, 0.0);
  for (long long i = 0; i < n; ++i)
    for (long long j = 0; j <= i; ++j) {
      double sum = cov[i * n + j];
      for (long long k = 0; k < j; ++k) sum -= l[i * n + k] * l[j * n + k];
      if (i == j) {
        GM_REQ(sum > 0 && std::isfinite(sum), "covariance is not positive definite");
        l[i * n + j] = std::sqrt(sum);
      } else {
        l[i * n + j] = sum / l[j * n + j];
      }
    }
  double logdet = 0;
  for (long long i = 0; i < n; ++i) logdet += 2.0 * std::log(l[i * n + i]);
  for (long long i = 0; i < n; ++i) {
    inv_l[i * n + i] = 1.0 / l[i * n + i];
    for (long long j = i + 1; j < n; ++j) {
      double sum = 0;
      for (long long k = i; k < j; ++k) sum += l[j * n + k] * inv_l[k * n + i];
      inv_l[j * n + i] = -sum / l[j * n + j];
    }
  }
  for (long long i = 0; i < n; ++i)
    for (long long j = 0; j <= i; ++j) {
      double sum = 0;
      for (long long k = (i > j ? i : j); k < n; ++k) sum += inv_l[k * n + i] * inv_l[k * n + j];
      prec[i * n + j] = sum;
      prec[j * n + i] = sum;
    }
  *nc = -((double)n * std::log(2.0 * pi) + logdet) / 2.0;
  return GM_OK;
}

int gm_init_positions_rows(uint64_t seed, int64_t row0, int64_t n, int64_t dim, gm_dtype dtype, void* out) {
  GM_REQ(n >= 0 && dim >= 0 && row0 >= 0 && (out || n * dim == 0), "bad arguments");
  GM_REQ(row0 + n <= 0x100000000LL, "row ids must fit in 32 bits");
  GM_REQ(dtype == GM_F32 || dtype == GM_F64, "bad dtype");
  // rows are independent (keyed by their global id): large requests are
  // split over host threads (a 131,072 x 256 start is 33.5M draws)
  auto rows = [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i)
      for (int64_t d = 0; d < dim; ++d) {
        const double z = normal<double>(seed, (uint32_t)(row0 + i), 0, TAG_INIT, (uint32_t)d);
        if (dtype == GM_F32) ((float*)out)[i * dim + d] = (float)z;
        else ((double*)out)[i * dim + d] = z;
      }
  };
  const int64_t work = n * dim;
  int nt = work >= (1 << 20) ? (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())) : 1;
  if (nt > n) nt = (int)std::max<int64_t>(1, n);
  if (nt <= 1) {
    rows(0, n);
    return GM_OK;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back(rows, n * t / nt, n * (t + 1) / nt);
  for (auto& x : th) x.join();
  return GM_OK;
}

int gm_init_positions(uint64_t seed, int64_t n, int64_t dim, gm_dtype dtype, void* out) {
  return gm_init_positions_rows(seed, 0, n, dim, dtype, out);
}

int gm_target_logp_grad(const gm_target* target, gm_dtype dtype, int64_t n, const void* x,
                        void* logp_out, void* grad_out) {
  GM_REQ(dtype == GM_F32 || dtype == GM_F64, "bad dtype");
  GM_REQ(n >= 0 && (n == 0 || x), "bad arguments");
  GM_REQ(target != nullptr, "target is NULL");
  TargetDev tg;
  void *d_mu = nullptr, *d_prec = nullptr;
  int rc = build_target(target, dtype, target->dim, &tg, &d_mu, &d_prec);
  if (rc) return rc;
  const size_t esz = dtype == GM_F32 ? 4 : 8;
  const long long D = target->dim;
  void *dx = nullptr, *dl = nullptr, *dg = nullptr;
  int out = GM_OK;
  if (n > 0) {
    if (hipMalloc(&dx, n * D * esz) != hipSuccess || hipMalloc(&dl, n * esz) != hipSuccess ||
        hipMalloc(&dg, n * D * esz) != hipSuccess) {
      set_error("device allocation failed");
      out = GM_ENOMEM;
    } else {
      hipMemcpy(dx, x, n * D * esz, hipMemcpyHostToDevice);
      Layout lay = default_layout((int)D, dtype, target->kind);
      hipError_t e = launch_logp_grad(dtype, tg, lay, n, dx, dl, dg, nullptr);
      if (e == hipSuccess) e = hipDeviceSynchronize();
      if (e != hipSuccess) {
        set_error(std::string("logp_grad launch failed: ") + hipGetErrorString(e));
        out = GM_EHIP;
      } else {
        if (logp_out) hipMemcpy(logp_out, dl, n * esz, hipMemcpyDeviceToHost);
        if (grad_out) hipMemcpy(grad_out, dg, n * D * esz, hipMemcpyDeviceToHost);
      }
    }
  }
  if (dx) hipFree(dx);
  if (dl) hipFree(dl);
  if (dg) hipFree(dg);
  if (d_mu) hipFree(d_mu);
  if (d_prec) hipFree(d_prec);
  return out;
}

static int create_common(int kind, const gm_target* target, gm_dtype dtype, int64_t n_chains,
                         int64_t dim, const void* init, int64_t chain_offset, gm_sampler** out) {
  GM_REQ(out != nullptr, "out is NULL");
  *out = nullptr;
  GM_REQ(dtype == GM_F32 || dtype == GM_F64, "bad dtype");
  GM_REQ(n_chains >= 1, "n_chains must be >= 1");
  GM_REQ(init != nullptr, "init is NULL");
  GM_REQ(chain_offset >= 0 && chain_offset + n_chains <= 0xffffffffLL,
         "global chain ids must fit in 32 bits");
  GM_REQ(dim <= 1024 || kind == K_HMC, "dim > 1024 is supported by the HMC sampler only");
  gm_sampler* s = new gm_sampler();
  s->kind = kind;
  s->dt = dtype;
  s->esz = dtype == GM_F32 ? 4 : 8;
  s->C = n_chains;
  s->D = (int)dim;
  s->chain_offset = (uint32_t)chain_offset;
  std::random_device rd;
  s->seed = ((uint64_t)rd() << 32) ^ rd();  // reference: SmallRng::from_rng(thread rng)
  int rc = build_target(target, dtype, dim, &s->tg, &s->d_mu, &s->d_prec);
  if (rc) {
    gm_destroy(s);
    return rc;
  }
  s->lay = default_layout((int)dim, dtype, target->kind);
  if (target->kind == GM_TARGET_CUSTOM) {
    // compile the user target into this sampler's kernel now, so that a
    // source error surfaces here with the compiler log
    const JitKernel jk = kind == K_HMC ? JIT_HMC : kind == K_MH ? JIT_MH : JIT_NUTS;
    rc = jit_prepare(jk, dtype, s->tg);
    if (rc) {
      const std::string msg = gm_last_error();
      gm_destroy(s);
      set_error(msg);
      return rc;
    }
  } else if (kind == K_NUTS && dim > 16 && dim <= 64) {
    // NUTS: two coordinates per lane halve the lanes that wait in each
    // per-chain reduction and put twice the chains in a wave (measured at
    // 8192 x 32-D f64: 1.47x over 32x1 for the dense Gaussian, 1.07x for the
    // isotropic one)
    s->lay.lanes = next_pow2((int)dim) / 2;
    s->lay.elems = 2;
  } else if (kind == K_NUTS && dim > 256 && dim <= 1024 &&
             (target->kind == GM_TARGET_ROSENBROCK || target->kind == GM_TARGET_ISO_GAUSS)) {
    s->lay = nuts_wide_default((int)dim, dtype);
  }
  hipError_t e = hipGetDevice(&s->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&s->d_q, n_chains * dim * s->esz);
  if (e == hipSuccess) e = hipMalloc(&s->d_logp, n_chains * s->esz);
  if (e == hipSuccess) e = hipMalloc((void**)&s->d_acc, n_chains * sizeof(long long));
  if (e == hipSuccess) e = hipMemcpy(s->d_q, init, n_chains * dim * s->esz, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(s->d_acc, 0, n_chains * sizeof(long long));
  if (e != hipSuccess) {
    set_error(std::string("sampler setup failed: ") + hipGetErrorString(e));
    gm_destroy(s);
    return GM_EHIP;
  }
  *out = s;
  return GM_OK;
}

int gm_hmc_create(const gm_target* target, gm_dtype dtype, int64_t n_chains, int64_t dim,
                  const void* init, double step_size, int64_t n_leapfrog, int64_t chain_offset,
                  gm_sampler** out) {
  GM_REQ(n_leapfrog >= 0 && n_leapfrog < (1 << 30), "n_leapfrog out of range");
  GM_REQ(std::isfinite(step_size), "step_size must be finite");
  int rc = create_common(K_HMC, target, dtype, n_chains, dim, init, chain_offset, out);
  if (rc) return rc;
  (*out)->eps = step_size;
  (*out)->L = (int)n_leapfrog;
  return GM_OK;
}

int gm_mh_create(const gm_target* target, gm_dtype dtype, int64_t n_chains, int64_t dim,
                 const void* init, double proposal_std, int64_t chain_offset, gm_sampler** out) {
  GM_REQ(proposal_std > 0 && std::isfinite(proposal_std), "proposal_std must be > 0");
  int rc = create_common(K_MH, target, dtype, n_chains, dim, init, chain_offset, out);
  if (rc) return rc;
  (*out)->prop_std = proposal_std;
  return GM_OK;
}

int gm_nuts_create(const gm_target* target, gm_dtype dtype, int64_t n_chains, int64_t dim,
                   const void* init, double target_accept_p, int32_t max_depth,
                   int64_t chain_offset, gm_sampler** out) {
  GM_REQ(max_depth >= 0 && max_depth <= NUTS_MAX_DEPTH_LIMIT, "max_depth out of range");
  int rc = create_common(K_NUTS, target, dtype, n_chains, dim, init, chain_offset, out);
  if (rc) return rc;
  gm_sampler* s = *out;
  s->target_accept = target_accept_p;
  s->max_depth = max_depth == 0 ? NUTS_DEFAULT_MAX_DEPTH : max_depth;
  rc = nuts_init_state(&s->nuts, s->dt, s->C, s->D, s->max_depth);
  if (rc) {
    gm_destroy(s);
    *out = nullptr;
    return rc;
  }
  return GM_OK;
}

int gm_set_seed(gm_sampler* s, uint64_t seed) {
  GM_REQ(s, "sampler is NULL");
  s->seed = seed;
  s->step = 0;
  return GM_OK;
}

int gm_sampler_layout(gm_sampler* s, int32_t* lanes, int32_t* elems) {
  GM_REQ(s, "sampler is NULL");
  if (lanes) *lanes = s->lay.lanes;
  if (elems) *elems = s->lay.elems;
  return GM_OK;
}

int gm_sampler_set_layout(gm_sampler* s, int32_t lanes, int32_t elems) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(s->tg.kind != GM_TARGET_CUSTOM || (lanes == 1 && elems == s->D),
         "CUSTOM targets run one chain per lane (layout 1 x dim)");
  if (s->tg.kind == GM_TARGET_CUSTOM) return GM_OK;
  const bool wide = lanes > 64;
  if (wide && s->kind == K_NUTS) {  // one chain per workgroup (nuts_wide.hip)
    GM_REQ(nuts_wide_layout_supported(lanes, elems), "wide NUTS layout (lanes, elems) is not compiled in");
    GM_REQ(s->tg.kind == GM_TARGET_ROSENBROCK || s->tg.kind == GM_TARGET_ISO_GAUSS,
           "wide NUTS layouts take the Rosenbrock and isotropic Gaussian targets");
    GM_REQ(s->nuts.mass_mode != 2, "wide NUTS layouts take the identity or diagonal metric");
  } else {
    GM_REQ(wide ? wide_layout_supported(lanes, elems, s->dt) : layout_supported(lanes, elems),
           "layout (lanes, elems) is not compiled in");
    GM_REQ(!wide || s->kind == K_HMC, "wide layouts (lanes > 64) are for the HMC and NUTS samplers");
  }
  GM_REQ((long long)lanes * elems >= s->D, "lanes*elems must cover dim");
  GM_REQ((long long)lanes * elems < 2LL * s->D || lanes == 1 ||
             ((long long)(lanes / 2) * elems < s->D),
         "layout wastes more than half of its lanes");
  s->lay.lanes = lanes;
  s->lay.elems = elems;
  s->lay_from_wide = false;  // the caller's choice stands
  return GM_OK;
}

int gm_sampler_set_async(gm_sampler* s, int32_t on) {
  GM_REQ(s, "sampler is NULL");
  s->async_runs = on != 0;
  return GM_OK;
}

int gm_sampler_synchronize(gm_sampler* s) {
  GM_REQ(s, "sampler is NULL");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  return GM_OK;
}

int gm_sampler_set_steps_per_launch(gm_sampler* s, int64_t steps) {
  GM_REQ(s, "sampler is NULL");
  // the kernels take a launch's transition count as an int
  GM_REQ(steps >= 1 && steps <= INT32_MAX, "steps must be in [1, 2^31 - 1]");
  s->steps_per_launch = steps;
  return GM_OK;
}

int gm_sampler_set_unroll(gm_sampler* s, int32_t n) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(n == 0 || n == 1 || n == 2 || n == 4, "unroll must be 0 (automatic), 1, 2 or 4");
  s->lf_unroll = n;
  return GM_OK;
}

int gm_sampler_reserve(gm_sampler* s, int64_t n_collect) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(n_collect >= 0, "n_collect must be >= 0");
  GM_HIP(hipSetDevice(s->device));
  return ensure_buf(&s->d_samples, &s->samples_bytes, (size_t)n_collect * s->C * s->D * s->esz);
}

int gm_sampler_last_run_stats(gm_sampler* s, double* kernel_ms, int64_t* launches) {
  GM_REQ(s, "sampler is NULL");
  if (s->last_ms_pending) {  // the run's event pair, read only when asked for (off the run's path)
    float t = 0;
    GM_HIP(hipEventSynchronize(s->evs[1]));  // an asynchronous run may still be in flight
    GM_HIP(hipEventElapsedTime(&t, s->evs[0], s->evs[1]));
    s->last_ms = t;
    s->last_ms_pending = false;
  }
  if (kernel_ms) *kernel_ms = s->last_ms;
  if (launches) *launches = s->last_launches;
  return GM_OK;
}

// Leapfrog-loop unroll of the HMC kernel (identical results). Measured
// (tools/probe_hmc_scaling.py): x4 is ~12% faster while the grid has at most
// one wave per SIMD (latency bound), and 10-20% slower from two waves per
// SIMD up.
static int hmc_lf_unroll(long long waves) {
  static const int simds = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return 4 * cus;
  }();
  // x4 at <= 1 wave per SIMD, x2 at <= 4 (the cfg2 headline), x1 above
  // (cfg4's 8 and the north star's 16 waves per SIMD), measured per regime
  return waves <= simds ? 4 : waves <= 4 * simds ? 2 : 1;
}

// hipSetDevice only when the calling thread is on another device (the call
// is on every run's path). The current device is asked of the runtime
// (a thread-local read in HIP), never cached here: gm_set_device and the
// other entry points switch devices too.
static hipError_t use_device(int dev) {
  int cur = -1;
  const hipError_t g = hipGetDevice(&cur);
  if (g == hipSuccess && cur == dev) return hipSuccess;
  return hipSetDevice(dev);
}

// One event pair per run (before the first launch, after the last): the
// device time of the run's launches, read back after the run's stream
// synchronize.
static int ensure_run_events(gm_sampler* s) {
  while (s->evs.size() < 2) {
    hipEvent_t ev;
    GM_HIP(hipEventCreate(&ev));
    s->evs.push_back(ev);
  }
  return GM_OK;
}

// Runs `total` transitions; transitions with index >= collect_from (0-based
// within this call) are stored at sample rows (index - collect_from).
static int run_steps(gm_sampler* s, long long total, long long collect_from, int progress,
                     const TrackLaunch* trk = nullptr, const StepHook* hook = nullptr,
                     long long chunk_override = 0) {
  GM_HIP(use_device(s->device));
  s->last_ms = 0;
  s->last_launches = 0;
  s->last_ms_pending = false;
  // NUTS always launches: init_chain_state + row 0 even with zero transitions
  if (total <= 0 && s->kind != K_NUTS) return GM_OK;
  if (s->kind == K_NUTS) {
    int rc = nuts_run(s->nuts, s->dt, s->tg, s->lay, s->d_q, s->d_acc, s->d_samples, s->C, s->D,
                      s->target_accept, s->seed, &s->step, s->chain_offset, total, collect_from,
                      progress, chunk_override > 0 ? chunk_override : s->steps_per_launch,
                      s->stream, s->evs, &s->last_ms, &s->last_launches, trk, hook);
    return rc;
  }
  const long long chunk = chunk_override > 0 ? chunk_override : s->steps_per_launch;
  const long long n_launch = (total + chunk - 1) / chunk;
  int rc = ensure_run_events(s);
  if (rc) return rc;
  const int lf_unroll = s->kind != K_HMC ? 1 : s->lf_unroll ? s->lf_unroll
                                                             : hmc_lf_unroll((s->C * s->lay.lanes + 63) / 64);
  for (long long start = 0; start < total; start += chunk) {
    LaunchEvents ev;  // start with the first launch, stop with the last
    if (start == 0) ev.start = s->evs[0];
    if (start + chunk >= total) ev.stop = s->evs[1];
    const long long n = total - start < chunk ? total - start : chunk;
    long long cf = collect_from - start;
    if (cf < 0) cf = 0;
    if (cf > n) cf = n;
    long long row0 = start - collect_from;
    if (row0 < 0) row0 = 0;
    hipError_t e;
    if (s->kind == K_HMC) {
      HmcLaunch a;
      a.q = s->d_q;
      a.logp = s->d_logp;
      a.accepts = s->d_acc;
      a.samples = s->d_samples;
      a.C = s->C;
      a.D = s->D;
      a.eps = s->eps;
      a.L = s->L;
      a.seed = s->seed;
      a.step0 = s->step + start;
      a.chain_offset = s->chain_offset;
      a.n_steps = (int)n;
      a.collect_from = (int)cf;
      a.sample_row0 = row0;
      a.lf_unroll = lf_unroll;
      if (layout_is_wide(s->lay)) {
        const size_t need = (size_t)s->C * (s->dt == GM_F32 ? 4 : 2) * s->lay.lanes * s->lay.elems * s->esz;
        rc = ensure_buf(&s->d_zs, &s->zs_bytes, need);
        if (rc) return rc;
        a.zs = s->d_zs;
      }
      e = launch_hmc(s->dt, s->tg, s->lay, a, s->stream, ev);
    } else {
      MhLaunch a;
      a.q = s->d_q;
      a.logp = s->d_logp;
      a.accepts = s->d_acc;
      a.samples = s->d_samples;
      a.C = s->C;
      a.D = s->D;
      a.prop_std = s->prop_std;
      a.seed = s->seed;
      a.step0 = s->step + start;
      a.chain_offset = s->chain_offset;
      a.n_steps = (int)n;
      a.collect_from = (int)cf;
      a.sample_row0 = row0;
      if (trk) {
        a.trk = *trk;
        a.trk.n0 = trk->n0 + (unsigned long long)start;
      }
      e = launch_mh(s->dt, s->tg, s->lay, a, s->stream, ev);
    }
    if (e != hipSuccess) {
      set_error(std::string("kernel launch failed: ") + hipGetErrorString(e));
      return GM_EHIP;
    }
    if (hook && *hook) {
      rc = (*hook)(start + n);
      if (rc) return rc;
    }
  }
  s->step += total;
  s->total_steps += total;
  if (!(s->async_runs && s->may_async)) GM_HIP(hipStreamSynchronize(s->stream));
  s->last_ms_pending = true;
  s->last_launches = n_launch;
  return GM_OK;
}

static int run_impl(gm_sampler* s, int64_t n_collect, int64_t n_discard, int progress) {
  GM_REQ(s, "sampler is NULL");
  s->last_rows = n_collect;
  GM_REQ(n_collect >= 0 && n_discard >= 0, "n_collect and n_discard must be >= 0");
  GM_HIP(use_device(s->device));
  int rc = ensure_buf(&s->d_samples, &s->samples_bytes, (size_t)n_collect * s->C * s->D * s->esz);
  if (rc) return rc;
  long long total = n_discard + n_collect;
  if (s->kind == K_NUTS && !progress) {
    // NUTS::run performs n_collect + n_discard - 1 transitions (nuts.rs:232-257);
    // row r is the state after n_discard + r of them.
    if (n_collect == 0) return GM_OK;
    total = n_discard + n_collect - 1;
    return run_steps(s, total, n_discard, progress ? 1 : 0);
  }
  return run_steps(s, total, n_discard, progress ? 1 : 0);
}

int gm_run_device(gm_sampler* s, int64_t n_collect, int64_t n_discard, const void** dev_samples) {
  RoctxRange rr("gm_run_device");
  GM_REQ(s, "sampler is NULL");
  s->may_async = true;  // the samples stay on the device: the caller may wait later
  int rc = run_impl(s, n_collect, n_discard, 0);
  s->may_async = false;
  if (rc) return rc;
  if (dev_samples) *dev_samples = s->d_samples;
  return GM_OK;
}

int gm_run_device_progress(gm_sampler* s, int64_t n_collect, int64_t n_discard,
                           const void** dev_samples) {
  int rc = run_impl(s, n_collect, n_discard, 1);
  if (rc) return rc;
  if (dev_samples) *dev_samples = s->d_samples;
  return GM_OK;
}

// Device -> caller's (pageable) host memory through two pinned staging slots:
// the DMA of chunk i runs while host threads copy chunk i-1 out of the other
// slot. The threads also take the first-touch page faults of a fresh output
// array in parallel, which a single-threaded pageable hipMemcpy serialises.
static constexpr size_t kStageChunk = (size_t)16 << 20;

static int host_copy_threads() {
  const char* e = std::getenv("OMP_NUM_THREADS");
  int n = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
  return n < 1 ? 1 : (n > 16 ? 16 : n);
}

static void parallel_memcpy(char* dst, const char* src, size_t n, int threads) {
  const size_t min_part = (size_t)1 << 20;
  int t = (int)std::min<size_t>((size_t)threads, (n + min_part - 1) / min_part);
  if (t <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> pool;
  const size_t part = (n + t - 1) / t;
  for (int i = 1; i < t; ++i) {
    const size_t o = (size_t)i * part;
    if (o >= n) break;
    pool.emplace_back([=] { std::memcpy(dst + o, src + o, std::min(part, n - o)); });
  }
  std::memcpy(dst, src, std::min(part, n));
  for (auto& th : pool) th.join();
}

static int stage_to_host(gm_sampler* s, void* out, const void* dsrc, size_t bytes) {
  if (bytes == 0) return GM_OK;
  if (!s->h_stage[0]) {
    for (int k = 0; k < 2; ++k) {
      GM_HIP(hipHostMalloc(&s->h_stage[k], kStageChunk, hipHostMallocDefault));
      GM_HIP(hipEventCreateWithFlags(&s->stage_ev[k], hipEventDisableTiming));
    }
  }
  const int threads = host_copy_threads();
  const size_t n_chunks = (bytes + kStageChunk - 1) / kStageChunk;
  for (size_t i = 0; i <= n_chunks; ++i) {
    if (i < n_chunks) {  // DMA of chunk i into slot i % 2
      const size_t o = i * kStageChunk, n = std::min(kStageChunk, bytes - o);
      GM_HIP(hipMemcpyAsync(s->h_stage[i & 1], (const char*)dsrc + o, n, hipMemcpyDeviceToHost, s->stream));
      GM_HIP(hipEventRecord(s->stage_ev[i & 1], s->stream));
    }
    if (i >= 1) {  // host copy of chunk i-1 while chunk i is in flight
      const size_t j = i - 1, o = j * kStageChunk, n = std::min(kStageChunk, bytes - o);
      GM_HIP(hipEventSynchronize(s->stage_ev[j & 1]));
      parallel_memcpy((char*)out + o, (const char*)s->h_stage[j & 1], n, threads);
    }
  }
  return GM_OK;
}

static int copy_samples_impl(gm_sampler* s, void* out) {
  GM_HIP(hipSetDevice(s->device));
  const long long n_collect = s->last_rows;
  if (n_collect == 0) return GM_OK;
  const size_t bytes = (size_t)n_collect * s->C * s->D * s->esz;
  int rc = ensure_buf(&s->d_tmp, &s->tmp_bytes, bytes);
  if (rc) return rc;
  hipError_t e = launch_transpose_samples(s->dt, s->d_samples, s->d_tmp, n_collect, s->C, s->D,
                                          s->stream);
  if (e != hipSuccess) {
    set_error(std::string("transpose failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  return stage_to_host(s, out, s->d_tmp, bytes);
}

int gm_copy_samples(gm_sampler* s, int64_t n_rows, void* out) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(n_rows == s->last_rows,
         "n_rows does not match the last run's n_collect (" + std::to_string(s->last_rows) + ")");
  if (n_rows == 0) return GM_OK;
  GM_REQ(out != nullptr, "out is NULL");
  return copy_samples_impl(s, out);
}

int gm_copy_sample_block(gm_sampler* s, int64_t row0, int64_t n_rows, int64_t chain0, int64_t n_chains,
                         void* out) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(row0 >= 0 && n_rows >= 0 && row0 + n_rows <= s->last_rows, "rows out of range of the last run");
  GM_REQ(chain0 >= 0 && n_chains >= 0 && chain0 + n_chains <= s->C, "chains out of range");
  if (n_rows == 0 || n_chains == 0) return GM_OK;
  GM_REQ(out != nullptr, "out is NULL");
  GM_HIP(hipSetDevice(s->device));
  const size_t row_bytes = (size_t)s->C * s->D * s->esz, w = (size_t)n_chains * s->D * s->esz;
  const char* src = (const char*)s->d_samples + (size_t)row0 * row_bytes + (size_t)chain0 * s->D * s->esz;
  GM_HIP(hipMemcpy2DAsync(out, w, src, row_bytes, w, (size_t)n_rows, hipMemcpyDeviceToHost, s->stream));
  GM_HIP(hipStreamSynchronize(s->stream));
  return GM_OK;
}

int gm_run(gm_sampler* s, int64_t n_collect, int64_t n_discard, void* out) {
  RoctxRange rr("gm_run");
  int rc = run_impl(s, n_collect, n_discard, 0);
  if (rc) return rc;
  if (!out || n_collect == 0) return GM_OK;
  return copy_samples_impl(s, out);
}

static float max_skipnan(const float* v, long long n) {  // stats.rs:154-161
  float m = NAN;
  bool any = false;
  for (long long i = 0; i < n; ++i)
    if (!std::isnan(v[i])) {
      m = any ? std::fmax(m, v[i]) : v[i];
      any = true;
    }
  return m;
}

int gm_run_progress_cb(gm_sampler* s, int64_t n_collect, int64_t n_discard, void* out,
                       float* rhat_out, float* ess_out, gm_progress_fn cb, void* user,
                       double interval_s) {
  RoctxRange rr("gm_run_progress");
  GM_REQ(s, "sampler is NULL");
  GM_REQ(n_collect >= 0 && n_discard >= 0, "n_collect and n_discard must be >= 0");
  GM_HIP(hipSetDevice(s->device));
  s->last_rows = n_collect;
  int rc = ensure_buf(&s->d_samples, &s->samples_bytes, (size_t)n_collect * s->C * s->D * s->esz);
  if (rc) return rc;
  const long long C = s->C, total = n_collect + n_discard;
  const int D = s->D;
  using clk = std::chrono::steady_clock;
  auto t_last = clk::now();
  auto due = [&](bool last) {
    return last || std::chrono::duration<double>(clk::now() - t_last).count() >= interval_s;
  };
  // with a callback, launches are cut so that it can fire between them
  long long chunk = 0;
  if (cb) {
    chunk = total / 32 > 0 ? total / 32 : 1;
    if (chunk > s->steps_per_launch) chunk = s->steps_per_launch;
  }
  std::vector<float> rh(D);
  gm_progress info{};
  if (s->kind == K_HMC) {
    // burn-in, then the collection with a MultiChainTracker stepped on the
    // current positions at each sync point (hmc.rs:252-290)
    if (n_discard > 0) {
      rc = run_steps(s, n_discard, n_discard, 1);
      if (rc) return rc;
    }
    StepHook hook;
    unsigned long long mct_n = 0;
    if (cb) {
      rc = ensure_buf(&s->d_mct, &s->mct_bytes, TrackSet::bytes(C, D));
      if (rc) return rc;
      GM_HIP(hipMemsetAsync(s->d_mct, 0, TrackSet::bytes(C, D), s->stream));  // new(): zeros, p 0
      hook = [&](long long done) -> int {
        const bool last = done >= n_collect;
        if (!due(last)) return GM_OK;
        TrackSet ts(s->d_mct, C, D);
        ++mct_n;
        GM_HIP(launch_mct_step(s->dt, C, D, s->d_q, ts.mean, ts.msq, ts.last, ts.flags, ts.p, mct_n,
                               s->stream));
        GM_HIP(launch_mct_rhat(C, D, mct_n, ts.mean, ts.msq, ts.rhat, s->stream));
        float p = 0;
        GM_HIP(hipMemcpyAsync(rh.data(), ts.rhat, sizeof(float) * D, hipMemcpyDeviceToHost, s->stream));
        GM_HIP(hipMemcpyAsync(&p, ts.p, sizeof(float), hipMemcpyDeviceToHost, s->stream));
        GM_HIP(hipStreamSynchronize(s->stream));
        info.done = done;
        info.total = n_collect;
        info.p_accept = p;
        info.max_rhat = max_skipnan(rh.data(), D);
        cb(user, &info);
        t_last = clk::now();
        return GM_OK;
      };
    }
    rc = run_steps(s, n_collect, 0, 1, nullptr, cb ? &hook : nullptr, chunk);
    if (rc) return rc;
  } else {
    // MH (core.rs:132-176) and NUTS (generic_nuts.rs:675-716): every chain's
    // ChainTracker steps after every transition, burn-in included
    rc = ensure_buf(&s->d_trk, &s->trk_bytes, TrackSet::bytes(C, D));
    if (rc) return rc;
    TrackSet ts(s->d_trk, C, D);
    TrackLaunch tl = ts.launch();
    GM_HIP(launch_ct_init(s->dt, C, D, s->d_q, tl, s->stream));
    s->trk_n = 0;
    StepHook hook = [&](long long done) -> int {
      const bool last = done >= total;
      if (!due(last)) return GM_OK;
      float pm = 0;
      GM_HIP(launch_ct_rhat(C, D, (unsigned long long)done, tl, ts.rhat, ts.scalar, s->stream));
      GM_HIP(hipMemcpyAsync(rh.data(), ts.rhat, sizeof(float) * D, hipMemcpyDeviceToHost, s->stream));
      GM_HIP(hipMemcpyAsync(&pm, ts.scalar, sizeof(float), hipMemcpyDeviceToHost, s->stream));
      GM_HIP(hipStreamSynchronize(s->stream));
      info.done = done;
      info.total = total;
      info.p_accept = pm;
      info.max_rhat = C >= 2 ? max_skipnan(rh.data(), D) : NAN;  // core.rs:321 (>= 2 chains)
      cb(user, &info);
      t_last = clk::now();
      return GM_OK;
    };
    rc = run_steps(s, total, n_discard, 1, &tl, cb ? &hook : nullptr, chunk);
    if (rc) return rc;
    s->trk_n = (unsigned long long)total;
  }
  if (out && n_collect > 0) {
    rc = copy_samples_impl(s, out);
    if (rc) return rc;
  }
  if (rhat_out || ess_out) {
    GM_REQ(n_collect >= 2, "run_progress statistics need n_collect >= 2");
    std::vector<float> r(s->D), e(s->D);
    rc = gm_split_rhat_ess_device(s->d_samples, s->dt, s->C, n_collect, s->D, s->D,
                                  s->C * s->D, 1, r.data(), e.data());
    if (rc) return rc;
    if (rhat_out) memcpy(rhat_out, r.data(), sizeof(float) * s->D);
    if (ess_out) memcpy(ess_out, e.data(), sizeof(float) * s->D);
  }
  return GM_OK;
}

int gm_run_progress(gm_sampler* s, int64_t n_collect, int64_t n_discard, void* out,
                    float* rhat_out, float* ess_out) {
  return gm_run_progress_cb(s, n_collect, n_discard, out, rhat_out, ess_out, nullptr, nullptr, 0.0);
}

int gm_sampler_chain_stats(gm_sampler* s, uint64_t* n, float* p_accept, float* mean, float* sm2) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(s->kind != K_HMC, "chain trackers are kept by the MH and NUTS run_progress");
  GM_REQ(s->d_trk != nullptr, "no run_progress has been run");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  const long long C = s->C;
  const int D = s->D;
  TrackSet ts(s->d_trk, C, D);
  if (n) *n = s->trk_n;
  if (p_accept) GM_HIP(hipMemcpy(p_accept, ts.p, sizeof(float) * C, hipMemcpyDeviceToHost));
  if (mean || sm2) {
    std::vector<float> m((size_t)C * D), q((size_t)C * D);
    GM_HIP(hipMemcpy(m.data(), ts.mean, sizeof(float) * C * D, hipMemcpyDeviceToHost));
    GM_HIP(hipMemcpy(q.data(), ts.msq, sizeof(float) * C * D, hipMemcpyDeviceToHost));
    if (mean) memcpy(mean, m.data(), sizeof(float) * C * D);
    if (sm2) {  // ChainTracker::stats (stats.rs:122-131)
      const float nf = (float)s->trk_n;
      for (long long i = 0; i < C * D; ++i) sm2[i] = (q[i] - m[i] * m[i]) * nf / (nf - 1.0f);
    }
  }
  return GM_OK;
}

// HMC::step (hmc.rs:316-330), ChainRunner's step (core.rs:81), NUTS::step
// (nuts.rs:431-433 -> generic_nuts.rs:755-925): one transition of every chain,
// nothing collected. A NUTS step continues the adaptation counter of the last
// run (dual averaging only while m <= that run's n_discard, which a step past a
// completed run never is; then eps = eps_bar) and does not re-run
// init_chain_state, exactly as the reference's step() does.
int gm_step(gm_sampler* s) {
  RoctxRange rr("gm_step");
  GM_REQ(s, "sampler is NULL");
  s->may_async = true;
  const int rc = run_steps(s, 1, 1, s->kind == K_NUTS ? 2 : 0);
  s->may_async = false;
  return rc;
}

int gm_get_positions(gm_sampler* s, void* out) {
  GM_REQ(s && out, "bad arguments");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  GM_HIP(hipMemcpy(out, s->d_q, s->C * s->D * s->esz, hipMemcpyDeviceToHost));
  return GM_OK;
}

int gm_set_positions(gm_sampler* s, const void* in) {
  GM_REQ(s && in, "bad arguments");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  GM_HIP(hipMemcpy(s->d_q, in, s->C * s->D * s->esz, hipMemcpyHostToDevice));
  return GM_OK;
}

int gm_get_accept_counts(gm_sampler* s, int64_t* out) {
  GM_REQ(s && out, "bad arguments");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  GM_HIP(hipMemcpy(out, s->d_acc, s->C * sizeof(long long), hipMemcpyDeviceToHost));
  return GM_OK;
}

int gm_get_leapfrog_counts(gm_sampler* s, int64_t* out) {
  GM_REQ(s && out, "bad arguments");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  if (s->kind == K_NUTS) return nuts_get_leapfrogs(s->nuts, s->C, (long long*)out);
  for (long long i = 0; i < s->C; ++i) out[i] = s->kind == K_HMC ? (int64_t)s->total_steps * s->L : 0;
  return GM_OK;
}

int gm_nuts_get_step_size(gm_sampler* s, double* eps, double* eps_bar) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(s->kind == K_NUTS, "not a NUTS sampler");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  return nuts_get_step_size(s->nuts, s->dt, s->C, eps, eps_bar);
}

int gm_nuts_set_mass_adaptation(gm_sampler* s, int32_t mode, int64_t start_buffer, int64_t end_buffer,
                                int64_t initial_window, double regularize, double jitter,
                                int64_t dense_max_dim) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(s->kind == K_NUTS, "not a NUTS sampler");
  GM_REQ(mode >= 0 && mode <= 2, "mode must be 0 (none), 1 (diagonal) or 2 (dense)");
  GM_REQ(start_buffer >= 0 && end_buffer >= 0 && initial_window >= 0, "window sizes must be >= 0");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  // dense only up to dense_max_dim, else diagonal (generic_nuts.rs:613-620)
  if (mode == 2 && s->D > dense_max_dim) mode = 1;
  const int rc = nuts_set_mass(&s->nuts, s->dt, s->C, s->D, mode, start_buffer, end_buffer, initial_window,
                               regularize, jitter);
  if (rc != GM_OK) return rc;  // (the layout is left as it was)
  if (mode == 2 && layout_is_wide(s->lay)) {
    // a dense metric's products broadcast within one wave: off the wide
    // layouts, remembered so that a later identity / diagonal mode gets the
    // wide layout back (the one-wave layouts spill at D > 256)
    s->lay_wide = s->lay;
    s->lay = default_layout(s->D, s->dt, s->tg.kind);
    s->lay_from_wide = true;
  } else if (mode != 2 && s->lay_from_wide) {
    s->lay = s->lay_wide;
    s->lay_from_wide = false;
  }
  return GM_OK;
}

int gm_nuts_set_momentum_pass(gm_sampler* s, int32_t on) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(s->kind == K_NUTS, "not a NUTS sampler");
  s->nuts.momentum_pass = on != 0;
  if (!s->nuts.momentum_pass && s->nuts.zbuf) {  // the pass's buffer is released with it
    GM_HIP(hipSetDevice(s->device));
    GM_HIP(hipStreamSynchronize(s->stream));
    GM_HIP(hipFree(s->nuts.zbuf));
    s->nuts.zbuf = nullptr;
    s->nuts.zbuf_bytes = 0;
  }
  return GM_OK;
}

int gm_nuts_set_lds_levels(gm_sampler* s, int32_t levels) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(s->kind == K_NUTS, "not a NUTS sampler");
  GM_REQ(levels >= -1 && levels <= NUTS_MAX_DEPTH_LIMIT, "levels must be -1 (automatic) or 0..30");
  s->nuts.lds_levels_cap = levels;
  return GM_OK;
}

int gm_nuts_set_dense_forms(gm_sampler* s, int32_t minv_lds, int32_t chol_lds) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(s->kind == K_NUTS, "not a NUTS sampler");
  GM_REQ(minv_lds >= -1 && minv_lds <= 2, "minv_lds must be -1 (automatic), 0, 1 or 2");
  GM_REQ(chol_lds >= -1 && chol_lds <= 1, "chol_lds must be -1 (automatic), 0 or 1");
  // automatic: the packed M^-1 in LDS and L in global memory, which leaves
  // 6 subtree-stack levels on chip (HBM 3.2 GB per cfg3 sampling launch
  // instead of 34.7 GB with the full matrices, 1.8 % slower:
  // profiles/r04/dense_forms_carried.jsonl, dense_traffic.json)
  s->nuts.dense_minv_lds = minv_lds < 0 ? 1 : minv_lds;
  s->nuts.dense_chol_lds = chol_lds < 0 ? 0 : chol_lds;
  return GM_OK;
}

int gm_nuts_get_plan(gm_sampler* s, int32_t* plan, int32_t cap) {
  GM_REQ(s && plan, "NULL argument");
  GM_REQ(s->kind == K_NUTS, "not a NUTS sampler");
  GM_REQ(cap >= 1, "cap must be >= 1 (the values plan can hold)");
  for (int i = 0; i < 6 && i < cap; ++i) plan[i] = s->nuts.plan[i];
  return GM_OK;
}

int gm_nuts_get_mass(gm_sampler* s, int32_t* mode, int32_t* kind, void* dinv, void* dsqrt, void* minv,
                     void* mchol) {
  GM_REQ(s, "sampler is NULL");
  GM_REQ(s->kind == K_NUTS, "not a NUTS sampler");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  if (mode) *mode = s->nuts.mass_mode;
  return nuts_get_mass(s->nuts, s->dt, s->C, s->D, kind, dinv, dsqrt, minv, mchol);
}

// ---- checkpoint / resume ----------------------------------------------------
// The reference keeps a sampler's state only inside the object across run
// calls (positions, batched_hmc.rs:40; NUTS epsilon / epsilon_bar / h_bar,
// generic_nuts.rs:573-582, 744; the metric and the warm-up window schedule);
// core.rs:177 leaves checkpointing as a TODO. The blob holds exactly that
// state plus the Philox stream position, so a restored sampler continues bit
// for bit (runs start at init_chain_state, so NUTS needs no mid-trajectory
// state; HMC and MH re-evaluate logp at every launch start).
}  // extern "C"

namespace {
// v2 header: the sampler's configuration too, so that a blob is only loaded
// into a sampler that would continue it with the same semantics
struct StateHeader {
  char magic[8];  // "GMCMCST2"
  int32_t kind, dtype;
  int64_t C, D;
  uint64_t seed, step;
  int64_t total_steps;
  uint32_t chain_offset;
  int32_t mass_mode;
  int64_t m_sb, m_eb, sched_next, sched_len;
  double m_reg, m_jit;
  // configuration (checked on load): HMC eps / L, MH proposal std, NUTS
  // target accept / max depth, and the NUTS run position (m, n_discard)
  double eps, prop_std, target_accept;
  int32_t L, max_depth;
  int64_t nuts_m, nuts_n_discard;
};
struct StatePart {
  void* dev;
  size_t bytes;
};
// the blob's parts for a sampler of this kind / shape / metric mode; sizes
// only depend on the header fields, so a blob can be validated before any
// state is touched
std::vector<StatePart> state_parts_for(gm_sampler* s, int mass_mode) {
  const size_t C = (size_t)s->C, D = (size_t)s->D, e = s->esz;
  std::vector<StatePart> v{{s->d_q, C * D * e}, {s->d_acc, C * sizeof(long long)}};
  if (s->kind == K_NUTS) {
    NutsState& n = s->nuts;
    v.push_back({n.eps, C * e});
    v.push_back({n.eps_bar, C * e});
    v.push_back({n.h_bar, C * e});
    v.push_back({n.mu, C * e});
    v.push_back({n.n_leapfrog, C * sizeof(long long)});
    if (mass_mode) {
      v.push_back({n.mkind, C * sizeof(int)});
      v.push_back({n.dinv, C * D * e});
      v.push_back({n.dsq, C * D * e});
    }
    if (mass_mode == 2) {
      v.push_back({n.minv, C * D * D * e});
      v.push_back({n.mchol, C * D * D * e});
    }
  }
  return v;
}
size_t parts_bytes(const std::vector<StatePart>& v) {
  size_t b = sizeof(StateHeader);
  for (auto& p : v) b += p.bytes;
  return b;
}
size_t state_bytes(gm_sampler* s) { return parts_bytes(state_parts_for(s, s->kind == K_NUTS ? s->nuts.mass_mode : 0)); }
}  // namespace

extern "C" {

#ifdef GM_HOST_TEST
// Host-only test hooks, compiled into the AddressSanitizer build of the host
// code only (tools/asan, tests/test_asan_host.py): a sampler shell with no
// device memory, and a well-formed state header for it, so that blob parsing
// and argument validation run under ASan on a machine without a GPU.
gm_sampler* gm_test_sampler(int kind, int dtype, long long C, int D, int mass_mode) {
  gm_sampler* s = new gm_sampler();
  s->kind = kind;
  s->dt = (gm_dtype)dtype;
  s->esz = dtype == GM_F32 ? 4 : 8;
  s->C = C;
  s->D = D;
  s->eps = 0.01;
  s->L = 5;
  s->nuts.mass_mode = kind == K_NUTS ? mass_mode : 0;
  return s;
}
void gm_test_sampler_free(gm_sampler* s) { delete s; }
uint64_t gm_test_state_header(gm_sampler* s, void* out) {
  StateHeader h;
  memset(&h, 0, sizeof(h));
  memcpy(h.magic, "GMCMCST2", 8);
  h.kind = s->kind;
  h.dtype = s->dt;
  h.C = s->C;
  h.D = s->D;
  h.eps = s->eps;
  h.L = s->L;
  h.prop_std = s->prop_std;
  h.target_accept = s->target_accept;
  h.max_depth = s->max_depth;
  h.mass_mode = s->kind == K_NUTS ? s->nuts.mass_mode : 0;
  memcpy(out, &h, sizeof(h));
  return sizeof(h);
}
#endif

int gm_state_size(gm_sampler* s, uint64_t* bytes) {
  GM_REQ(s && bytes, "bad arguments");
  *bytes = state_bytes(s);
  return GM_OK;
}

int gm_state_save(gm_sampler* s, void* out, uint64_t bytes) {
  GM_REQ(s && out, "bad arguments");
  GM_REQ(bytes >= state_bytes(s), "buffer smaller than gm_state_size");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  StateHeader h;
  memset(&h, 0, sizeof(h));
  memcpy(h.magic, "GMCMCST2", 8);
  h.kind = s->kind;
  h.dtype = s->dt;
  h.C = s->C;
  h.D = s->D;
  h.seed = s->seed;
  h.step = s->step;
  h.total_steps = s->total_steps;
  h.chain_offset = s->chain_offset;
  h.eps = s->eps;
  h.L = s->L;
  h.prop_std = s->prop_std;
  h.target_accept = s->target_accept;
  h.max_depth = s->max_depth;
  if (s->kind == K_NUTS) {
    const NutsState& n = s->nuts;
    h.mass_mode = n.mass_mode;
    h.m_sb = n.m_sb;
    h.m_eb = n.m_eb;
    h.sched_next = n.sched_next;
    h.sched_len = n.sched_len;
    h.m_reg = n.m_reg;
    h.m_jit = n.m_jit;
    h.nuts_m = n.m;
    h.nuts_n_discard = n.n_discard;
  }
  unsigned char* o = (unsigned char*)out;
  memcpy(o, &h, sizeof(h));
  o += sizeof(h);
  for (auto& p : state_parts_for(s, h.mass_mode)) {
    GM_HIP(hipMemcpy(o, p.dev, p.bytes, hipMemcpyDeviceToHost));
    o += p.bytes;
  }
  return GM_OK;
}

// Every check happens before the sampler is changed: a truncated, corrupt or
// foreign blob returns GM_EINVAL and leaves the sampler as it was.
int gm_state_load(gm_sampler* s, const void* in, uint64_t bytes) {
  GM_REQ(s && in, "bad arguments");
  GM_REQ(bytes >= sizeof(StateHeader), "state blob too short");
  StateHeader h;
  memcpy(&h, in, sizeof(h));
  GM_REQ(memcmp(h.magic, "GMCMCST2", 8) == 0, "not a libgmcmc state blob (v2)");
  GM_REQ(h.kind == s->kind && h.dtype == (int32_t)s->dt && h.C == s->C && h.D == s->D &&
             h.chain_offset == s->chain_offset,
         "state blob is for a different sampler kind, dtype, shape or chain offset");
  switch (s->kind) {
    case K_HMC:
      GM_REQ(h.eps == s->eps && h.L == s->L, "state blob is for a different step size / n_leapfrog");
      break;
    case K_MH:
      GM_REQ(h.prop_std == s->prop_std, "state blob is for a different proposal std");
      break;
    case K_NUTS:
      GM_REQ(h.target_accept == s->target_accept && h.max_depth == s->max_depth,
             "state blob is for a different target_accept_p / max_depth");
      GM_REQ(h.mass_mode >= 0 && h.mass_mode <= 2, "corrupt state blob (mass mode)");
      GM_REQ(h.nuts_m >= 0 && h.nuts_n_discard >= 0 && h.sched_len >= 0, "corrupt state blob (counters)");
      break;
  }
  if (s->kind != K_NUTS) GM_REQ(h.mass_mode == 0, "corrupt state blob (mass mode)");
  GM_REQ(bytes >= parts_bytes(state_parts_for(s, h.mass_mode)), "state blob too short");
  GM_HIP(hipSetDevice(s->device));
  GM_HIP(hipStreamSynchronize(s->stream));
  if (s->kind == K_NUTS && (h.mass_mode != s->nuts.mass_mode || h.mass_mode)) {
    const int rc = nuts_set_mass(&s->nuts, s->dt, s->C, s->D, h.mass_mode, h.m_sb, h.m_eb, 0,
                                 h.m_reg, h.m_jit);
    if (rc) return rc;
  }
  const unsigned char* p = (const unsigned char*)in + sizeof(h);
  for (auto& part : state_parts_for(s, h.mass_mode)) {
    GM_HIP(hipMemcpy(part.dev, p, part.bytes, hipMemcpyHostToDevice));
    p += part.bytes;
  }
  s->seed = h.seed;
  s->step = h.step;
  s->total_steps = h.total_steps;
  if (s->kind == K_NUTS) {
    s->nuts.sched_next = h.sched_next;
    s->nuts.sched_len = h.sched_len;
    s->nuts.m = h.nuts_m;
    s->nuts.n_discard = h.nuts_n_discard;
  }
  return GM_OK;
}

struct gm_mct {
  long long C = 0;
  int P = 0;
  int device = 0;
  unsigned long long n = 0;
  void* buf = nullptr;
};

int gm_mct_create(int64_t n_chains, int64_t n_params, gm_mct** out) {
  GM_REQ(out, "out is NULL");
  *out = nullptr;
  GM_REQ(n_chains >= 1 && n_params >= 1 && n_params <= (1 << 30), "bad tracker shape");
  gm_mct* t = new gm_mct();
  t->C = n_chains;
  t->P = (int)n_params;
  hipGetDevice(&t->device);
  size_t cap = 0;
  int rc = ensure_buf(&t->buf, &cap, TrackSet::bytes(t->C, t->P));
  if (rc) {
    delete t;
    return rc;
  }
  GM_HIP(hipMemset(t->buf, 0, TrackSet::bytes(t->C, t->P)));
  *out = t;
  return GM_OK;
}

int gm_mct_step(gm_mct* t, const void* x, gm_dtype dt) {
  GM_REQ(t && x, "bad arguments");
  GM_REQ(dt == GM_F32 || dt == GM_F64, "bad dtype");
  GM_HIP(hipSetDevice(t->device));
  TrackSet ts(t->buf, t->C, t->P);
  ++t->n;
  GM_HIP(launch_mct_step(dt, t->C, t->P, x, ts.mean, ts.msq, ts.last, ts.flags, ts.p, t->n, nullptr));
  return GM_OK;
}

int gm_mct_stats(gm_mct* t, float* p_accept, float* rhat, float* max_rhat) {
  GM_REQ(t, "tracker is NULL");
  GM_HIP(hipSetDevice(t->device));
  TrackSet ts(t->buf, t->C, t->P);
  if (p_accept) GM_HIP(hipMemcpy(p_accept, ts.p, sizeof(float), hipMemcpyDeviceToHost));
  if (rhat || max_rhat) {
    GM_HIP(launch_mct_rhat(t->C, t->P, t->n, ts.mean, ts.msq, ts.rhat, nullptr));
    std::vector<float> r(t->P);
    GM_HIP(hipMemcpy(r.data(), ts.rhat, sizeof(float) * t->P, hipMemcpyDeviceToHost));
    if (rhat) memcpy(rhat, r.data(), sizeof(float) * t->P);
    if (max_rhat) {  // MultiChainTracker::max_rhat: reduce(f32::max) (stats.rs:298-305)
      float m = r[0];
      for (int i = 1; i < t->P; ++i) m = std::fmax(m, r[i]);
      *max_rhat = m;
    }
  }
  return GM_OK;
}

int gm_mct_destroy(gm_mct* t) {
  if (!t) return GM_OK;
  hipSetDevice(t->device);
  hipDeviceSynchronize();
  if (t->buf) hipFree(t->buf);
  delete t;
  return GM_OK;
}

int gm_destroy(gm_sampler* s) {
  if (!s) return GM_OK;
  hipSetDevice(s->device);
  if (s->stream) hipStreamSynchronize(s->stream);
  for (auto ev : s->evs) hipEventDestroy(ev);
  if (s->d_mu) hipFree(s->d_mu);
  if (s->d_prec) hipFree(s->d_prec);
  if (s->d_zs) hipFree(s->d_zs);
  if (s->d_q) hipFree(s->d_q);
  if (s->d_logp) hipFree(s->d_logp);
  if (s->d_acc) hipFree(s->d_acc);
  if (s->d_samples) hipFree(s->d_samples);
  if (s->d_tmp) hipFree(s->d_tmp);
  for (int k = 0; k < 2; ++k) {
    if (s->h_stage[k]) hipHostFree(s->h_stage[k]);
    if (s->stage_ev[k]) hipEventDestroy(s->stage_ev[k]);
  }
  if (s->d_trk) hipFree(s->d_trk);
  if (s->d_mct) hipFree(s->d_mct);
  nuts_free_state(&s->nuts);
  if (s->stream) hipStreamDestroy(s->stream);
  delete s;
  return GM_OK;
}

}  // extern "C"
