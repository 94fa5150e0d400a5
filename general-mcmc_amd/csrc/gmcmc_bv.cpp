// gmcmc_bv.cpp — C ABI of the granular BatchVector ops (tier 2 of the
// boundary, include/gmcmc.h): argument checks, then one kernel launch each
// (bv_kernels.hip) on the null stream.
#include <map>
#include <hip/hip_runtime.h>

#include <string>

#include "gm_internal.h"
#include "gm_rng.h"

using namespace gm;

#define BV_REQ(cond, msg)  \
  do {                     \
    if (!(cond)) {         \
      set_error(msg);      \
      return GM_EINVAL;    \
    }                      \
  } while (0)

static int bv_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return GM_OK;
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  return GM_EHIP;
}
static bool dtype_ok(gm_dtype dt) { return dt == GM_F32 || dt == GM_F64; }

struct gm_bv_target {
  gm_dtype dt = GM_F32;
  TargetDev tg;
  void* d_mu = nullptr;
  void* d_prec = nullptr;
};

extern "C" {

int gm_malloc(void** dev_ptr, size_t bytes) {
  BV_REQ(dev_ptr != nullptr, "dev_ptr is NULL");
  *dev_ptr = nullptr;
  if (bytes == 0) return GM_OK;
  if (hipMalloc(dev_ptr, bytes) != hipSuccess) {
    *dev_ptr = nullptr;
    set_error("device allocation failed");
    return GM_ENOMEM;
  }
  return GM_OK;
}
int gm_free(void* dev_ptr) { return bv_status(hipFree(dev_ptr), "hipFree"); }
int gm_memcpy_htod(void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return GM_OK;
  BV_REQ(dst && src, "NULL pointer");
  return bv_status(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), "hipMemcpy H2D");
}
int gm_memcpy_dtoh(void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return GM_OK;
  BV_REQ(dst && src, "NULL pointer");
  return bv_status(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), "hipMemcpy D2H");
}
int gm_memcpy_dtod(void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return GM_OK;
  BV_REQ(dst && src, "NULL pointer");
  // 16-byte aligned buffers of a whole number of 16-byte words (the
  // allocator's buffers), both on the calling thread's current device: the
  // engine's own copy kernel; otherwise (another device, host memory,
  // unaligned) the runtime, which also handles cross-device copies
  if ((((uintptr_t)dst | (uintptr_t)src | (uintptr_t)bytes) & 15) == 0) {
    int dev = -1;
    hipPointerAttribute_t as{}, ad{};
    const bool qd = hipGetDevice(&dev) == hipSuccess;
    const bool qs = qd && hipPointerGetAttributes(&as, src) == hipSuccess;
    const bool qt = qs && hipPointerGetAttributes(&ad, dst) == hipSuccess;
    if (qt && as.type == hipMemoryTypeDevice && ad.type == hipMemoryTypeDevice && as.device == dev &&
        ad.device == dev)
      return bv_status(launch_copy16(src, dst, (long long)(bytes / 16), nullptr), "copy16");
    // only a query that itself failed (e.g. host memory the runtime does not
    // know) left an error to clear; an earlier pending error stays visible
    if (!qt) (void)hipGetLastError();
  }
  return bv_status(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, nullptr), "hipMemcpy D2D");
}

int gm_bv_kinetic_energy(gm_dtype dt, int64_t C, int64_t D, const void* p, void* ke) {
  BV_REQ(dtype_ok(dt), "bad dtype");
  BV_REQ(C >= 0 && D >= 1 && D <= 1024, "n_chains >= 0 and dim in [1, 1024] required");
  if (C == 0) return GM_OK;
  BV_REQ(p && ke, "NULL pointer");
  const Layout lay = default_layout((int)D, dt, GM_TARGET_ROSENBROCK);
  return bv_status(launch_bv_kinetic(dt, lay, C, (int)D, p, ke, nullptr), "kinetic_energy");
}
int gm_bv_masked_assign(gm_dtype dt, int64_t C, int64_t D, void* x, const void* o, const uint8_t* mask) {
  BV_REQ(dtype_ok(dt), "bad dtype");
  BV_REQ(C >= 0 && D >= 1, "bad shape");
  if (C == 0) return GM_OK;
  BV_REQ(x && o && mask, "NULL pointer");
  return bv_status(launch_bv_masked_assign(dt, C, (int)D, x, o, mask, nullptr), "masked_assign");
}
int gm_bv_add_scaled_assign(gm_dtype dt, int64_t n, void* x, const void* o, double alpha) {
  BV_REQ(dtype_ok(dt), "bad dtype");
  BV_REQ(n >= 0, "bad size");
  if (n == 0) return GM_OK;
  BV_REQ(x && o, "NULL pointer");
  return bv_status(launch_bv_axpy(dt, n, x, o, alpha, nullptr), "add_scaled_assign");
}
int gm_bv_scale_assign(gm_dtype dt, int64_t n, void* x, double alpha) {
  BV_REQ(dtype_ok(dt) && n >= 0 && (x || n == 0), "bad arguments");
  if (n == 0) return GM_OK;
  return bv_status(launch_bv_scale(dt, n, x, alpha, nullptr), "scale_assign");
}
int gm_bv_fill(gm_dtype dt, int64_t n, void* x, double value) {
  BV_REQ(dtype_ok(dt) && n >= 0 && (x || n == 0), "bad arguments");
  if (n == 0) return GM_OK;
  return bv_status(launch_bv_fill(dt, n, x, value, nullptr), "fill");
}
int gm_bv_dot(gm_dtype dt, int64_t n, const void* a, const void* b, double* out) {
  BV_REQ(dtype_ok(dt) && n >= 0 && out && ((a && b) || n == 0), "bad arguments");
  // one result slot per device (the calling thread may switch devices
  // between calls; a slot is never used across devices)
  static thread_local std::map<int, double*> slots;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    set_error("hipGetDevice failed in dot");
    return GM_EHIP;
  }
  double*& dres = slots[dev];
  if (!dres && hipMalloc(&dres, sizeof(double)) != hipSuccess) {
    dres = nullptr;
    set_error("device allocation failed in dot");
    return GM_ENOMEM;
  }
  int rc = bv_status(launch_bv_dot(dt, n, a, b, dres, nullptr), "dot");
  if (rc) return rc;
  return bv_status(hipMemcpy(out, dres, sizeof(double), hipMemcpyDeviceToHost), "dot copy");
}
int gm_bv_fill_random_normal(gm_dtype dt, int64_t C, int64_t D, void* out, uint64_t seed,
                             uint32_t chain_offset, uint64_t step) {
  BV_REQ(dtype_ok(dt), "bad dtype");
  BV_REQ(C >= 0 && D >= 1, "bad shape");
  if (C == 0) return GM_OK;
  BV_REQ(out, "NULL pointer");
  return bv_status(launch_bv_normal(dt, C, (int)D, out, seed, chain_offset, step, TAG_MOM, nullptr),
                   "fill_random_normal");
}
int gm_bv_sample_uniform(gm_dtype dt, int64_t C, void* out, uint64_t seed, uint32_t chain_offset,
                         uint64_t step) {
  BV_REQ(dtype_ok(dt), "bad dtype");
  BV_REQ(C >= 0, "bad size");
  if (C == 0) return GM_OK;
  BV_REQ(out, "NULL pointer");
  return bv_status(launch_bv_uniform(dt, C, out, seed, chain_offset, step, TAG_ACC, nullptr),
                   "sample_uniform");
}
static int energy(int op, gm_dtype dt, int64_t n, const void* a, const void* b, void* out) {
  BV_REQ(dtype_ok(dt), "bad dtype");
  BV_REQ(n >= 0, "bad size");
  if (n == 0) return GM_OK;
  BV_REQ(a && out && (b || op >= 2), "NULL pointer");
  return bv_status(launch_bv_energy(dt, op, n, a, b, out, nullptr), "energy op");
}
int gm_bv_energy_sub(gm_dtype dt, int64_t n, const void* a, const void* b, void* out) {
  return energy(0, dt, n, a, b, out);
}
int gm_bv_energy_add(gm_dtype dt, int64_t n, const void* a, const void* b, void* out) {
  return energy(1, dt, n, a, b, out);
}
int gm_bv_energy_neg(gm_dtype dt, int64_t n, const void* a, void* out) { return energy(2, dt, n, a, nullptr, out); }
int gm_bv_energy_ln(gm_dtype dt, int64_t n, const void* a, void* out) { return energy(3, dt, n, a, nullptr, out); }
int gm_bv_accept_mask(gm_dtype dt, int64_t n, const void* la, const void* lnu, uint8_t* mask) {
  BV_REQ(dtype_ok(dt), "bad dtype");
  BV_REQ(n >= 0, "bad size");
  if (n == 0) return GM_OK;
  BV_REQ(la && lnu && mask, "NULL pointer");
  return bv_status(launch_bv_accept(dt, n, la, lnu, mask, nullptr), "accept_mask");
}

int gm_bv_target_create(const gm_target* target, gm_dtype dt, gm_bv_target** out) {
  BV_REQ(out != nullptr, "out is NULL");
  *out = nullptr;
  BV_REQ(dtype_ok(dt), "bad dtype");
  BV_REQ(target != nullptr, "target is NULL");
  gm_bv_target* t = new gm_bv_target();
  t->dt = dt;
  const int rc = build_target(target, dt, target->dim, &t->tg, &t->d_mu, &t->d_prec);
  if (rc) {
    delete t;
    return rc;
  }
  *out = t;
  return GM_OK;
}
int gm_bv_logp_and_grad(gm_bv_target* t, int64_t C, const void* x, void* grad, void* logp) {
  BV_REQ(t != nullptr, "target is NULL");
  BV_REQ(C >= 0, "bad size");
  if (C == 0) return GM_OK;
  BV_REQ(x != nullptr, "x is NULL");
  const Layout lay = default_layout(t->tg.D, t->dt, t->tg.kind);
  return bv_status(launch_logp_grad(t->dt, t->tg, lay, C, x, logp, grad, nullptr), "logp_and_grad");
}
int gm_bv_leapfrog(gm_bv_target* t, int64_t C, void* q, void* p, void* g, void* logp, double step_size) {
  BV_REQ(t != nullptr, "target is NULL");
  BV_REQ(C >= 0, "bad size");
  BV_REQ(t->tg.kind != GM_TARGET_CUSTOM,
         "gm_bv_leapfrog: built-in targets only (compose gm_bv_add_scaled_assign and gm_bv_logp_and_grad)");
  if (C == 0) return GM_OK;
  BV_REQ(q && p && g, "NULL pointer");
  const Layout lay = default_layout(t->tg.D, t->dt, t->tg.kind);
  BV_REQ(!layout_is_wide(lay), "gm_bv_leapfrog: dim <= 1024");
  return bv_status(launch_leapfrog_hbm(t->dt, t->tg, lay, C, q, p, g, logp, step_size, nullptr), "leapfrog");
}
int gm_bv_target_destroy(gm_bv_target* t) {
  if (!t) return GM_OK;
  if (t->d_mu) hipFree(t->d_mu);
  if (t->d_prec) hipFree(t->d_prec);
  delete t;
  return GM_OK;
}

}  // extern "C"
