// gmcmc_diag.cpp — C ABI of the diagnostics (stats.rs split_rhat_mean_ess,
// stats.rs:439-450) and of the multi-GPU exchange (RCCL all-gather over
// xGMI of per-split-chain summaries).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <array>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>


#include "gm_diag.h"

using namespace gm;

#define GM_REQ(cond, msg) \
  do {                    \
    if (!(cond)) {        \
      set_error(msg);     \
      return GM_EINVAL;   \
    }                     \
  } while (0)
#define GM_HIP(expr)                                                               \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      set_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " #expr); \
      return GM_EHIP;                                                              \
    }                                                                              \
  } while (0)
#define GM_NCCL(expr)                                                                   \
  do {                                                                                  \
    ncclResult_t _r = (expr);                                                           \
    if (_r != ncclSuccess) {                                                            \
      set_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " #expr);    \
      return GM_ERCCL;                                                                  \
    }                                                                                   \
  } while (0)

namespace {
// Device buffers of the diagnostics, kept per (host thread, device) and only
// grown: a call then costs its kernels and copies, not hipMalloc/hipFree
// (hipFree synchronises the device). Never freed (process lifetime).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int alloc(size_t n) {
    if (n == 0) n = 8;
    if (cap >= n) return GM_OK;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, n) != hipSuccess) {
      p = nullptr;
      set_error("device allocation failed in diagnostics");
      return GM_ENOMEM;
    }
    cap = n;
    return GM_OK;
  }
};
struct DiagBufs {
  DevBuf cm, s2, ac, cm_all, s2_all, ac_all, out, cnt, cnt_all;
  DiagScratch ws;
};
DiagBufs& diag_bufs() {
  static thread_local std::map<int, DiagBufs*> per_device;
  int dev = 0;
  hipGetDevice(&dev);
  DiagBufs*& b = per_device[dev];
  if (!b) b = new DiagBufs();
  return *b;
}
}  // namespace

struct gm_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1;
  int rank = 0;
  int device = 0;
  hipStream_t stream = nullptr;
};

static int local_diag(const void* dev_sample, gm_dtype dtype, int64_t C, int64_t N, int64_t P,
                      int64_t sc, int64_t sd, int64_t sp, gm_comm* comm, float* rhat_out,
                      float* ess_out, hipStream_t st) {
  struct R {  // GMCMC_ROCTX=1: a roctx range per diagnostic call (gm::roctx_push)
    bool on;
    ~R() {
      if (on) gm::roctx_pop();
    }
  } rr{gm::roctx_push(comm ? "gm_split_rhat_ess_dist" : "gm_split_rhat_ess")};
  GM_REQ(dtype == GM_F32 || dtype == GM_F64, "bad dtype");
  GM_REQ(C >= 1 && N >= 2 && P >= 1, "need n_chains >= 1, n_draws >= 2, n_params >= 1");
  GM_REQ(dev_sample && rhat_out && ess_out, "NULL argument");
  const int h = (int)(N / 2);
  const int R = comm ? comm->nranks : 1;
  // local products
  DiagBufs& B = diag_bufs();
  DevBuf &cm = B.cm, &s2 = B.s2, &ac = B.ac, &cm_all = B.cm_all, &s2_all = B.s2_all,
         &ac_all = B.ac_all, &out = B.out;
  DiagScratch& ws = B.ws;
  int rc;
  if ((rc = cm.alloc(sizeof(double) * 2 * C * P)) || (rc = s2.alloc(sizeof(double) * 2 * C * P)) ||
      (rc = ac.alloc(sizeof(double) * h * P)) || (rc = out.alloc(sizeof(float) * 2 * P)))
    return rc;
  rc = diag_series(dtype, dev_sample, C, N, P, sc, sd, sp, (double*)cm.p, (double*)s2.p,
                   (double*)ac.p, ws, st);
  if (rc) return rc;
  const double *pcm = (double*)cm.p, *ps2 = (double*)s2.p, *pac = (double*)ac.p;
  if (R > 1) {
    // Every rank must pass the same shape: the grouped all-gather below is
    // sized from it, and unequal sizes would not match up across ranks (a
    // hang or corrupt data). The shape is therefore checked on EVERY call
    // (one 4-word all-gather + a host sync, tens of microseconds against the
    // summaries' kernels): a mismatch is GM_EINVAL on every rank, never a
    // mismatched collective.
    {
      const std::array<long long, 4> shape{(long long)C, (long long)N, (long long)P, (long long)dtype};
      DevBuf &cnt = B.cnt, &cnt_all = B.cnt_all;
      if ((rc = cnt.alloc(sizeof(shape))) || (rc = cnt_all.alloc(sizeof(shape) * R))) return rc;
      GM_HIP(hipMemcpyAsync(cnt.p, shape.data(), sizeof(shape), hipMemcpyHostToDevice, st));
      GM_NCCL(ncclAllGather(cnt.p, cnt_all.p, 4, ncclInt64, comm->comm, st));
      std::vector<std::array<long long, 4>> all(R);
      GM_HIP(hipMemcpyAsync(all.data(), cnt_all.p, sizeof(shape) * R, hipMemcpyDeviceToHost, st));
      GM_HIP(hipStreamSynchronize(st));
      for (int r = 0; r < R; ++r)
        if (all[r] != shape) {
          set_error("gm_split_rhat_ess_dist: all ranks must pass the same chain count, draws, params and dtype");
          return GM_EINVAL;
        }
    }
    if ((rc = cm_all.alloc(sizeof(double) * 2 * C * P * R)) ||
        (rc = s2_all.alloc(sizeof(double) * 2 * C * P * R)) ||
        (rc = ac_all.alloc(sizeof(double) * h * P * R)))
      return rc;
    GM_NCCL(ncclGroupStart());
    GM_NCCL(ncclAllGather(cm.p, cm_all.p, 2 * C * P, ncclFloat64, comm->comm, st));
    GM_NCCL(ncclAllGather(s2.p, s2_all.p, 2 * C * P, ncclFloat64, comm->comm, st));
    GM_NCCL(ncclAllGather(ac.p, ac_all.p, (size_t)h * P, ncclFloat64, comm->comm, st));
    GM_NCCL(ncclGroupEnd());
    pcm = (double*)cm_all.p;
    ps2 = (double*)s2_all.p;
    pac = (double*)ac_all.p;
  }
  rc = diag_final(pcm, ps2, pac, 2 * C * R, R, h, P, (float*)out.p, (float*)out.p + P, st);
  if (rc == GM_OK) {
    hipError_t e = hipMemcpyAsync(rhat_out, out.p, sizeof(float) * P, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
      e = hipMemcpyAsync(ess_out, (float*)out.p + P, sizeof(float) * P, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      set_error(std::string("diagnostics copy failed: ") + hipGetErrorString(e));
      rc = GM_EHIP;
    }
  }
  return rc;
}

extern "C" {

int gm_split_rhat_ess_device(const void* dev_sample, gm_dtype dtype, int64_t n_chains,
                             int64_t n_draws, int64_t n_params, int64_t stride_chain,
                             int64_t stride_draw, int64_t stride_param, float* rhat_out,
                             float* ess_out) {
  return local_diag(dev_sample, dtype, n_chains, n_draws, n_params, stride_chain, stride_draw,
                    stride_param, nullptr, rhat_out, ess_out, nullptr);
}

int gm_split_rhat_ess(const void* sample, gm_dtype dtype, int64_t n_chains, int64_t n_draws,
                      int64_t n_params, float* rhat_out, float* ess_out) {
  GM_REQ(dtype == GM_F32 || dtype == GM_F64, "bad dtype");
  GM_REQ(sample, "sample is NULL");
  GM_REQ(n_chains >= 1 && n_draws >= 2 && n_params >= 1,
         "need n_chains >= 1, n_draws >= 2, n_params >= 1");
  const size_t esz = dtype == GM_F32 ? 4 : 8;
  const size_t bytes = (size_t)n_chains * n_draws * n_params * esz;
  void* d = nullptr;  // the host sample's device copy lives for this call only
  if (hipMalloc(&d, bytes) != hipSuccess) {
    set_error("device allocation failed in diagnostics");
    return GM_ENOMEM;
  }
  int rc = GM_OK;
  if (hipMemcpy(d, sample, bytes, hipMemcpyHostToDevice) != hipSuccess) {
    set_error("copying the sample to the device failed");
    rc = GM_EHIP;
  } else {
    rc = local_diag(d, dtype, n_chains, n_draws, n_params, n_draws * n_params, n_params, 1, nullptr,
                    rhat_out, ess_out, nullptr);
  }
  hipFree(d);
  return rc;
}

int gm_comm_get_unique_id(void* id_out) {
  GM_REQ(id_out, "id_out is NULL");
  static_assert(sizeof(ncclUniqueId) <= GM_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId id;
  GM_NCCL(ncclGetUniqueId(&id));
  memset(id_out, 0, GM_UNIQUE_ID_BYTES);
  memcpy(id_out, &id, sizeof(id));
  return GM_OK;
}

int gm_comm_init(const void* id, int32_t nranks, int32_t rank, gm_comm** out) {
  GM_REQ(id && out && nranks >= 1 && rank >= 0 && rank < nranks, "bad arguments");
  *out = nullptr;
  gm_comm* c = new gm_comm();
  c->nranks = nranks;
  c->rank = rank;
  if (hipGetDevice(&c->device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    set_error("gm_comm_init: HIP setup failed");
    return GM_EHIP;
  }
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    hipStreamDestroy(c->stream);
    delete c;
    set_error(std::string("ncclCommInitRank failed: ") + ncclGetErrorString(r));
    return GM_ERCCL;
  }
  *out = c;
  return GM_OK;
}

int gm_comm_destroy(gm_comm* comm) {
  if (!comm) return GM_OK;
  hipSetDevice(comm->device);
  if (comm->comm) ncclCommDestroy(comm->comm);
  if (comm->stream) hipStreamDestroy(comm->stream);
  delete comm;
  return GM_OK;
}

int gm_comm_info(gm_comm* comm, int32_t* nranks, int32_t* rank, int32_t* device) {
  GM_REQ(comm && comm->comm, "comm is NULL");
  int n = 0, r = 0, d = 0;
  GM_NCCL(ncclCommCount(comm->comm, &n));
  GM_NCCL(ncclCommUserRank(comm->comm, &r));
  GM_NCCL(ncclCommCuDevice(comm->comm, &d));
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  if (device) *device = d;
  return GM_OK;
}

int gm_split_rhat_ess_dist(gm_comm* comm, const void* dev_sample, gm_dtype dtype,
                           int64_t n_chains_local, int64_t n_draws, int64_t n_params,
                           int64_t stride_chain, int64_t stride_draw, int64_t stride_param,
                           float* rhat_out, float* ess_out) {
  GM_REQ(comm, "comm is NULL");
  GM_HIP(hipSetDevice(comm->device));
  return local_diag(dev_sample, dtype, n_chains_local, n_draws, n_params, stride_chain, stride_draw,
                    stride_param, comm, rhat_out, ess_out, comm->stream);
}

int gm_split_rhat_ess_shards(const void* const* dev_shards, int32_t n_shards, gm_dtype dtype,
                             int64_t n_chains_per_shard, int64_t n_draws, int64_t n_params,
                             int64_t stride_chain, int64_t stride_draw, int64_t stride_param,
                             float* rhat_out, float* ess_out) {
  // The exchange of gm_split_rhat_ess_dist with every rank's shard on this
  // device: shard r's per-split-chain summaries are written where the RCCL
  // all-gather puts rank r's block ([R][P][2C], [R][h][P]), then the same
  // final kernel reads them.
  GM_REQ(dtype == GM_F32 || dtype == GM_F64, "bad dtype");
  GM_REQ(dev_shards && n_shards >= 1, "need n_shards >= 1 shard pointers");
  const int64_t C = n_chains_per_shard, N = n_draws, P = n_params;
  GM_REQ(C >= 1 && N >= 2 && P >= 1, "need n_chains >= 1, n_draws >= 2, n_params >= 1");
  GM_REQ(rhat_out && ess_out, "NULL argument");
  for (int r = 0; r < n_shards; ++r) GM_REQ(dev_shards[r], "shard pointer is NULL");
  const int h = (int)(N / 2), R = n_shards;
  DiagBufs& B = diag_bufs();
  int rc;
  if ((rc = B.cm_all.alloc(sizeof(double) * 2 * C * P * R)) ||
      (rc = B.s2_all.alloc(sizeof(double) * 2 * C * P * R)) ||
      (rc = B.ac_all.alloc(sizeof(double) * h * P * R)) || (rc = B.out.alloc(sizeof(float) * 2 * P)))
    return rc;
  double *cm = (double*)B.cm_all.p, *s2 = (double*)B.s2_all.p, *ac = (double*)B.ac_all.p;
  for (int r = 0; r < R; ++r) {
    rc = diag_series(dtype, dev_shards[r], C, N, P, stride_chain, stride_draw, stride_param,
                     cm + (size_t)r * 2 * C * P, s2 + (size_t)r * 2 * C * P, ac + (size_t)r * h * P,
                     B.ws, nullptr);
    if (rc) return rc;
  }
  rc = diag_final(cm, s2, ac, 2 * C * R, R, h, P, (float*)B.out.p, (float*)B.out.p + P, nullptr);
  if (rc) return rc;
  GM_HIP(hipMemcpy(rhat_out, B.out.p, sizeof(float) * P, hipMemcpyDeviceToHost));
  GM_HIP(hipMemcpy(ess_out, (float*)B.out.p + P, sizeof(float) * P, hipMemcpyDeviceToHost));
  return GM_OK;
}

}  // extern "C"
