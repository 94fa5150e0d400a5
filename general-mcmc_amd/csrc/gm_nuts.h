// gm_nuts.h — host-side interface of the NUTS engine (nuts_kernels.hip).
#pragma once
#include <functional>
#include <vector>

#include "gm_internal.h"

namespace gm {

constexpr int NUTS_DEFAULT_MAX_DEPTH = 10;
constexpr int NUTS_MAX_DEPTH_LIMIT = 30;

struct NutsState {
  bool inited = false;
  int max_depth = 0;
  void* eps = nullptr;      // [C] T   step size (generic_nuts.rs:573)
  void* eps_bar = nullptr;  // [C] T   (:581)
  void* h_bar = nullptr;    // [C] T   (:582)
  void* mu = nullptr;       // [C] T   (:580)
  // subtree-stack levels held in HBM: per chain max_depth entries of
  // stk_es bytes, entry = [3][D] T (left-subtree first q, first p, proposal
  // q), then alpha (T), n, n_alpha (int); one contiguous stretch per (chain,
  // level) (nuts_stack_entry_bytes)
  void* stk_vec = nullptr;
  long long stk_es = 0;
  long long lds_levels_cap = -1;  // subtree-stack levels in LDS: -1 as many as fit
  int dense_minv_lds = 1;     // dense M^-1 in LDS: 1 packed (the default: room for 6 stack levels),
                              // 2 full when it fits (else packed), 0 off
  int dense_chol_lds = 0;     // its Cholesky factor too (packed form only)
  int plan[6] = {0, 0, 0, 0, 0, 0};  // last launch: stack levels in LDS, M^-1 form, offset, L form, offset, frozen
  long long* n_leapfrog = nullptr;  // [C] cumulative leapfrog count
  long long m = 0;            // transitions since the last init_chain_state (:735)
  long long n_discard = 0;    // warm-up length of the current run (:734)
  // mass-matrix warm-up (GenericNUTS::new_with_mass_matrix, generic_nuts.rs:33-359)
  int mass_mode = 0;          // 0 off (identity), 1 diagonal, 2 dense
  long long m_sb = 0, m_eb = 0;
  double m_reg = 0, m_jit = 0;
  long long sched_next = 0, sched_len = 0;  // MassMatrixWarmup window schedule (persists)
  int* mkind = nullptr;       // [C] 0 identity, 1 diagonal, 2 dense
  void* dinv = nullptr;       // [C][D]
  void* dsq = nullptr;        // [C][D]
  void* minv = nullptr;       // [C][D][D]
  void* mchol = nullptr;      // [C][D][D]
  int* rn = nullptr;          // [C] RunningCov
  void* rmean = nullptr;      // [C][D]
  void* rm2d = nullptr;       // [C][D]
  void* rm2 = nullptr;        // [C][D][D]
  int* updated = nullptr;     // [C]
  void* mscratch = nullptr;   // [C][4][D][D] dense update workspace
  void* zbuf = nullptr;       // [steps][C][D] momentum normals of a launch (nuts_momenta_kernel)
  bool momentum_pass = true;  // gm_nuts_set_momentum_pass
#ifndef GM_NUTS_ZBUF_MAX
#define GM_NUTS_ZBUF_MAX (4ull << 30)  // at most 4 GiB (cfg3: 1 GiB per 500-transition launch)
#endif
  size_t zbuf_bytes = 0;
};

int nuts_init_state(NutsState* ns, gm_dtype dt, long long C, int D, int max_depth);
void nuts_free_state(NutsState* ns);
// Called after each launch with the transitions done so far in the run (the
// launch may still be in flight); non-zero aborts the run with that status.
using StepHook = std::function<int(long long)>;
// progress = 0: NUTS::run semantics; 1: run_progress semantics (see gmcmc.h);
// 2: NUTS::step, `total` transitions continuing the state (no init, nothing
// collected, n_discard ignored: the last run's)
int nuts_run(NutsState& ns, gm_dtype dt, const TargetDev& tg, const Layout& lay, void* q,
             long long* accepts, void* samples, long long C, int D, double target_accept,
             uint64_t seed, uint64_t* step, uint32_t chain_offset, long long total,
             long long n_discard, int progress, long long steps_per_launch, hipStream_t st,
             std::vector<hipEvent_t>& evs, double* ms, long long* launches,
             const TrackLaunch* trk = nullptr, const StepHook* hook = nullptr);
int nuts_set_mass(NutsState* ns, gm_dtype dt, long long C, int D, int mode, long long start_buffer,
                  long long end_buffer, long long initial_window, double regularize, double jitter);
int nuts_get_mass(NutsState& ns, gm_dtype dt, long long C, int D, int32_t* kind, void* dinv, void* dsqrt,
                  void* minv, void* mchol);
int nuts_get_step_size(NutsState& ns, gm_dtype dt, long long C, double* eps, double* eps_bar);
int nuts_get_leapfrogs(NutsState& ns, long long C, long long* out);

}  // namespace gm
