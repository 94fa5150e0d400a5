// gm_launch.h — kernel argument blocks (plain structs, device-safe: shared by
// the AOT kernels, the host launchers and the runtime-compiled user-target
// kernels of gm_jit.cpp).
#pragma once
#include <stdint.h>

namespace gm {

// ---- run_progress statistics (gm_track.h, tracker_kernels.hip) -------------
// Per-chain ChainTracker state (stats.rs:24-131), f32 [C][D] and [C]; mean
// is null when tracking is off. n0 = tracker steps before this launch.
struct TrackLaunch {
  float* mean = nullptr;
  float* msq = nullptr;
  float* last = nullptr;
  float* p = nullptr;
  unsigned long long n0 = 0;
};

// ---- HMC -------------------------------------------------------------------
struct HmcLaunch {
  void* q = nullptr;            // [C*D] state, in/out
  void* logp = nullptr;         // [C] out
  long long* accepts = nullptr; // [C] in/out (+= accepted count)
  void* samples = nullptr;      // [rows][C][D]
  long long C = 0;
  int D = 0;
  double eps = 0;
  int L = 0;
  uint64_t seed = 0;
  uint64_t step0 = 0;           // global transition index of the first step
  uint32_t chain_offset = 0;
  int n_steps = 0;
  int collect_from = 0;         // steps s >= collect_from are stored ...
  long long sample_row0 = 0;    // ... at row sample_row0 + (s - collect_from)
  int lf_unroll = 1;            // leapfrog loop unroll (1, 2 or 4; same results)
  void* zs = nullptr;           // wide layouts: momentum block scratch [C][S][lanes*elems]
};

// ---- MH --------------------------------------------------------------------
struct MhLaunch {
  void* q = nullptr;
  void* logp = nullptr;
  long long* accepts = nullptr;
  void* samples = nullptr;
  long long C = 0;
  int D = 0;
  double prop_std = 1;
  uint64_t seed = 0;
  uint64_t step0 = 0;
  uint32_t chain_offset = 0;
  int n_steps = 0;
  int collect_from = 0;
  long long sample_row0 = 0;
  TrackLaunch trk;              // run_progress chain trackers (off when trk.mean is null)
};

// ---- NUTS ------------------------------------------------------------------
// bytes of one HBM subtree-stack entry: three D-vectors, alpha, n, n_alpha,
// padded to whole 128-byte cache lines
inline long long nuts_stack_entry_bytes(int D, int tsz) {
  const long long b = 3LL * D * tsz + tsz + 8;
  return (b + 127) / 128 * 128;
}

struct NutsLaunch {
  void* q = nullptr;
  long long* accepts = nullptr;
  long long* n_leapfrog = nullptr;
  void* samples = nullptr;
  void* eps = nullptr;
  void* eps_bar = nullptr;
  void* h_bar = nullptr;
  void* mu = nullptr;
  void* stk_vec = nullptr;   // HBM stack levels: [C][max_depth] entries of stk_es bytes (gm_nuts.h)
  long long stk_es = 0;
  long long C = 0;
  int D = 0;
  int max_depth = 10;
  double target_accept = 0.8;
  uint64_t seed = 0;
  uint64_t step0 = 0;        // global transition index of this launch's first step
  uint64_t init_step = 0;    // transition counter value used for the init draw
  uint32_t chain_offset = 0;
  int n_steps = 0;
  long long m0 = 0;          // adaptation counter before this launch's first step
  long long n_discard = 0;
  int do_init = 0;           // run init_chain_state first (generic_nuts.rs:731-753)
  long long t0 = 0;          // transitions already done in this run before this launch
  long long row_shift = 0;   // state after t transitions goes to row t - row_shift
  long long n_rows = 0;
  TrackLaunch trk;           // run_progress chain trackers (off when trk.mean is null)
  // mass-matrix warm-up (generic_nuts.rs:33-359); mass_mode 0 = identity, off
  int mass_mode = 0;         // 1 diagonal, 2 dense
  int* mkind = nullptr;      // [C] current metric of each chain: 0 identity, 1 diag, 2 dense
  void* dinv = nullptr;      // [C][D]
  void* dsq = nullptr;       // [C][D]
  void* minv = nullptr;      // [C][D][D]
  void* mchol = nullptr;     // [C][D][D]
  void* mchol_rm = nullptr;  // [C][D][D] + D slack: L row-major (mchol is the per-chain transpose)
  int* rn = nullptr;         // [C] RunningCov::n
  void* rmean = nullptr;     // [C][D]
  void* rm2d = nullptr;      // [C][D]
  void* rm2 = nullptr;       // [C][D][D] (upper triangle used)
  int* updated = nullptr;    // [C] metric replaced at the previous launch's last step
  // levels k < lds_levels of the subtree stack live in LDS (after the
  // target's staging area, at byte offset lds_stack_off), the rest in HBM
  int lds_levels = 0;
  unsigned lds_stack_off = 0;
  // dense metric (mass_mode 2): each chain's M^-1 copied into LDS at kernel
  // start as its packed lower triangle (layout 16 x 2, at byte offset
  // minv_lds_off) when minv_lds, instead of re-read from L2/MALL at every
  // product (nuts_size_lds decides; nuts_device.h minv_packed_lds)
  int minv_lds = 0;
  unsigned minv_lds_off = 0;
  // and its Cholesky factor (the momentum draws), packed the same way, when
  // chol_lds (after M^-1, before the stack levels)
  int chol_lds = 0;
  unsigned chol_lds_off = 0;
  long long sb = 0, eb = 0;  // start_buffer, end_buffer (should_collect, :153-162)
  int do_refind = 0;         // re-find eps for updated chains first (:905-918)
  uint64_t refind_step = 0;  // transition index of the update (probe draws)
  // every chain's metric dense and no warm-up window in this launch: the
  // frozen-dense instantiation (nuts_device.h MASS 3, GM_FROZEN_WAVES waves
  // per SIMD) instead of the general adaptive one
  int dense_frozen = 0;
  // the launch's transition momenta as standard normals [n_steps][C][D]
  // (nuts_momenta_kernel: the same Philox/Box-Muller values the kernel would
  // draw), or null: drawn in the kernel
  const void* zmom = nullptr;
  // with zmom, each transition's start record from the same pass
  // (nuts_starts_kernel, [n_steps][C] of NutsStartRec<T>): the stream key K
  // of the TAG_NUTS_EXP block, ln of its Exp1 uniform, and the doublings'
  // direction bits (bit j: u(K, 2j) < 1/2) -- the values the kernel would
  // compute
  const void* zrec = nullptr;
  // frozen-dense launches (MASS 3) with zmom: the pass has also applied the
  // metric (nuts_dense_momenta_kernel), so zmom holds the momenta p0 = L z
  // themselves and pv0 their M^-1 p0, [n_steps][C][D] each -- the products
  // sample_momentum and the start's kinetic energy would otherwise take in
  // the tree kernel, with the same sums in the same order. Null: the kernel
  // applies L and M^-1 to zmom's normals itself.
  const void* pv0 = nullptr;
};
// the frozen-dense kernel takes its momenta from the pass (pv0 always set;
// nuts_run launches it for no other launch). 0: A/B builds only, the kernel
// applies the metric itself when pv0 is null
#ifndef GM_DENSE_PREP
#define GM_DENSE_PREP 1
#endif
// one start record: 16 bytes (f32) or 32 (f64), read as one 16-byte load
// (key, ln u) and, in f64, one 4-byte load (the direction bits)
template <class T> struct alignas(16) NutsStartRec {
  uint64_t key;
  T lnu;
  uint32_t dir;
};

// waves per SIMD of the NUTS dense-metric instantiations (their launch
// bounds, which the LDS plan of nuts_size_lds follows): the adaptive one
// (MASS 2) at 512 registers, the frozen one (MASS 3)
#ifndef GM_DENSE_WAVES
#define GM_DENSE_WAVES 1
#endif
#ifndef GM_FROZEN_WAVES
#define GM_FROZEN_WAVES 2
#endif
// waves per SIMD of the wide NUTS layouts (one chain per workgroup of
// lanes/64 waves, nuts_wide.hip): 2 up to 16 bytes of state per lane and
// vector (f64 x 2, f32 x 4), else 1 (f64 x 4 spills 58-140 registers at 2)
__host__ __device__ constexpr int nuts_wide_waves(int esz, int E) { return esz * E <= 16 ? 2 : 1; }

}  // namespace gm
