#include <cstdlib>
#include <cstdio>
// nuts_kernels.hip — many-chain No-U-Turn sampler for gfx950.
//
// Restates GenericNUTSChain::step (generic_nuts.rs:755-925) with the identity
// mass matrix that NUTS::new selects (generic_nuts.rs:370-377), including the
// reference's variant details:
//   * slice variable logu = joint - Exp1                         (:765-768)
//   * leaf: n' = [logu < joint], s' = [logu - 1000 < joint],
//           alpha' = min(1, exp(joint - joint0)) (Rust min: NaN -> 1) (:1197-1207)
//   * merge: right-half proposal taken iff U_f64 < n''/max(n'+n'',1)  (:1305-1306)
//           s' &= s'' & U-turn(endpoints, identity mass)            (:1316-1323)
//   * top level: move iff s' & U < min(1, n'/n), n starts at 1       (:860-868)
//   * dual averaging from the LAST subtree's alpha/n_alpha only      (:882-889)
// The reference's recursive build_tree is evaluated here iteratively: leaves
// are integrated in trajectory order and a completed subtree is merged with
// the stored left sibling of its level, which performs the merges (and their
// random draws) in exactly the recursion's post-order. A truncated subtree
// (s' = false) stops the leaf integration, and is still merged into every
// enclosing subtree of which it is (part of) the right half, as the
// recursion returns it upward.
//
// One lane group (LPC lanes x E coordinates) owns one chain; chains follow
// their own control flow. The per-level stack of stored left subtrees lives in
// global memory laid out [level][field][chain][coordinate]; every lane only
// ever reads back what it wrote itself, so no cross-lane ordering is needed.
#include "nuts_device.h"
#include "gm_jit.h"
#include "gm_layouts.h"
#include "nuts_launch.h"
#include "gm_nuts.h"
#include "gm_track.h"

namespace gm {
// ---- metric update at a window end (generic_nuts.rs:948-997, 175-359) ----
// One thread per chain, the reference's sequential arithmetic.
template <class T> __device__ __forceinline__ T rust_max(T a, T b) {  // Float::max
  return (a != a) ? b : (b != b) ? a : (a > b ? a : b);
}
template <class T> __device__ bool cholesky_spd(const T* a, int dim, T* l) {
  for (int i = 0; i < dim * dim; ++i) l[i] = (T)0;
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j <= i; ++j) {
      T sum = a[i * dim + j];
      for (int k = 0; k < j; ++k) sum = sum - l[i * dim + k] * l[j * dim + k];
      if (i == j) {
        if (sum <= (T)0 || !(sum - sum == (T)0)) return false;
        l[i * dim + j] = gsqrt(sum);
      } else {
        const T d = l[j * dim + j];
        if (d <= (T)0 || !(d - d == (T)0)) return false;
        l[i * dim + j] = sum / d;
      }
    }
  return true;
}
template <class T> __device__ bool invert_spd_from_cholesky(const T* l, int dim, T* inv, T* inv_l) {
  for (int i = 0; i < dim * dim; ++i) inv_l[i] = (T)0;
  for (int i = 0; i < dim; ++i) {
    const T d = l[i * dim + i];
    if (d <= (T)0 || !(d - d == (T)0)) return false;
    inv_l[i * dim + i] = (T)1 / d;
    for (int j = i + 1; j < dim; ++j) {
      T sum = (T)0;
      for (int k = i; k < j; ++k) sum = sum + l[j * dim + k] * inv_l[k * dim + i];
      inv_l[j * dim + i] = -sum / l[j * dim + j];
    }
  }
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j <= i; ++j) {
      T sum = (T)0;
      for (int k = (i > j ? i : j); k < dim; ++k) sum = sum + inv_l[k * dim + i] * inv_l[k * dim + j];
      inv[i * dim + j] = sum;
      inv[j * dim + i] = sum;
    }
  return true;
}
template <class T>
__device__ void diag_from_var(const T* var, int D, T jitter, T* inv, T* sq) {  // :205-216
  for (int i = 0; i < D; ++i) {
    const T v = rust_max(var[i], jitter);
    inv[i] = (T)1 / v;
    sq[i] = gsqrt(v);
  }
}

template <class T>
__global__ void nuts_mass_update_kernel(long long C, int D, int mode, double regularize, double jitter_cfg,
                                        int* __restrict__ mkind, T* dinv, T* dsq, T* minv, T* mchol,
                                        int* __restrict__ rn, T* rmean, T* rm2d, T* rm2,
                                        int* __restrict__ updated, T* scratch /* [C][4][D][D] */) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  updated[c] = 0;
  const int n = rn[c];
  if (n < 5) return;  // maybe_update_mass_matrix: None
  const T nd = (T)(n - 1);
  const T reg = (T)regularize;
  const T omr = (T)1 - reg;
  const T jitter = (T)(jitter_cfg > 1e-10 ? jitter_cfg : 1e-10);
  T* di = dinv + c * D;
  T* ds = dsq + c * D;
  bool ok = false;
  if (mode == 1) {
    T* var = rmean + c * D;  // the running stats are reset below; reuse mean as scratch
    const T* m2d = rm2d + c * D;
    for (int i = 0; i < D; ++i) var[i] = rust_max(omr * (m2d[i] / nd) + reg, jitter);
    diag_from_var(var, D, jitter, di, ds);
    mkind[c] = 1;
    ok = true;
  } else {
    const long long DD = (long long)D * D;
    T* cov = scratch + c * 4 * DD;
    T* tr = cov + DD;
    T* chol = tr + DD;
    T* il = chol + DD;
    const T* m2 = rm2 + c * DD;
    for (int i = 0; i < D; ++i)
      for (int j = i; j < D; ++j) {
        const T raw = m2[i * D + j] / nd;
        const T v = (i == j) ? rust_max(omr * raw + reg, jitter) : omr * raw;
        cov[i * D + j] = v;
        cov[j * D + i] = v;
      }
    // dense_from_cov (:218-236): up to 8 tries with a growing diagonal jitter
    T jj = rust_max(jitter, (T)1e-10);
    T* inv = minv + c * DD;
    for (int t = 0; t < 8 && !ok; ++t) {
      for (long long k = 0; k < DD; ++k) tr[k] = cov[k];
      for (int d = 0; d < D; ++d) tr[d * D + d] = tr[d * D + d] + jj;
      if (cholesky_spd(tr, D, chol) && invert_spd_from_cholesky(chol, D, tr, il)) ok = true;
      else jj = jj * (T)10;
    }
    if (ok) {
      for (long long k = 0; k < DD; ++k) {
        inv[k] = tr[k];
        mchol[c * DD + k] = chol[k];
      }
      mkind[c] = 2;
    } else if (mkind[c] == 0) {  // identity -> diagonal_from_var(ones)
      T* var = cov;
      for (int i = 0; i < D; ++i) var[i] = (T)1;
      diag_from_var(var, D, jitter, di, ds);
      mkind[c] = 1;
      ok = true;
    }
  }
  if (ok) {  // RunningCov::reset after a successful update (:920)
    updated[c] = 1;
    rn[c] = 0;
    for (int i = 0; i < D; ++i) {
      rmean[c * D + i] = (T)0;
      rm2d[c * D + i] = (T)0;
    }
    if (mode == 2)
      for (long long k = 0; k < (long long)D * D; ++k) rm2[c * (long long)D * D + k] = (T)0;
  }
}

// The transition momenta of a NUTS launch as standard normals, out[s][c][i]
// for steps step0 .. step0 + n - 1: the values nuts_kernel would draw at each
// transition start (normals_of over the (seed, chain, step / S, TAG_NUTS_MOM,
// i) Philox blocks, S steps per block), drawn here in one fully parallel pass
// -- every (block, chain, coordinate) at once -- instead of inside the tree
// loop, where each draw held up the wave's other chains at their transition
// start. Consecutive threads take consecutive coordinates (coalesced rows).
template <class T>
__global__ void nuts_momenta_kernel(uint64_t seed, uint32_t chain_offset, uint64_t step0, long long n, long long C,
                                    int D, T* __restrict__ out) {
  constexpr int S = Blk<T>::S;
  const uint64_t b0 = step0 / S;
  const long long nb = (long long)((step0 + (uint64_t)n - 1) / S - b0 + 1);
  const long long total = nb * C * D;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < total;
       k += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(k % D);
    const long long r = k / D;
    const long long c = r % C;
    const uint64_t b = b0 + (uint64_t)(r / C);
    T z[S];
    normals_of(draw_block(seed, chain_offset + (uint32_t)c, b, TAG_NUTS_MOM, (uint32_t)i), z);
#pragma unroll
    for (int u = 0; u < S; ++u) {
      const uint64_t st = b * S + (uint64_t)u;
      if (st >= step0 && st < step0 + (uint64_t)n) out[((long long)(st - step0) * C + c) * D + i] = z[u];
    }
  }
}

// Frozen-dense launches: the metric applied to the pass's normals, for every
// transition of the launch at once -- p0 = L z (sample_momentum,
// generic_nuts.rs:275-303) in place of z, and M^-1 p0 (the start's kinetic
// energy and carried velocity, :244-273) into v0 -- instead of at each
// transition start inside the tree kernel, where L came from HBM on the
// start's critical path and streamed 8 KiB per transition through the L2 the
// subtree stack lives in. The sums are the tree kernel's (nuts_device.h
// momentum_from / chol_global_cols and inv_mul / packed_cols): p_i from +0,
// j ascending, a separate multiply and add (the build does not contract);
// (M^-1 p)_i from +0 by fma, j ascending. The kernel's padded terms (j > i in
// L, columns past D) add +-0 to a +0-started sum and change no bit, so they
// are left out here. One block per chain: its L (transposed) and M^-1
// (transposed, as the tree kernel's copy) staged in LDS once, then
// R = DPREP_THREADS / D transitions per round, thread (r, i) computing
// coordinate i of transition s0 + r. Its LDS: nuts_dense_prep_lds (<= 64 KiB, else the tree
// kernel applies the metric itself).
constexpr int DPREP_THREADS = 1024;  // (cfg3_dense: 1.6 ms with 256 or 1024; 4.8 ms before the conflict-free [j][i] M^-1 view)
static size_t nuts_dense_prep_lds(int D, size_t esz) {
  if (D < 1 || D > 256) return 0;
  const size_t b = (2 * (size_t)D * D + 2 * (size_t)(DPREP_THREADS / D) * D) * esz;
  return b <= 64 * 1024 ? b : 0;
}
template <class T>
__global__ __launch_bounds__(DPREP_THREADS) void nuts_dense_momenta_kernel(long long n, long long C, int D,
                                                                 const T* __restrict__ chol_rm,
                                                                 const T* __restrict__ minvT, T* __restrict__ pz,
                                                                 T* __restrict__ v0) {
  extern __shared__ __align__(16) unsigned char dm_lds[];
  // [j][i] (lane i of a row reads consecutive words: no bank conflicts)
  T* lt = (T*)dm_lds;       // L_ij
  T* mt = lt + D * D;       // row i's entry j of the tree kernel's packed M^-1:
                            // M^-1_ij while j <= i, M^-1_ji after (the same
                            // values: M^-1 is exactly symmetric, and these are
                            // the very words its product reads)
  T* zl = mt + D * D;       // [r][j] this round's normals, then momenta
  const long long c = blockIdx.x;
  const T* L = chol_rm + c * (long long)D * D;
  const T* Mi = minvT + c * (long long)D * D;  // Mi[j*D + i] = M^-1_ij
  for (int k = threadIdx.x; k < D * D; k += blockDim.x) {
    const int j = k / D, i = k - j * D;
    lt[k] = L[i * D + j];  // L row-major
    mt[k] = j <= i ? Mi[k] : Mi[i * D + j];
  }
  const int R = DPREP_THREADS / D;
  const int r = threadIdx.x / D, i = threadIdx.x - r * D;
  const bool act = r < R;
  T* pl = zl + R * D;  // [r][j] this round's momenta
  // (the next round's normal loaded while this round's sums run; zl is
  // rewritten only after every thread's reads of it, behind the second
  // barrier of the previous round, and pl likewise behind the first)
  T zn = (act && r < n) ? pz[((long long)r * C + c) * D + i] : (T)0;
  for (long long s0 = 0; s0 < n; s0 += R) {
    const long long s = s0 + r;
    const bool on = act && s < n;
    const long long o = (s * C + c) * D + i;
    if (on) zl[r * D + i] = zn;
    __syncthreads();
    if (act && s + R < n) zn = pz[o + (long long)R * C * D];
    T p = (T)0;
    if (on) {
      for (int j = 0; j <= i; ++j) p = p + lt[j * D + i] * zl[r * D + j];
      pl[r * D + i] = p;
    }
    __syncthreads();
    if (on) {
      T w = (T)0;
      for (int j = 0; j < D; ++j) w = gfma(mt[j * D + i], pl[r * D + j], w);
      pz[o] = p;
      v0[o] = w;
    }
  }
}

// Each transition's start record (nuts_device.h, transition start and
// doubling ends): the TAG_NUTS_EXP block's stream key, ln of its Exp1
// uniform and the direction bits of doublings 0..max_depth-1 -- a Philox
// block, a log and max_depth hashes that a starting chain's wave otherwise
// waits for in the tree kernel. The same functions, so the same bits.
template <class T>
__global__ void nuts_starts_kernel(uint64_t seed, uint32_t chain_offset, uint64_t step0, long long n, long long C,
                                   int max_depth, NutsStartRec<T>* __restrict__ rec) {
  const long long total = n * C;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < total;
       k += (long long)gridDim.x * blockDim.x) {
    const long long c = k % C;
    const uint64_t st = step0 + (uint64_t)(k / C);
    const u32x4 kw = draw_block(seed, chain_offset + (uint32_t)c, st, TAG_NUTS_EXP, 0u);
    const uint64_t K = nuts_key(kw);
    uint32_t bits = 0;
    for (int j = 0; j < max_depth && j < 32; ++j)
      bits |= (nuts_u<T>(K, 2u * (uint32_t)j) < (T)0.5) ? (1u << j) : 0u;
    NutsStartRec<T> r;
    r.key = K;
    r.lnu = glog_pos(Unif<T>::oc(kw.z, kw.w));
    r.dir = bits;
    rec[k] = r;
  }
}

template <class T>
__global__ void nuts_fill_kernel(T* eps, T* eps_bar, T* h_bar, T* mu, long long C) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C) return;
  eps[i] = (T)-1;                   // generic_nuts.rs:619
  eps_bar[i] = (T)1;                // :645
  h_bar[i] = (T)0;                  // :646
  mu[i] = glog((T)10 * (T)1);       // :644
}

// [C][D][D] -> per-chain transposes (the sampling kernel reads a chain's
// dense metric column by column: with the transpose, the chain's lanes read
// one contiguous row per column instead of one cache line each)
template <class T>
__global__ void mat_transpose_kernel(long long C, int D, const T* __restrict__ in, T* __restrict__ out) {
  const long long dd = (long long)D * D, n = C * dd;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (long long)gridDim.x * blockDim.x) {
    const long long c = k / dd;
    const int r = (int)(k - c * dd), i = r / D, j = r - i * D;
    out[c * dd + (long long)j * D + i] = in[k];
  }
}

int nuts_init_state(NutsState* ns, gm_dtype dt, long long C, int D, int max_depth) {
  const size_t esz = dt == GM_F32 ? 4 : 8;
  ns->max_depth = max_depth;
  hipError_t e = hipSuccess;
  e = hipMalloc(&ns->eps, C * esz);
  if (e == hipSuccess) e = hipMalloc(&ns->eps_bar, C * esz);
  if (e == hipSuccess) e = hipMalloc(&ns->h_bar, C * esz);
  if (e == hipSuccess) e = hipMalloc(&ns->mu, C * esz);
  if (e == hipSuccess) e = hipMalloc((void**)&ns->n_leapfrog, C * sizeof(long long));
  ns->stk_es = nuts_stack_entry_bytes(D, (int)esz);
  if (e == hipSuccess && max_depth > 0) e = hipMalloc(&ns->stk_vec, (size_t)C * max_depth * ns->stk_es);
  if (e != hipSuccess) {
    set_error(std::string("NUTS state allocation failed: ") + hipGetErrorString(e));
    return GM_ENOMEM;
  }
  hipMemset(ns->n_leapfrog, 0, C * sizeof(long long));
  const unsigned blocks = (unsigned)((C + 255) / 256);
  if (dt == GM_F32)
    hipLaunchKernelGGL(nuts_fill_kernel<float>, dim3(blocks), dim3(256), 0, 0, (float*)ns->eps,
                       (float*)ns->eps_bar, (float*)ns->h_bar, (float*)ns->mu, C);
  else
    hipLaunchKernelGGL(nuts_fill_kernel<double>, dim3(blocks), dim3(256), 0, 0, (double*)ns->eps,
                       (double*)ns->eps_bar, (double*)ns->h_bar, (double*)ns->mu, C);
  e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    set_error(std::string("NUTS state init failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  ns->inited = true;
  return GM_OK;
}

static void ffree(void* p) {
  if (p) hipFree(p);
}

static void mass_free(NutsState* ns) {
  ffree(ns->mkind);
  ffree(ns->dinv);
  ffree(ns->dsq);
  ffree(ns->minv);
  ffree(ns->mchol);
  ffree(ns->rn);
  ffree(ns->rmean);
  ffree(ns->rm2d);
  ffree(ns->rm2);
  ffree(ns->updated);
  ffree(ns->mscratch);
  ns->mkind = ns->rn = ns->updated = nullptr;
  ns->dinv = ns->dsq = ns->minv = ns->mchol = ns->rmean = ns->rm2d = ns->rm2 = ns->mscratch = nullptr;
  ns->mass_mode = 0;
}

int nuts_set_mass(NutsState* ns, gm_dtype dt, long long C, int D, int mode, long long start_buffer,
                  long long end_buffer, long long initial_window, double regularize, double jitter) {
  mass_free(ns);
  if (mode == 0) return GM_OK;
  const size_t esz = dt == GM_F32 ? 4 : 8;
  const size_t cd = (size_t)C * D * esz, cdd = (size_t)C * D * D * esz;
  hipError_t e = hipMalloc((void**)&ns->mkind, C * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&ns->dinv, cd);
  if (e == hipSuccess) e = hipMalloc(&ns->dsq, cd);
  if (e == hipSuccess) e = hipMalloc((void**)&ns->rn, C * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&ns->rmean, cd);
  if (e == hipSuccess) e = hipMalloc(&ns->rm2d, cd);
  if (e == hipSuccess) e = hipMalloc((void**)&ns->updated, C * sizeof(int));
  if (mode == 2) {
    if (e == hipSuccess) e = hipMalloc(&ns->minv, cdd);
    // (+ D elements: the 16 x 2 start's row reads run past a chain's last row
    // into the padded columns of a D < 32 metric; nuts_device.h chol_global_cols)
    if (e == hipSuccess) e = hipMalloc(&ns->mchol, cdd + (size_t)D * esz);
    if (e == hipSuccess) e = hipMalloc(&ns->rm2, cdd);
    if (e == hipSuccess) e = hipMalloc(&ns->mscratch, 4 * cdd);
  }
  if (e != hipSuccess) {
    mass_free(ns);
    set_error(std::string("mass-matrix state allocation failed: ") + hipGetErrorString(e));
    return GM_ENOMEM;
  }
  hipMemset(ns->mkind, 0, C * sizeof(int));  // MassMatrix::identity
  hipMemset(ns->dinv, 0, cd);
  hipMemset(ns->dsq, 0, cd);
  if (mode == 2) {
    hipMemset(ns->minv, 0, cdd);
    hipMemset(ns->mchol, 0, cdd + (size_t)D * esz);
  }
  ns->mass_mode = mode;
  ns->m_sb = start_buffer;
  ns->m_eb = end_buffer;
  ns->m_reg = regularize;
  ns->m_jit = jitter;
  // MassMatrixWarmup::new (generic_nuts.rs:141-151)
  ns->sched_len = initial_window > 10 ? initial_window : 10;
  ns->sched_next = (start_buffer > 1 ? start_buffer : 1) + ns->sched_len;
  return hipDeviceSynchronize() == hipSuccess ? GM_OK : GM_EHIP;
}

int nuts_get_mass(NutsState& ns, gm_dtype dt, long long C, int D, int32_t* kind, void* dinv, void* dsqrt,
                  void* minv, void* mchol) {
  const size_t esz = dt == GM_F32 ? 4 : 8;
  if (!ns.mass_mode) {
    if (kind)
      for (long long c = 0; c < C; ++c) kind[c] = 0;
    return GM_OK;
  }
  hipError_t e = hipSuccess;
  if (kind) e = hipMemcpy(kind, ns.mkind, C * sizeof(int), hipMemcpyDeviceToHost);
  if (e == hipSuccess && dinv) e = hipMemcpy(dinv, ns.dinv, (size_t)C * D * esz, hipMemcpyDeviceToHost);
  if (e == hipSuccess && dsqrt) e = hipMemcpy(dsqrt, ns.dsq, (size_t)C * D * esz, hipMemcpyDeviceToHost);
  if (ns.mass_mode == 2) {
    if (e == hipSuccess && minv) e = hipMemcpy(minv, ns.minv, (size_t)C * D * D * esz, hipMemcpyDeviceToHost);
    if (e == hipSuccess && mchol) e = hipMemcpy(mchol, ns.mchol, (size_t)C * D * D * esz, hipMemcpyDeviceToHost);
  }
  if (e != hipSuccess) {
    set_error(std::string("mass-matrix copy failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  return GM_OK;
}

void nuts_free_state(NutsState* ns) {
  mass_free(ns);
  ffree(ns->eps);
  ffree(ns->eps_bar);
  ffree(ns->h_bar);
  ffree(ns->mu);
  ffree(ns->stk_vec);
  ffree(ns->n_leapfrog);
  ffree(ns->zbuf);
  *ns = NutsState();
}

int nuts_run(NutsState& ns, gm_dtype dt, const TargetDev& tg, const Layout& lay, void* q,
             long long* accepts, void* samples, long long C, int D, double target_accept,
             uint64_t seed, uint64_t* step, uint32_t chain_offset, long long total,
             long long n_discard, int progress, long long steps_per_launch, hipStream_t st,
             std::vector<hipEvent_t>& evs, double* ms, long long* launches, const TrackLaunch* trk,
             const StepHook* hook) {
  const size_t esz = dt == GM_F32 ? 4 : 8;
  // progress == 2: NUTS::step (nuts.rs:431-433 -> generic_nuts.rs:755-925):
  // transitions that continue the chain state without init_chain_state, the
  // adaptation counter running on against the last run's n_discard, nothing
  // collected
  const bool step_mode = progress == 2;
  if (!step_mode) {  // init_chain_state at the start of every run (generic_nuts.rs:731-753)
    ns.m = 0;
    ns.n_discard = n_discard;
  }
  const uint64_t init_step = *step;
  const long long n_rows_total = step_mode ? 0 : progress ? total - n_discard : total - n_discard + 1;
  const long long row_shift = progress ? n_discard + 1 : n_discard;
  // Launch segments: at most steps_per_launch transitions each, and a
  // segment also ends at every warm-up window end, after which the metric
  // update kernel runs and the next segment starts with the probe + epsilon
  // re-find (generic_nuts.rs:897-921). The window schedule depends on m and
  // n_discard only, so it is the same for every chain.
  const long long chunk = steps_per_launch;
  std::vector<long long> seg_start, seg_len;
  std::vector<char> seg_update;
  {
    std::vector<long long> wends;
    if (ns.mass_mode && !step_mode) {  // (a step runs past the warm-up: m > n_discard)
      const long long lim = n_discard > ns.m_eb ? n_discard - ns.m_eb : 0;
      for (long long m = 1; m <= total && m <= n_discard; ++m) {
        if (m <= ns.m_sb || !(m < lim)) continue;  // should_collect
        if (m >= ns.sched_next || m + 1 >= lim) {  // note_if_window_end
          ns.sched_next += ns.sched_len;
          ns.sched_len = ns.sched_len * 2 < 400 ? ns.sched_len * 2 : 400;
          wends.push_back(m);
        }
      }
    }
    size_t wi = 0;
    long long s0 = 0;
    do {
      long long n = total - s0 < chunk ? total - s0 : chunk;
      if (n < 0) n = 0;
      char upd = 0;
      if (wi < wends.size() && wends[wi] <= s0 + n) {  // cut at the window end (step m = s0 + n)
        n = wends[wi] - s0;
        upd = 1;
        ++wi;
      }
      seg_start.push_back(s0);
      seg_len.push_back(n);
      seg_update.push_back(upd);
      s0 += n;
    } while (s0 < total);
    if (seg_update.back()) {  // an update on the last transition still re-finds epsilon
      seg_start.push_back(total);
      seg_len.push_back(0);
      seg_update.push_back(0);
    }
  }
  const long long n_launch = (long long)seg_start.size();
  while ((long long)evs.size() < 2 * n_launch) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) {
      set_error("hipEventCreate failed");
      return GM_EHIP;
    }
    evs.push_back(ev);
  }
  if (ns.mass_mode && !step_mode) {  // RunningCov::reset in init_chain_state (:744-746)
    hipMemsetAsync(ns.rn, 0, C * sizeof(int), st);
    hipMemsetAsync(ns.rmean, 0, (size_t)C * D * esz, st);
    hipMemsetAsync(ns.rm2d, 0, (size_t)C * D * esz, st);
    if (ns.mass_mode == 2) hipMemsetAsync(ns.rm2, 0, (size_t)C * D * D * esz, st);
    hipMemsetAsync(ns.updated, 0, C * sizeof(int), st);
  }
  // The frozen-dense instantiation (MASS 3) for launches without a window
  // end or Welford collection when every chain's metric is dense: read the
  // chains' kinds back once (after the stream's earlier work)
  bool all_dense = false;
  bool any_update = false;
  for (char u : seg_update) any_update = any_update || u;
  if (ns.mass_mode == 2 && !any_update && tg.kind != GM_TARGET_CUSTOM && lay.lanes == 16 && lay.elems == 2) {
    std::vector<int> kinds((size_t)C);
    if (hipMemcpyAsync(kinds.data(), ns.mkind, C * sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      set_error("copy of the NUTS metric kinds failed");
      return GM_EHIP;
    }
    all_dense = C > 0;
    for (int k : kinds) all_dense = all_dense && k == 2;
  }
  int pending_refind = 0;
  uint64_t refind_step = 0;
  NutsLdsBudget budget;
  budget.lds_cap = ns.lds_levels_cap;  // gm_nuts_set_lds_levels (-1: as many as fit)
  // dense M^-1 resident in LDS (layout 16 x 2) when it fits: full matrices
  // or packed lower triangles (nuts_size_lds); gm_nuts_set_dense_forms picks
  // packed only or global memory (identical results)
  budget.minv_lds = ns.dense_minv_lds;
  budget.chol_lds = ns.dense_chol_lds;
  {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&budget.ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        budget.ncu < 1)
      budget.ncu = 256;
    if (hipDeviceGetAttribute(&budget.lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess ||
        budget.lds_max < 1)
      budget.lds_max = 64 * 1024;
  }
  for (long long li = 0; li < n_launch; ++li) {
    const long long start = seg_start[li], nst = seg_len[li];
    NutsLaunch a;
    a.q = q;
    a.accepts = accepts;
    a.n_leapfrog = ns.n_leapfrog;
    a.samples = samples;
    a.eps = ns.eps;
    a.eps_bar = ns.eps_bar;
    a.h_bar = ns.h_bar;
    a.mu = ns.mu;
    a.stk_vec = ns.stk_vec;
    a.stk_es = ns.stk_es;
    a.C = C;
    a.D = D;
    a.max_depth = ns.max_depth;
    a.target_accept = target_accept;
    a.seed = seed;
    a.step0 = *step + start;
    a.init_step = init_step;
    a.chain_offset = chain_offset;
    a.n_steps = (int)nst;
    a.m0 = ns.m + start;
    a.n_discard = ns.n_discard;
    a.do_init = (!step_mode && start == 0 && li == 0) ? 1 : 0;
    a.t0 = start;
    a.row_shift = row_shift;
    a.n_rows = n_rows_total > 0 ? n_rows_total : 0;
    if (ns.mass_mode) {
      a.mass_mode = ns.mass_mode;
      a.mkind = ns.mkind;
      a.dinv = ns.dinv;
      a.dsq = ns.dsq;
      a.minv = ns.minv;
      a.mchol = ns.mchol;
      a.mchol_rm = ns.mchol;
      if (ns.mass_mode == 2) {  // the transposes, in the update kernel's scratch (free between its launches)
        const size_t esz = dt == GM_F32 ? 4 : 8, cdd = (size_t)C * D * D * esz;
        void* mT = ns.mscratch;
        void* lT = (char*)ns.mscratch + cdd;
        const long long n = C * (long long)D * D;
        const unsigned tb = (unsigned)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
        if (dt == GM_F32) {
          hipLaunchKernelGGL(mat_transpose_kernel<float>, dim3(tb), dim3(256), 0, st, C, D, (const float*)ns.minv,
                             (float*)mT);
          hipLaunchKernelGGL(mat_transpose_kernel<float>, dim3(tb), dim3(256), 0, st, C, D,
                             (const float*)ns.mchol, (float*)lT);
        } else {
          hipLaunchKernelGGL(mat_transpose_kernel<double>, dim3(tb), dim3(256), 0, st, C, D,
                             (const double*)ns.minv, (double*)mT);
          hipLaunchKernelGGL(mat_transpose_kernel<double>, dim3(tb), dim3(256), 0, st, C, D,
                             (const double*)ns.mchol, (double*)lT);
        }
        a.minv = mT;
        a.mchol = lT;
      }
      a.rn = ns.rn;
      a.rmean = ns.rmean;
      a.rm2d = ns.rm2d;
      a.rm2 = ns.rm2;
      a.updated = ns.updated;
      a.sb = ns.m_sb;
      a.eb = ns.m_eb;
      a.do_refind = pending_refind;
      a.refind_step = refind_step;
      // no Welford collection in the launch: every m >= lim or m <= start_buffer
      const long long lim = ns.n_discard > ns.m_eb ? ns.n_discard - ns.m_eb : 0;
      a.dense_frozen = (all_dense && !a.do_refind && (a.m0 + 1 >= lim || a.m0 + nst <= ns.m_sb)) ? 1 : 0;
    }
    if (trk) {
      a.trk = *trk;
      a.trk.n0 = trk->n0 + (unsigned long long)start;
    }
    hipEventRecord(evs[2 * li], st);
    // the launch's momenta in one parallel pass ahead of the tree kernel
    // (same values; skipped past GM_NUTS_ZBUF_MAX bytes, the kernel then draws
    // them itself), timed with the launch
    {
      // [nst][C][D] momenta, then the start records [nst][C] (16-byte aligned)
      const size_t nsc = (size_t)(nst > 0 ? nst : 0) * (size_t)C;
      const size_t zmb = (nsc * (size_t)D * esz + 15) / 16 * 16;
      const size_t zrb = nsc * (dt == GM_F32 ? sizeof(NutsStartRec<float>) : sizeof(NutsStartRec<double>));
      // a frozen-dense launch (the MASS 3 kernel, 16 x 2): the metric applied
      // in the pass as well, M^-1 p0 [nst][C][D] after the records
      // (the frozen kernel is built for this pass, GM_DENSE_PREP: a launch the
      // pass cannot serve -- pass off, buffer past its cap or not allocated --
      // takes the adaptive dense kernel instead, the same bits)
      const size_t dpl = (a.mass_mode == 2 && a.dense_frozen) ? nuts_dense_prep_lds(D, esz) : 0;
      const size_t zvo = (zmb + zrb + 15) / 16 * 16;
      if (GM_DENSE_PREP && a.dense_frozen &&
          !(dpl > 0 && C <= 0x7fffffff && ns.momentum_pass && zvo + zmb <= (size_t)GM_NUTS_ZBUF_MAX))
        a.dense_frozen = 0;
      const bool dprep = GM_DENSE_PREP && a.dense_frozen;
      const size_t zb = dprep ? zvo + zmb : zmb + zrb;
      if (ns.momentum_pass && zb > 0 && zb <= (size_t)GM_NUTS_ZBUF_MAX) {
        if (zb > ns.zbuf_bytes) {
          if (ns.zbuf) hipFree(ns.zbuf);
          ns.zbuf = nullptr;
          ns.zbuf_bytes = 0;
          // at most a quarter of the device memory free now: the buffer is
          // kept for the sampler's later launches (gm_nuts_set_momentum_pass(s,
          // 0) releases it), and must not crowd out other samplers' or the
          // caller's allocations; without it the kernel draws its momenta
          size_t fr = 0, tot = 0;
          if (hipMemGetInfo(&fr, &tot) == hipSuccess && zb <= fr / 4 && hipMalloc(&ns.zbuf, zb) == hipSuccess)
            ns.zbuf_bytes = zb;
          else
            (void)hipGetLastError();
        }
        if (ns.zbuf) {
          const long long S = dt == GM_F32 ? 4 : 2;
          const long long nb = (long long)((a.step0 + (uint64_t)nst - 1) / S - a.step0 / S + 1);
          const long long work = nb * C * D;
          const unsigned zbk = (unsigned)((work + 255) / 256 < 65536 ? (work + 255) / 256 : 65536);
          void* zr = (char*)ns.zbuf + zmb;
          const unsigned sbk = (unsigned)((nsc + 255) / 256 < 65536 ? (nsc + 255) / 256 : 65536);
          // (the frozen-dense kernel draws its starts itself: GM_SREC_DENSE)
          const bool recs = !(a.mass_mode == 2 && a.dense_frozen && !GM_SREC_DENSE);
          if (dt == GM_F32) {
            hipLaunchKernelGGL(nuts_momenta_kernel<float>, dim3(zbk), dim3(256), 0, st, seed, chain_offset, a.step0,
                               nst, C, D, (float*)ns.zbuf);
            if (recs)
              hipLaunchKernelGGL(nuts_starts_kernel<float>, dim3(sbk), dim3(256), 0, st, seed, chain_offset, a.step0,
                                 nst, C, ns.max_depth, (NutsStartRec<float>*)zr);
          } else {
            hipLaunchKernelGGL(nuts_momenta_kernel<double>, dim3(zbk), dim3(256), 0, st, seed, chain_offset,
                               a.step0, nst, C, D, (double*)ns.zbuf);
            if (recs)
              hipLaunchKernelGGL(nuts_starts_kernel<double>, dim3(sbk), dim3(256), 0, st, seed, chain_offset,
                                 a.step0, nst, C, ns.max_depth, (NutsStartRec<double>*)zr);
          }
          if (dprep) {  // p0 = L z in place of z, M^-1 p0 at zvo
            void* pv = (char*)ns.zbuf + zvo;
            if (dt == GM_F32)
              hipLaunchKernelGGL(nuts_dense_momenta_kernel<float>, dim3((unsigned)C), dim3(DPREP_THREADS), dpl, st, nst, C, D,
                                 (const float*)a.mchol_rm, (const float*)a.minv, (float*)ns.zbuf, (float*)pv);
            else
              hipLaunchKernelGGL(nuts_dense_momenta_kernel<double>, dim3((unsigned)C), dim3(DPREP_THREADS), dpl, st, nst, C,
                                 D, (const double*)a.mchol_rm, (const double*)a.minv, (double*)ns.zbuf,
                                 (double*)pv);
            a.pv0 = pv;
          }
          a.zmom = ns.zbuf;
          a.zrec = recs ? zr : nullptr;
        }
      }
      if (GM_DENSE_PREP && a.dense_frozen && a.pv0 == nullptr) a.dense_frozen = 0;  // (no buffer)
    }
    hipError_t e;
    if (tg.kind == GM_TARGET_CUSTOM) {  // user target, runtime-compiled (gm_jit.cpp)
      const unsigned blocks = (unsigned)((C + 255) / 256);
      const size_t lds = nuts_size_lds(a, budget, blocks, 0, 1, D, esz);
      UserTargetArg ut{tg.params, tg.D};
      void* args[] = {&a, &ut};
      e = jit_launch(JIT_NUTS, dt, tg, blocks, 256, lds, st, args);
    } else {
      e = nuts_launch_layout(dt, tg, lay, a, st, budget);
    }
    ns.plan[0] = a.lds_levels;  // gm_nuts_get_plan
    ns.plan[1] = a.minv_lds;
    ns.plan[2] = (int)a.minv_lds_off;
    ns.plan[3] = a.chol_lds;
    ns.plan[4] = (int)a.chol_lds_off;
    ns.plan[5] = a.dense_frozen;
    if (e != hipSuccess) {
      set_error(std::string("NUTS launch failed: ") + hipGetErrorString(e));
      return GM_EHIP;
    }
    hipEventRecord(evs[2 * li + 1], st);
    pending_refind = 0;
    if (seg_update[li]) {  // maybe_update_mass_matrix for every chain
      const unsigned blocks = (unsigned)((C + 63) / 64);
      if (dt == GM_F32)
        hipLaunchKernelGGL(nuts_mass_update_kernel<float>, dim3(blocks), dim3(64), 0, st, C, D, ns.mass_mode,
                           ns.m_reg, ns.m_jit, ns.mkind, (float*)ns.dinv, (float*)ns.dsq, (float*)ns.minv,
                           (float*)ns.mchol, ns.rn, (float*)ns.rmean, (float*)ns.rm2d, (float*)ns.rm2,
                           ns.updated, (float*)ns.mscratch);
      else
        hipLaunchKernelGGL(nuts_mass_update_kernel<double>, dim3(blocks), dim3(64), 0, st, C, D, ns.mass_mode,
                           ns.m_reg, ns.m_jit, ns.mkind, (double*)ns.dinv, (double*)ns.dsq, (double*)ns.minv,
                           (double*)ns.mchol, ns.rn, (double*)ns.rmean, (double*)ns.rm2d, (double*)ns.rm2,
                           ns.updated, (double*)ns.mscratch);
      hipError_t e2 = hipGetLastError();
      if (e2 != hipSuccess) {
        set_error(std::string("mass update launch failed: ") + hipGetErrorString(e2));
        return GM_EHIP;
      }
      pending_refind = 1;
      refind_step = *step + (uint64_t)(start + nst - 1);
    }
    if (hook && *hook) {
      const int rc = (*hook)(start + nst);
      if (rc) return rc;
    }
  }
  ns.m += total;
  *step += (uint64_t)total + (step_mode ? 0 : 1);  // +1: the init draw consumed a counter value
  hipError_t e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    set_error(std::string("NUTS run failed: ") + hipGetErrorString(e));
    return GM_EHIP;
  }
  double tot = 0;
  for (long long i = 0; i < n_launch; ++i) {
    float t = 0;
    hipEventElapsedTime(&t, evs[2 * i], evs[2 * i + 1]);
    tot += t;
  }
  *ms = tot;
  *launches = n_launch;
  return GM_OK;
}

int nuts_get_step_size(NutsState& ns, gm_dtype dt, long long C, double* eps, double* eps_bar) {
  const size_t esz = dt == GM_F32 ? 4 : 8;
  std::vector<unsigned char> b1(C * esz), b2(C * esz);
  if (hipMemcpy(b1.data(), ns.eps, C * esz, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(b2.data(), ns.eps_bar, C * esz, hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("copy of NUTS step sizes failed");
    return GM_EHIP;
  }
  for (long long i = 0; i < C; ++i) {
    if (dt == GM_F32) {
      if (eps) eps[i] = ((float*)b1.data())[i];
      if (eps_bar) eps_bar[i] = ((float*)b2.data())[i];
    } else {
      if (eps) eps[i] = ((double*)b1.data())[i];
      if (eps_bar) eps_bar[i] = ((double*)b2.data())[i];
    }
  }
  return GM_OK;
}

int nuts_get_leapfrogs(NutsState& ns, long long C, long long* out) {
  if (hipMemcpy(out, ns.n_leapfrog, C * sizeof(long long), hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("copy of NUTS leapfrog counts failed");
    return GM_EHIP;
  }
  return GM_OK;
}

}  // namespace gm

