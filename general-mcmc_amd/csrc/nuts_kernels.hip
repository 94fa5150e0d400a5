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
#include <cstdlib>

#include "gm_layouts.h"
#include "gm_nuts.h"
#include "gm_track.h"

namespace gm {

struct NutsLaunch {
  void* q = nullptr;
  long long* accepts = nullptr;
  long long* n_leapfrog = nullptr;
  void* samples = nullptr;
  void* eps = nullptr;
  void* eps_bar = nullptr;
  void* h_bar = nullptr;
  void* mu = nullptr;
  void* stk_vec = nullptr;
  void* stk_alpha = nullptr;
  int* stk_n = nullptr;
  int* stk_na = nullptr;
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
  int* rn = nullptr;         // [C] RunningCov::n
  void* rmean = nullptr;     // [C][D]
  void* rm2d = nullptr;      // [C][D]
  void* rm2 = nullptr;       // [C][D][D] (upper triangle used)
  int* updated = nullptr;    // [C] metric replaced at the previous launch's last step
  // levels k < lds_levels of the subtree stack live in LDS (after the
  // target's staging area, at byte offset lds_stack_off), the rest in HBM
  int lds_levels = 0;
  unsigned lds_stack_off = 0;
  long long sb = 0, eb = 0;  // start_buffer, end_buffer (should_collect, :153-162)
  int do_refind = 0;         // re-find eps for updated chains first (:905-918)
  uint64_t refind_step = 0;  // transition index of the update (probe draws)
};

// coordinate j of a chain's vector: lane j/E of the group, slot j%E
template <int LPC, int E, class T>
__device__ __forceinline__ T coord(const T (&x)[E], int j) {
  const int src = j / E, slot = j % E;
  T mine = x[0];
#pragma unroll
  for (int e = 1; e < E; ++e) mine = (slot == e) ? x[e] : mine;
  if constexpr (LPC == 1) return mine;
  else return __shfl(mine, src, LPC);
}

// MassMatrix (generic_nuts.rs:175-304) of one chain, this lane's view
template <class T, int E> struct MassDev {
  int kind = 0;             // 0 identity, 1 diagonal, 2 dense
  T inv[E], sq[E];          // diagonal
  const T* minv = nullptr;  // dense [D][D]
  const T* chol = nullptr;
  int D = 0;
};

// inv_mul (:255-273): v = M^-1 p
template <int LPC, int E, class T>
__device__ __forceinline__ void inv_mul(const MassDev<T, E>& M, const T (&p)[E], T (&v)[E], int lane) {
  if (M.kind == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = M.inv[e] * p[e];
  } else if (M.kind == 2) {
    T acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = (T)0;
    for (int j = 0; j < M.D; ++j) {
      const T pj = coord<LPC, E>(p, j);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        if (i < M.D) acc[e] = acc[e] + M.minv[(long long)i * M.D + j] * pj;
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = acc[e];
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = p[e];
  }
}

// sample_momentum (:275-303) applied to standard normals z
template <int LPC, int E, class T>
__device__ __forceinline__ void momentum_from(const MassDev<T, E>& M, const T (&z)[E], T (&p)[E], int lane) {
  if (M.kind == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) p[e] = z[e] * M.sq[e];
  } else if (M.kind == 2) {
    T acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = (T)0;
    for (int j = 0; j < M.D; ++j) {
      const T zj = coord<LPC, E>(z, j);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        if (i < M.D && j <= i) acc[e] = acc[e] + M.chol[(long long)i * M.D + j] * zj;
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) p[e] = acc[e];
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) p[e] = z[e];
  }
}

template <int LPC, int E, class T>
__device__ __forceinline__ T dot_group(const T (&a)[E], const T (&b)[E]) {
  T part = a[0] * b[0];
#pragma unroll
  for (int e = 1; e < E; ++e) part = part + a[e] * b[e];
  return group_sum<LPC>(part);
}

// MassMatrix::kinetic, identity (generic_nuts.rs:230-238): 0.5 * sum p^2
template <int LPC, int E, class T>
__device__ __forceinline__ T kinetic(const T (&p)[E]) {
  return (T)0.5 * dot_group<LPC, E>(p, p);
}

// leapfrog_with_mass, identity (generic_nuts.rs:1396-1418)
template <int LPC, int E, class T, class TG>
__device__ __forceinline__ T leapfrog(const TG& tg, T (&q)[E], T (&p)[E], T (&g)[E], T epsv, int lane) {
  const T h = epsv * (T)0.5;
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = p[e] + g[e] * h;
#pragma unroll
  for (int e = 0; e < E; ++e) q[e] = q[e] + p[e] * epsv;
  const T lp = tg.template eval<LPC, E, true>(q, g, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = p[e] + g[e] * h;
  return lp;
}

// stop_criterion (generic_nuts.rs:1354-1378), identity mass:
// (q+ - q-) . p- >= 0  and  (q+ - q-) . p+ >= 0
template <int LPC, int E, class T>
__device__ __forceinline__ bool no_uturn(const T (&qm)[E], const T (&qp)[E], const T (&pm)[E],
                                         const T (&pp)[E]) {
  T d[E];
#pragma unroll
  for (int e = 0; e < E; ++e) d[e] = qp[e] - qm[e];
  const T dm = dot_group<LPC, E>(d, pm);
  const T dp = dot_group<LPC, E>(d, pp);
  return dm >= (T)0 && dp >= (T)0;
}

// MassMatrix::kinetic (:226-253), canonical-order sum of the per-coordinate
// terms p*p*inv (diagonal) or p_i (M^-1 p)_i (dense)
template <int LPC, int E, class T>
__device__ __forceinline__ T kinetic_m(const MassDev<T, E>& M, const T (&p)[E], int lane) {
  if (M.kind == 0) return kinetic<LPC, E>(p);
  T t[E];
  if (M.kind == 1) {
#pragma unroll
    for (int e = 0; e < E; ++e) t[e] = p[e] * p[e] * M.inv[e];
  } else {
    inv_mul<LPC, E>(M, p, t, lane);
#pragma unroll
    for (int e = 0; e < E; ++e) t[e] = p[e] * t[e];
  }
  T part = t[0];
#pragma unroll
  for (int e = 1; e < E; ++e) part = part + t[e];
  return (T)0.5 * group_sum<LPC>(part);
}

// leapfrog_with_mass (:1396-1418): drift by M^-1 p
template <int LPC, int E, class T, class TG>
__device__ __forceinline__ T leapfrog_m(const TG& tg, const MassDev<T, E>& M, T (&q)[E], T (&p)[E],
                                        T (&g)[E], T epsv, int lane) {
  if (M.kind == 0) return leapfrog<LPC, E>(tg, q, p, g, epsv, lane);
  const T h = epsv * (T)0.5;
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = p[e] + g[e] * h;
  T v[E];
  inv_mul<LPC, E>(M, p, v, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) q[e] = q[e] + v[e] * epsv;
  const T lp = tg.template eval<LPC, E, true>(q, g, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) p[e] = p[e] + g[e] * h;
  return lp;
}

// stop_criterion_with_mass (:1354-1378), the top-level U-turn
template <int LPC, int E, class T>
__device__ __forceinline__ bool no_uturn_m(const MassDev<T, E>& M, const T (&qm)[E], const T (&qp)[E],
                                           const T (&pm)[E], const T (&pp)[E], int lane) {
  if (M.kind == 0) return no_uturn<LPC, E>(qm, qp, pm, pp);
  T d[E], vm[E], vp[E];
#pragma unroll
  for (int e = 0; e < E; ++e) d[e] = qp[e] - qm[e];
  inv_mul<LPC, E>(M, pm, vm, lane);
  inv_mul<LPC, E>(M, pp, vp, lane);
  const T dm = dot_group<LPC, E>(d, vm);
  const T dp = dot_group<LPC, E>(d, vp);
  return dm >= (T)0 && dp >= (T)0;
}

template <int LPC, class T>
__device__ __forceinline__ bool all_finite(const T (&x)[1]) { return true; }

template <int LPC, int E, class T>
__device__ __forceinline__ bool group_all_finite(const T (&x)[E], int lane, int D) {
  int bad = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    const T v = x[e];
    if (i < D && !(v - v == (T)0)) bad = 1;  // inf - inf and NaN - NaN are NaN
  }
  return group_sum<LPC>(bad) == 0;
}

template <class T> __device__ __forceinline__ T rust_min1(T x) {  // T::one().min(x)
  if (x != x) return (T)1;
  return x < (T)1 ? x : (T)1;
}

template <class T> struct MachEps;
template <> struct MachEps<float> { static constexpr float v = 1.1920928955078125e-07f; };
template <> struct MachEps<double> { static constexpr double v = 2.220446049250313e-16; };

// find_reasonable_epsilon_with_mass (generic_nuts.rs:1025-1102), identity mass.
template <int LPC, int E, class T, class TG>
__device__ T find_reasonable_epsilon(const TG& tg, const T (&q0)[E], const T (&p0)[E], int lane, int D) {
  const T half = (T)0.5;
  T eps = (T)1;
  T g0[E];
  const T ulogp = tg.template eval<LPC, E, true>(q0, g0, lane);
  T q[E], p[E], g[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { q[e] = q0[e]; p[e] = p0[e]; g[e] = g0[e]; }
  T ulogp1 = leapfrog<LPC, E>(tg, q, p, g, eps, lane);
  T k = (T)1;
  for (int it = 0; it < 1100; ++it) {  // bounded: k underflows to 0 long before
    const bool fin = (ulogp1 - ulogp1 == (T)0) && group_all_finite<LPC, E>(g, lane, D);
    if (fin) break;
    k = k * half;
#pragma unroll
    for (int e = 0; e < E; ++e) { q[e] = q0[e]; p[e] = p0[e]; g[e] = g0[e]; }
    ulogp1 = leapfrog<LPC, E>(tg, q, p, g, eps * k, lane);
  }
  eps = half * k * eps;
  const T k0 = kinetic<LPC, E>(p0);
  T la = ulogp1 - ulogp - (kinetic<LPC, E>(p) - k0);
  const T a = (la > glog(half)) ? (T)1 : (T)-1;
  const T ln2 = glog((T)2);
  for (int it = 0; it < 2200; ++it) {  // bounded (the reference is not)
    if (!(a * la > -a * ln2)) break;
    eps = eps * (a > (T)0 ? (T)2 : (T)0.5);  // 2^a, a = +-1
#pragma unroll
    for (int e = 0; e < E; ++e) { q[e] = q0[e]; p[e] = p0[e]; g[e] = g0[e]; }
    ulogp1 = leapfrog<LPC, E>(tg, q, p, g, eps, lane);
    la = ulogp1 - ulogp - (kinetic<LPC, E>(p) - k0);
  }
  return eps;
}

template <class T, int LPC, int E, class TG>
__global__ __launch_bounds__(256) void nuts_kernel(NutsLaunch a, TG tg_) {
  const long long gtid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long c = gtid / LPC;
  const int lane = (int)(gtid % LPC);
  const auto tg = tg_.template bind<LPC, E>(lane);  // per-lane target view
  if (c >= a.C) return;
  const int D = a.D;
  const long long C = a.C;
  const uint32_t cid = a.chain_offset + (uint32_t)c;
  T* __restrict__ qs = (T*)a.q;
  T* __restrict__ svec = (T*)a.stk_vec;
  T* __restrict__ salpha = (T*)a.stk_alpha;
  const long long slane = c * LPC + lane;  // scalar-stack slot of this lane
  const long long CL = C * LPC;
  // Subtree stack. Level k < KL: LDS, [k][field][thread*E + e] vectors and
  // [k][thread] scalars of this block (a lane reads back only what it wrote:
  // no synchronisation). Deeper levels: HBM [k][field][chain][coord].
  constexpr int NT = 256;  // threads per block (launch_nuts)
  const int KL = a.lds_levels;
  T* __restrict__ lvec = (T*)(gm_dyn_lds + a.lds_stack_off);
  T* __restrict__ lalpha = lvec + (long long)KL * 3 * NT * E;
  int* __restrict__ lnn = (int*)(lalpha + KL * NT);
  int* __restrict__ lnna = lnn + KL * NT;
  const int tix = threadIdx.x;
  auto stack_store = [&](int k, const T (&f0)[E], const T (&f1)[E], const T (&f2)[E], T al, int nn,
                         int nna) __attribute__((always_inline)) {
    if (k < KL) {
      T* v = lvec + (long long)k * 3 * NT * E + tix * E;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        v[e] = f0[e];
        v[NT * E + e] = f1[e];
        v[2 * NT * E + e] = f2[e];
      }
      lalpha[k * NT + tix] = al;
      lnn[k * NT + tix] = nn;
      lnna[k * NT + tix] = nna;
    } else {
      T* sv = svec + ((long long)(k * 3) * C + c) * D;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        if (i < D) {
          sv[i] = f0[e];
          sv[C * D + i] = f1[e];
          sv[2 * C * D + i] = f2[e];
        }
      }
      salpha[k * CL + slane] = al;
      a.stk_n[k * CL + slane] = nn;
      a.stk_na[k * CL + slane] = nna;
    }
  };
  // field f (0 first q, 1 first p, 2 proposal) of level k
  auto stack_vec = [&](int k, int f, T (&out)[E]) __attribute__((always_inline)) {
    if (k < KL) {
      const T* v = lvec + ((long long)k * 3 + f) * NT * E + tix * E;
#pragma unroll
      for (int e = 0; e < E; ++e) out[e] = v[e];
    } else {
      const T* sv = svec + ((long long)(k * 3 + f) * C + c) * D;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        out[e] = (i < D) ? sv[i] : (T)0;
      }
    }
  };
  auto stack_scalars = [&](int k, T& al, long long& nn, long long& nna) __attribute__((always_inline)) {
    if (k < KL) {
      al = lalpha[k * NT + tix];
      nn = lnn[k * NT + tix];
      nna = lnna[k * NT + tix];
    } else {
      al = salpha[k * CL + slane];
      nn = a.stk_n[k * CL + slane];
      nna = a.stk_na[k * CL + slane];
    }
  };

  T q[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    q[e] = (i < D) ? qs[c * D + i] : (T)0;
  }
  T eps = ((T*)a.eps)[c], eps_bar = ((T*)a.eps_bar)[c], h_bar = ((T*)a.h_bar)[c], mu = ((T*)a.mu)[c];
  const T gamma = (T)0.05, kappa = (T)0.75, delta = (T)a.target_accept;
  const long long t0c = 10;

  // the chain's metric and warm-up statistics (generic_nuts.rs:33-359)
  MassDev<T, E> M;
  M.D = D;
  int rn = 0;
  T rmean[E], rm2d[E];
  if (a.mass_mode) {
    M.kind = a.mkind[c];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      M.inv[e] = (i < D) ? ((const T*)a.dinv)[c * D + i] : (T)0;
      M.sq[e] = (i < D) ? ((const T*)a.dsq)[c * D + i] : (T)0;
      rmean[e] = (i < D) ? ((const T*)a.rmean)[c * D + i] : (T)0;
      rm2d[e] = (i < D) ? ((const T*)a.rm2d)[c * D + i] : (T)0;
    }
    if (a.mass_mode == 2) {
      M.minv = (const T*)a.minv + (long long)c * D * D;
      M.chol = (const T*)a.mchol + (long long)c * D * D;
    }
    rn = a.rn[c];
  }

  if (a.do_init) {  // init_chain_state (generic_nuts.rs:731-753)
    T z[E], p0[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      z[e] = (i < D) ? normal<T>(a.seed, cid, a.init_step, TAG_NUTS_INIT, (uint32_t)i) : (T)0;
    }
    momentum_from<LPC, E>(M, z, p0, lane);
    const T ae = eps + (T)1;
    if ((ae < (T)0 ? -ae : ae) <= MachEps<T>::v) eps = find_reasonable_epsilon<LPC, E>(tg, q, p0, lane, D);
    mu = glog((T)10 * eps);
  }
  if (a.do_refind && a.updated[c]) {  // after a metric update (generic_nuts.rs:905-918)
    T z[E], probe[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      z[e] = (i < D) ? normal<T>(a.seed, cid, a.refind_step, TAG_NUTS_PROBE, (uint32_t)i) : (T)0;
    }
    momentum_from<LPC, E>(M, z, probe, lane);
    eps = find_reasonable_epsilon<LPC, E>(tg, q, probe, lane, D);  // identity-mass leapfrog (:1009-1023)
    mu = glog((T)10 * eps);
    eps_bar = eps;
    h_bar = (T)0;
  }
  auto record = [&](long long t) {
    const long long row = t - a.row_shift;
    if (row >= 0 && row < a.n_rows) {
      T* __restrict__ out = (T*)a.samples + (row * C + c) * D;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        if (i < D) out[i] = q[e];
      }
    }
  };
  if (a.t0 == 0) record(0);

  long long acc = 0, nlf = 0;
  NormalCache<T> ncache[E];
  const bool track = a.trk.mean != nullptr;  // run_progress (generic_nuts.rs:688-704)
  ChainTrack<LPC, E> tr;
  if (track) tr.load(a.trk, c, lane, D);
  for (int s = 0; s < a.n_steps; ++s) {
    const uint64_t st = a.step0 + (uint64_t)s;
    const long long m = a.m0 + s + 1;
    // --- momentum, slice (generic_nuts.rs:758-768)
    T p0[E], g0[E];
    {
      T z[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        z[e] = (i < D) ? ncache[e].get(a.seed, cid, st, TAG_NUTS_MOM, (uint32_t)i) : (T)0;
      }
      momentum_from<LPC, E>(M, z, p0, lane);
    }
    const T logp0 = tg.template eval<LPC, E, true>(q, g0, lane);
    const T joint0 = logp0 - kinetic_m<LPC, E>(M, p0, lane);
    const T logu = joint0 - exp1<T>(a.seed, cid, st, TAG_NUTS_EXP, 0u);
    // trajectory ends
    T qm[E], pm[E], gm_[E], qp[E], pp[E], gp[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      qm[e] = q[e]; qp[e] = q[e];
      pm[e] = p0[e]; pp[e] = p0[e];
      gm_[e] = g0[e]; gp[e] = g0[e];
    }
    long long n = 1;
    bool s_ok = true;
    T alpha = (T)0;
    long long n_alpha = 0;
    uint32_t merge_ctr = 0;
    int j = 0;
    while (s_ok && j < a.max_depth) {
      const T u1 = uniform_co<T>(a.seed, cid, st, TAG_NUTS_DIR, (uint32_t)j);
      const int v = (u1 < (T)0.5) ? 1 : -1;
      const T epsv = (T)v * eps;
      // edge state = the trajectory end on side v
      T qe[E], pe[E], ge[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        qe[e] = v > 0 ? qp[e] : qm[e];
        pe[e] = v > 0 ? pp[e] : pm[e];
        ge[e] = v > 0 ? gp[e] : gm_[e];
      }
      // current subtree T
      T fq[E], fp[E], pr[E];
      long long tn = 0;
      bool ts = true;
      T ta = (T)0;
      long long tna = 0;
      const long long nleaves = 1LL << j;
      for (long long l = 0; l < nleaves; ++l) {
        const T lp = leapfrog_m<LPC, E>(tg, M, qe, pe, ge, epsv, lane);
        ++nlf;
        const T joint = lp - kinetic_m<LPC, E>(M, pe, lane);
        tn = (logu < joint) ? 1 : 0;
        ts = (logu - (T)1000) < joint;
        ta = rust_min1(gexp(joint - joint0));
        tna = 1;
#pragma unroll
        for (int e = 0; e < E; ++e) { fq[e] = qe[e]; fp[e] = pe[e]; pr[e] = qe[e]; }
        bool done = false;
        int k = 0;
        while (true) {
          if (k == j) { done = true; break; }
          if (((l >> k) & 1) == 0) {  // left child at level k
            // A truncated left subtree: its parent builds no right half and
            // returns it unchanged; going up, it is merged wherever that
            // parent is itself a right child (the recursion's post-order).
            if (!ts) { ++k; continue; }
            stack_store(k, fq, fp, pr, ta, (int)tn, (int)tna);
            break;
          }
          // right child: merge with the stored left sibling (generic_nuts.rs:1251-1323)
          T lq[E], lpv[E];
          stack_vec(k, 0, lq);
          stack_vec(k, 1, lpv);
          long long ln_, lna;
          T lal;
          stack_scalars(k, lal, ln_, lna);
          const double u = uniform_co<double>(a.seed, cid, st, TAG_NUTS_MRG, merge_ctr++);
          const long long den = (ln_ + tn) > 1 ? (ln_ + tn) : 1;
          if (!(u < (double)tn / (double)den)) stack_vec(k, 2, pr);
          tn = ln_ + tn;
          if (ts) ts = (v > 0) ? no_uturn<LPC, E>(lq, qe, lpv, pe) : no_uturn<LPC, E>(qe, lq, pe, lpv);
          ta = lal + ta;
          tna = lna + tna;
#pragma unroll
          for (int e = 0; e < E; ++e) { fq[e] = lq[e]; fp[e] = lpv[e]; }
          ++k;
        }
        if (done) break;
      }
      // the new trajectory end on side v is the last leaf integrated
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (v > 0) { qp[e] = qe[e]; pp[e] = pe[e]; gp[e] = ge[e]; }
        else { qm[e] = qe[e]; pm[e] = pe[e]; gm_[e] = ge[e]; }
      }
      alpha = ta;
      n_alpha = tna;
      const T tmp = rust_min1((T)tn / (T)n);
      const T u2 = uniform_co<T>(a.seed, cid, st, TAG_NUTS_TOP, (uint32_t)j);
      if (ts && (u2 < tmp)) {
#pragma unroll
        for (int e = 0; e < E; ++e) q[e] = pr[e];
        ++acc;
      }
      n += tn;
      s_ok = ts && no_uturn_m<LPC, E>(M, qm, qp, pm, pp, lane);
      ++j;
    }
    // dual averaging (generic_nuts.rs:882-924)
    T eta = (T)1 / (T)(m + t0c);
    h_bar = ((T)1 - eta) * h_bar + eta * (delta - alpha / (T)n_alpha);
    if (m <= a.n_discard) {
      const T mf = (T)m;
      eps = gexp(mu - gsqrt(mf) / gamma * h_bar);
      eta = gexp(-kappa * glog(mf));  // m^(-kappa)
      eps_bar = gexp(((T)1 - eta) * glog(eps_bar) + eta * glog(eps));
      // RunningCov::update inside the collection window (:897-903, 108-129)
      const long long lim = a.n_discard > a.eb ? a.n_discard - a.eb : 0;
      if (a.mass_mode && m > a.sb && m < lim) {
        rn += 1;
        const T ns = (T)rn;
        T d1[E], d2[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          d1[e] = q[e] - rmean[e];
          rmean[e] = rmean[e] + d1[e] / ns;
          d2[e] = q[e] - rmean[e];
          rm2d[e] = rm2d[e] + d1[e] * d2[e];
        }
        if (a.mass_mode == 2) {
          T* m2 = (T*)a.rm2 + (long long)c * D * D;
          for (int jj = 0; jj < D; ++jj) {
            const T dj = coord<LPC, E>(d2, jj);
#pragma unroll
            for (int e = 0; e < E; ++e) {
              const int i = lane * E + e;
              if (i < D && jj >= i) m2[(long long)i * D + jj] = m2[(long long)i * D + jj] + d1[e] * dj;
            }
          }
        }
      }
    } else {
      eps = eps_bar;
    }
    if (track) tr.step(q, a.trk.n0 + (unsigned long long)s + 1ull, lane, D);
    record(a.t0 + s + 1);
  }
  if (track) tr.store(a.trk, c, lane, D);
  if (a.mass_mode) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      if (i < D) {
        ((T*)a.rmean)[c * D + i] = rmean[e];
        ((T*)a.rm2d)[c * D + i] = rm2d[e];
      }
    }
    if (lane == 0) a.rn[c] = rn;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    if (i < D) qs[c * D + i] = q[e];
  }
  if (lane == 0) {
    ((T*)a.eps)[c] = eps;
    ((T*)a.eps_bar)[c] = eps_bar;
    ((T*)a.h_bar)[c] = h_bar;
    ((T*)a.mu)[c] = mu;
    a.accepts[c] += acc;
    a.n_leapfrog[c] += nlf;
  }
}

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

template <class T>
__global__ void nuts_fill_kernel(T* eps, T* eps_bar, T* h_bar, T* mu, long long C) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C) return;
  eps[i] = (T)-1;                   // generic_nuts.rs:619
  eps_bar[i] = (T)1;                // :645
  h_bar[i] = (T)0;                  // :646
  mu[i] = glog((T)10 * (T)1);       // :644
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
  if (e == hipSuccess && max_depth > 0)
    e = hipMalloc(&ns->stk_vec, (size_t)max_depth * 3 * C * D * esz);
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
    if (e == hipSuccess) e = hipMalloc(&ns->mchol, cdd);
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
    hipMemset(ns->mchol, 0, cdd);
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
  ffree(ns->stk_alpha);
  ffree(ns->stk_n);
  ffree(ns->stk_na);
  ffree(ns->n_leapfrog);
  *ns = NutsState();
}

int nuts_run(NutsState& ns, gm_dtype dt, const TargetDev& tg, const Layout& lay, void* q,
             long long* accepts, void* samples, long long C, int D, double target_accept,
             uint64_t seed, uint64_t* step, uint32_t chain_offset, long long total,
             long long n_discard, int progress, long long steps_per_launch, hipStream_t st,
             std::vector<hipEvent_t>& evs, double* ms, long long* launches, const TrackLaunch* trk,
             const StepHook* hook) {
  const size_t esz = dt == GM_F32 ? 4 : 8;
  // scalar stack is per lane; (re)size for the current layout
  const long long lanes_total = C * lay.lanes;
  if (ns.stk_lanes != lanes_total && ns.max_depth > 0) {
    ffree(ns.stk_alpha);
    ffree(ns.stk_n);
    ffree(ns.stk_na);
    ns.stk_alpha = nullptr;
    ns.stk_n = ns.stk_na = nullptr;
    hipError_t e = hipMalloc(&ns.stk_alpha, (size_t)ns.max_depth * lanes_total * esz);
    if (e == hipSuccess) e = hipMalloc((void**)&ns.stk_n, (size_t)ns.max_depth * lanes_total * sizeof(int));
    if (e == hipSuccess) e = hipMalloc((void**)&ns.stk_na, (size_t)ns.max_depth * lanes_total * sizeof(int));
    if (e != hipSuccess) {
      set_error("NUTS stack allocation failed");
      return GM_ENOMEM;
    }
    ns.stk_lanes = lanes_total;
  }
  // init_chain_state at the start of every run (generic_nuts.rs:731-753)
  ns.m = 0;
  ns.n_discard = n_discard;
  const uint64_t init_step = *step;
  const long long n_rows_total = progress ? total - n_discard : total - n_discard + 1;
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
    if (ns.mass_mode) {
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
  if (ns.mass_mode) {  // RunningCov::reset in init_chain_state (:744-746)
    hipMemsetAsync(ns.rn, 0, C * sizeof(int), st);
    hipMemsetAsync(ns.rmean, 0, (size_t)C * D * esz, st);
    hipMemsetAsync(ns.rm2d, 0, (size_t)C * D * esz, st);
    if (ns.mass_mode == 2) hipMemsetAsync(ns.rm2, 0, (size_t)C * D * D * esz, st);
    hipMemsetAsync(ns.updated, 0, C * sizeof(int), st);
  }
  int pending_refind = 0;
  uint64_t refind_step = 0;
  // GM_NUTS_LDS_LEVELS caps the LDS stack levels (tests cover both homes)
  const char* cap_env = getenv("GM_NUTS_LDS_LEVELS");
  const long long lds_cap = cap_env ? atoll(cap_env) : -1;
  int ncu = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1)
      ncu = 256;
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
    a.stk_alpha = ns.stk_alpha;
    a.stk_n = ns.stk_n;
    a.stk_na = ns.stk_na;
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
    a.n_discard = n_discard;
    a.do_init = (start == 0 && li == 0) ? 1 : 0;
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
      a.rn = ns.rn;
      a.rmean = ns.rmean;
      a.rm2d = ns.rm2d;
      a.rm2 = ns.rm2;
      a.updated = ns.updated;
      a.sb = ns.m_sb;
      a.eb = ns.m_eb;
      a.do_refind = pending_refind;
      a.refind_step = refind_step;
    }
    if (trk) {
      a.trk = *trk;
      a.trk.n0 = trk->n0 + (unsigned long long)start;
    }
    hipEventRecord(evs[2 * li], st);
    hipError_t e = dispatch(dt, tg, lay, [&]<class T, int LPC, int E, class TG>(TG t) -> hipError_t {
      const long long threads = C * LPC;
      const unsigned blocks = (unsigned)((threads + 255) / 256);
      // LDS: the target's staging area, then as many subtree-stack levels as
      // fit without costing occupancy (<= 4 blocks of 4 waves per CU by VGPRs)
      const size_t tgl = (t.template lds_bytes<LPC, E>() + 15) / 16 * 16;
      const size_t per_level = (size_t)3 * 256 * E * sizeof(T) + (size_t)256 * (sizeof(T) + 8);
      long long bpc = ((long long)blocks + ncu - 1) / ncu;
      bpc = bpc < 1 ? 1 : bpc > 4 ? 4 : bpc;
      size_t budget = (size_t)(160 * 1024) / (size_t)bpc - 1024;
      if (budget > 64 * 1024) budget = 64 * 1024;
      long long kl = budget > tgl ? (long long)((budget - tgl) / per_level) : 0;
      if (kl > a.max_depth) kl = a.max_depth;
      if (lds_cap >= 0 && kl > lds_cap) kl = lds_cap;
      a.lds_levels = (int)kl;
      a.lds_stack_off = (unsigned)tgl;
      const size_t lds = tgl + (size_t)kl * per_level;
      hipLaunchKernelGGL((nuts_kernel<T, LPC, E, TG>), dim3(blocks), dim3(256), lds, st, a, t);
      return hipGetLastError();
    });
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
  *step += (uint64_t)total + 1;  // +1: the init draw consumed a counter value
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
