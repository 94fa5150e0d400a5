// mh_device.h — the Metropolis-Hastings transition kernel (device code
// only; compiled ahead of time by mh_kernels.hip and at run time for user
// targets by gm_jit.cpp).
#pragma once
#include "gm_device.h"
#include "gm_launch.h"
#include "gm_track.h"

namespace gm {

template <class T, int LPC, int E, class TG>
__global__ __launch_bounds__(256) void mh_kernel(MhLaunch a, TG tg_) {
  const long long gtid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long c = gtid / LPC;
  const int lane = (int)(gtid % LPC);
  const auto tg = tg_.template bind<LPC, E>(lane);  // per-lane target view
  // f64 proposals: the table-driven Box-Muller (gm_rng.h normals_tab); its
  // tables in LDS, filled by the whole block before any thread returns
  constexpr bool TAB = sizeof(T) == 8;
  __shared__ BmLds bm_lds[1];
  if constexpr (TAB) {
    bm_lds_fill(bm_lds[0]);
    __syncthreads();
  }
  if (c >= a.C) return;
  const int D = a.D;
  T* __restrict__ qs = (T*)a.q;
  const uint32_t cid = a.chain_offset + (uint32_t)c;
  // wave-uniform chain id when one chain fills the wave: the per-chain draws
  // (accept uniform) then run on the scalar unit
  const uint32_t ucid = (LPC == 64) ? (uint32_t)__builtin_amdgcn_readfirstlane((int)cid) : cid;
  const T sd = (T)a.prop_std;
  const T var = sd * sd;
  const T two_var = (T)2 * var;
  const DivConst<T> dq = DivConst<T>::make(two_var);  // div_by_const_q: the exact quotient by two_var
  const T pi = (T)3.14159265358979323846;
  const T qconst = (-(T)D * (T)0.5) * glog(((var * pi) * sd) * sd);
  // log alpha = (lp' + log q_b) - (lp + log q_f) (metropolis_hastings.rs:312)
  // with log q_b = log q_f = L, the same bits ((-d)^2 = d^2). Whenever L is
  // finite -- 2 var a normal number and the constant finite, so that every
  // d^2 / (2 var) is (|d| < 1e154) -- the engine takes lp' - lp: the same
  // value up to the rounding of the two sums with L (form 0 of the oracle;
  // tied to the reference text by tests/test_gpu_forms.py at cfg5's shape),
  // without the per-coordinate quotients and their reduction. Otherwise
  // (e.g. var = 0, where the reference's 0/0 rejects every proposal) the
  // full form.
  const bool cancel = __builtin_isnormal(two_var) && __builtin_isfinite(qconst);

  T x[E], y[E], gdummy[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    x[e] = (i < D) ? qs[c * D + i] : (T)0;
  }
  T lp = tg.template eval<LPC, E, true>(x, gdummy, lane);
  long long acc = 0;
  NormalCache<T> ncache[E];  // f32: msun Box-Muller
  UniformCache<T> ucache;
  uint64_t lblk = ~0ull;  // LPC == 64: the 64-step window whose accept logs lnl holds (lane k: step 64 lblk + k)
  T lnl = (T)0;
  const bool track = a.trk.mean != nullptr;  // run_progress (core.rs:146-163)
  ChainTrack<LPC, E> tr;
  if (track) tr.load(a.trk, c, lane, D);
  // one step from x given its proposal normals z (+0 in padded slots, whose
  // y = +0 + +0 * sd then stays +0)
  auto step = [&](int s, const T (&z)[E]) __attribute__((always_inline)) {
    const uint64_t st = a.step0 + (uint64_t)s;
#pragma unroll
    for (int e = 0; e < E; ++e) y[e] = x[e] + z[e] * sd;
    T lp1, log_alpha;
    if (cancel) {
      // the symmetric proposal's log q terms cancel (see above): the target's
      // sum alone
      lp1 = tg.finish(group_sum<LPC>(tg.template eval_part<LPC, E>(y, gdummy, lane)));
      log_alpha = lp1 - lp;
    } else {
      T ex[E];
      bool qbad = false;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        const T d = y[e] - x[e];
        // -(d*d) / two_var (distributions.rs:385), the IEEE quotient: its fast
        // form for every coordinate first (div_by_const_q), one range test for
        // the lane's E quotients, the IEEE division in a branch no wave meets
        // in practice
        ex[e] = (i < D) ? div_by_const_q(-(d * d), dq, qbad) : (T)0;
      }
      if (__builtin_expect(qbad, 0)) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = lane * E + e;
          const T d = y[e] - x[e];
          if (i < D) ex[e] = -(d * d) / two_var;
        }
      }
      T qpart = ex[0];
#pragma unroll
      for (int e = 1; e < E; ++e) qpart = qpart + ex[e];
      // the proposal density's sum and the target's, reduced together: the
      // same stages (and bits) as two group_sums, each stage's DPP latency
      // covered by the other sum instead of wait states
      T sums[2];
      sums[0] = qpart;
      sums[1] = tg.template eval_part<LPC, E>(y, gdummy, lane);
      group_sum_n<LPC>(sums);
      const T logq = sums[0] + qconst;
      lp1 = tg.finish(sums[1]);
      log_alpha = (lp1 + logq) - (lp + logq);
    }
    T lnu;
    if constexpr (LPC == 64) {
      // the accept log-uniforms of 64 consecutive steps in one VALU pass:
      // lane k evaluates ln u of step 64 m + k (its draw block and word), and
      // each step reads lane st % 64 back as a scalar
      constexpr int S = Blk<T>::S;
      const uint64_t b = st / 64;
      if (b != lblk) {
        const uint64_t sk = b * 64 + (uint64_t)lane;
        T us[S];
        uniforms_of(draw_block_v(a.seed, ucid, sk / S, TAG_MH_ACC, 0u), us);
        T um = us[0];
#pragma unroll
        for (int k = 1; k < S; ++k) um = ((lane & (S - 1)) == k) ? us[k] : um;
        lnl = glog_unif(um);
        lblk = b;
      }
      lnu = lane_k(lnl, (int)(st % 64));
    } else {
      lnu = glog_unif(ucache.get(a.seed, ucid, st, TAG_MH_ACC, 0u));
    }
    // (one chain per wave: a wave-uniform decision, so the accepted copy is
    // a scalar branch, not a select per register every step)
    const bool accept = log_alpha > lnu;
    if (LPC == 64 ? (__builtin_amdgcn_readfirstlane((int)accept) != 0) : accept) {
#pragma unroll
      for (int e = 0; e < E; ++e) x[e] = y[e];
      lp = lp1;
      ++acc;
    }
    if (track) tr.step(x, a.trk.n0 + (unsigned long long)s + 1ull, lane, D);
    if (s >= a.collect_from) {
      T* __restrict__ out = (T*)a.samples + ((a.sample_row0 + (s - a.collect_from)) * a.C + c) * D;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        if (i < D) out[i] = x[e];
      }
    }
  };
  if constexpr (TAB) {
    // f64: one Philox block and Box-Muller pair per coordinate serve the steps
    // st = 2b (z0) and 2b + 1 (z1); the loop takes the block's steps in turn,
    // so each step reads its normals without a select. The lane's E blocks and
    // pairs are issued side by side (draw_blocks_v, normals_tab_n): the E
    // coordinates' Philox and Box-Muller chains are independent, so one
    // chain's f64 latency is covered by the others' instructions (1.414e9 ->
    // 1.432e9 chain-steps/s against each coordinate's pair in its own branch,
    // profiles/r06/ab_mh_draw_forms.log).
    for (int s = 0; s < a.n_steps;) {
      const uint64_t st = a.step0 + (uint64_t)s;
      u32x4 w[E];
      double z0[E], z1[E];
      draw_blocks_v<E>(w, a.seed, cid, st / 2, TAG_MH_PROP, (uint32_t)(lane * E));
      normals_tab_n<E>(w, z0, z1, bm_lds[0]);
      if (D < LPC * E) {  // padded slots (wave-uniform): their normals +0
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const bool in = lane * E + e < D;
          z0[e] = in ? z0[e] : 0.0;
          z1[e] = in ? z1[e] : 0.0;
        }
      }
      if ((st & 1u) == 0) {
        step(s, z0);
        ++s;
      }
      if (s < a.n_steps) {
        step(s, z1);
        ++s;
      }
    }
  } else {
    for (int s = 0; s < a.n_steps; ++s) {
      const uint64_t st = a.step0 + (uint64_t)s;
      T z[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        z[e] = (i < D) ? ncache[e].get(a.seed, cid, st, TAG_MH_PROP, (uint32_t)i) : (T)0;
      }
      step(s, z);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    if (i < D) qs[c * D + i] = x[e];
  }
  if (track) tr.store(a.trk, c, lane, D);
  if (lane == 0) {
    ((T*)a.logp)[c] = lp;
    a.accepts[c] += acc;
  }
}

}  // namespace gm
