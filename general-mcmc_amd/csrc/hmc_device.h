// hmc_device.h — the HMC transition kernels (device code only; compiled
// ahead of time by hmc_kernels.hip and at run time for user targets by
// gm_jit.cpp). See hmc_kernels.hip for the algorithm notes.
#pragma once
#include "gm_device.h"
#include "gm_launch.h"

namespace gm {

template <class T, int LPC, int E, class TG>
__global__ __launch_bounds__(256) void hmc_kernel(HmcLaunch a, TG tg_) {
  const long long gtid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long c = gtid / LPC;
  const int lane = (int)(gtid % LPC);
  const auto tg = tg_.template bind<LPC, E>(lane);  // per-lane target view
  // f32 momenta: the table-driven Box-Muller (gm_rng.h normals_tab32); its
  // tables in LDS, filled by the whole block before any thread returns
  __shared__ BmLds32 bm32[1];
  if constexpr (sizeof(T) == 4) {
    bm_lds_fill32(bm32[0]);
    __syncthreads();
  }
  if (c >= a.C) return;  // whole lane groups leave together
  const int D = a.D;
  T* __restrict__ qs = (T*)a.q;
  const T eps = (T)a.eps;
  const T half = (T)0.5 * eps;  // batched_hmc.rs:167
  const uint32_t cid = a.chain_offset + (uint32_t)c;
  // wave-uniform chain id when one chain fills the wave: the per-chain draws
  // (accept uniform) then run on the scalar unit
  const uint32_t ucid = (LPC == 64) ? (uint32_t)__builtin_amdgcn_readfirstlane((int)cid) : cid;

  T q[E], g[E], p[E], q1[E], p1[E], g1[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    q[e] = (i < D) ? qs[c * D + i] : (T)0;
  }
  T lp = tg.template eval<LPC, E, true>(q, g, lane);
  long long acc = 0;
  constexpr int S = Blk<T>::S;  // one Philox block serves S transitions
  const PhiloxKeys pk = philox_keys(a.seed);  // momentum streams' round keys, in VGPRs
  // Draw blocks: A = the current block (front = this step), B = the next
  // one, prefetched. Each wave prefetches on the step whose index matches its
  // wave phase, so the waves of a SIMD are not all in the Philox/Box-Muller
  // chain at once and the leapfrogs of the others hide its latency.
  T zsA[E][S], kesA[S], lusA[S];
  T zsB[E][S], kesB[S], lusB[S];
  bool hasB = false;
  const int phase = (int)((gtid >> 6) % S);  // wave index mod S (wave-uniform)
  // the momenta of block blk, their S kinetic energies (S independent
  // reductions) and the S accept log-uniforms
  auto fill = [&](T (&zs)[E][S], T (&kes)[S], T (&lus)[S], uint64_t blk) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      momenta_of(draw_block(pk, cid, blk, TAG_MOM, (uint32_t)i), zs[e], bm32[0]);
#pragma unroll
      for (int k = 0; k < S; ++k) zs[e][k] = (i < D) ? zs[e][k] : (T)0;
    }
    T kp[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const T sq = zs[e][k] * zs[e][k];
        kp[k] = (e == 0) ? sq : kp[k] + sq;
      }
    }
    group_sum_n<LPC>(kp);  // 2. kinetic energies, the S sums interleaved
#pragma unroll
    for (int k = 0; k < S; ++k) kes[k] = kp[k] * (T)0.5;
    T us[S];
    uniforms_of(draw_block(a.seed, ucid, blk, TAG_ACC, 0u), us);
    if constexpr (LPC == 64) {
      // the S logs of wave-uniform inputs: lane k evaluates ln u_k, one
      // VALU pass for all S, then each value is read back as a scalar
      T um = us[0];
#pragma unroll
      for (int k = 1; k < S; ++k) um = ((lane & (S - 1)) == k) ? us[k] : um;
      const T lm = glog_unif(um);
#pragma unroll
      for (int k = 0; k < S; ++k) lus[k] = lane_k(lm, k);
    } else {
#pragma unroll
      for (int k = 0; k < S; ++k) lus[k] = glog_unif(us[k]);
    }
  };
  const uint64_t st_end = a.step0 + (uint64_t)a.n_steps;
  // this lane's first sample slot; each stored transition advances it one row
  // (C*D elements) instead of recomputing the 64-bit row address
  T* __restrict__ out = (T*)a.samples + (a.sample_row0 * a.C + c) * D + lane * E;
  const long long row_stride = a.C * D;

  for (int s = 0; s < a.n_steps; ++s) {
    const uint64_t st = a.step0 + (uint64_t)s;
    const int k0 = (int)(st % S);
    if (s == 0 || k0 == 0) {
      if (s > 0 && hasB) {
#pragma unroll
        for (int k = 0; k < S; ++k) {
#pragma unroll
          for (int e = 0; e < E; ++e) zsA[e][k] = zsB[e][k];
          kesA[k] = kesB[k];
          lusA[k] = lusB[k];
        }
      } else {
        fill(zsA, kesA, lusA, st / S);
#pragma unroll
        for (int e = 0; e < E; ++e) skip_front(zsA[e], k0);
        skip_front(kesA, k0);
        skip_front(lusA, k0);
      }
      hasB = false;
    }
    // 1. momentum ~ N(0, I) and its kinetic energy: front of the block
#pragma unroll
    for (int e = 0; e < E; ++e) {
      p[e] = zsA[e][0];
      shift_front(zsA[e]);
    }
    const T ke0 = kesA[0];
    const T lnu = lusA[0];
    shift_front(kesA);
    shift_front(lusA);
    // prefetch the next block (if this launch reaches it)
    if (!hasB && k0 == phase && st - (uint64_t)k0 + S < st_end) {
      fill(zsB, kesB, lusB, st / S + 1);
      hasB = true;
    }
    // 4. proposal buffers
#pragma unroll
    for (int e = 0; e < E; ++e) {
      q1[e] = q[e];
      p1[e] = p[e];
      g1[e] = g[e];
    }
    // 5. leapfrog: L-1 gradient-only steps, then the last one with logp.
    // The kicks p + g*(eps/2) and the drift q + p*eps are the engine's fused
    // multiply-adds (one rounding each; the reference's tensor ops round the
    // product and the sum separately, batched_hmc.rs:166-190): 9 VALU per
    // 64-lane Rosenbrock leapfrog instead of 11 (+9 % headline,
    // profiles/r04/ab_hmc_fma_kick_drift.log); the oracle's engine form is
    // the same (gm_oracle_t.inc hmc_chains, form 0).
    T lp1 = lp;
    // (unrolled by hand: the DPP intrinsics are convergent, so the compiler
    // will not runtime-unroll, and a taken branch costs a wave ~20 cycles)
    auto lf = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < E; ++e) p1[e] = gfma(g1[e], half, p1[e]);
#pragma unroll
      for (int e = 0; e < E; ++e) q1[e] = gfma(p1[e], eps, q1[e]);
      tg.template eval<LPC, E, false>(q1, g1, lane);
#pragma unroll
      for (int e = 0; e < E; ++e) p1[e] = gfma(g1[e], half, p1[e]);
    };
    int l = 0;
    if (a.lf_unroll == 4)
      for (; l + 4 < a.L; l += 4) { lf(); lf(); lf(); lf(); }
    // two leapfrogs per loop trip at 2-4 waves per SIMD (one taken branch and
    // loop test per two): kernel -1.4 % at the headline's 4 waves per SIMD,
    // but cfg4 at 8 waves per SIMD -4.7 % (profiles/r04/ab_hmc_unroll2.log)
    if (a.lf_unroll == 2)
      for (; l + 2 < a.L; l += 2) { lf(); lf(); }
    for (; l + 1 < a.L; ++l) lf();
    // 6. proposed kinetic energy, from the in-lane sums of p'^2
    auto kin_part = [&]() __attribute__((always_inline)) {
      T kq = (T)0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const T sq = p1[e] * p1[e];
        kq = (e == 0) ? sq : kq + sq;
      }
      return kq;
    };
    T ke1;
    if (a.L >= 1) {
#pragma unroll
      for (int e = 0; e < E; ++e) p1[e] = gfma(g1[e], half, p1[e]);
#pragma unroll
      for (int e = 0; e < E; ++e) q1[e] = gfma(p1[e], eps, q1[e]);
      using TL = typename Bare<decltype(tg)>::type;  // the per-lane target view
      if constexpr (requires { TL::template has_part<LPC>; }) {
        if constexpr (TL::template has_part<LPC>) {
          // the log-density and kinetic-energy sums reduced together
          T sums[2];
          sums[0] = tg.template eval_part<LPC, E>(q1, g1, lane);
#pragma unroll
          for (int e = 0; e < E; ++e) p1[e] = gfma(g1[e], half, p1[e]);
          sums[1] = kin_part();
          group_sum_n<LPC>(sums);
          lp1 = tg.finish(sums[0]);
          ke1 = sums[1] * (T)0.5;
        } else {
          lp1 = tg.template eval<LPC, E, true>(q1, g1, lane);
#pragma unroll
          for (int e = 0; e < E; ++e) p1[e] = gfma(g1[e], half, p1[e]);
          ke1 = group_sum<LPC>(kin_part()) * (T)0.5;
        }
      } else {
        lp1 = tg.template eval<LPC, E, true>(q1, g1, lane);
#pragma unroll
        for (int e = 0; e < E; ++e) p1[e] = gfma(g1[e], half, p1[e]);
        ke1 = group_sum<LPC>(kin_part()) * (T)0.5;
      }
    } else {
      ke1 = group_sum<LPC>(kin_part()) * (T)0.5;
    }
    // 7-9. Metropolis accept (NaN log_alpha rejects)
    const T log_alpha = (lp1 - lp) + (ke0 - ke1);
    if (log_alpha >= lnu) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        q[e] = q1[e];
        g[e] = g1[e];
      }
      lp = lp1;
      ++acc;
    }
    if (s >= a.collect_from) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        if (i < D) out[e] = q[e];
      }
      out += row_stride;
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    if (i < D) qs[c * D + i] = q[e];
  }
  if (lane == 0) {
    ((T*)a.logp)[c] = lp;
    a.accepts[c] += acc;
  }
}

// ---------------------------------------------------------------------------
// hmc_wide_kernel: the same transition for dim > 1024, one chain per
// workgroup of W = blockDim/64 waves (WideCtx in gm_device.h). The per-step
// momenta of a draw block (S transitions) go to a per-chain scratch in HBM
// (each thread re-reads only what it wrote), the accept log-uniforms stay in
// registers; every per-chain sum is a block reduction, so the accept branch is
// uniform over the workgroup. The reference's 10,000-dimensional Rosenbrock
// benchmark (hmc.rs:757-791) runs here.
template <class T, int E, class TG>
__global__ __launch_bounds__(gm_wide_max_threads(sizeof(T), E)) void hmc_wide_kernel(HmcLaunch a, TG tg_) {
  __shared__ T xf[2 * GM_WIDE_MAX_WAVES], xl[2 * GM_WIDE_MAX_WAVES], red[GM_WIDE_MAX_WAVES];
  const int tid = threadIdx.x;
  const long long c = blockIdx.x;
  const auto tg = tg_.template bind<64, E>(tid);  // coordinates tid*E + e
  __shared__ BmLds32 bm32[1];  // f32 momenta: the table-driven Box-Muller
  if constexpr (sizeof(T) == 4) {
    bm_lds_fill32(bm32[0]);
    __syncthreads();
  }
  WideCtx<T> cx{tid >> 6, (int)(blockDim.x >> 6), tid & 63, xf, xl, red, 0};
  const int D = a.D;
  const long long Dp = (long long)blockDim.x * E;
  T* __restrict__ qs = (T*)a.q;
  const T eps = (T)a.eps;
  const T half = (T)0.5 * eps;
  const uint32_t cid = a.chain_offset + (uint32_t)c;
  constexpr int S = Blk<T>::S;
  T* __restrict__ zs = (T*)a.zs + c * S * Dp;
  // q: current position; g1: the gradient at q1, which is the current
  // position at every transition start (a rejected proposal re-evaluates the
  // gradient at q instead of keeping a copy: same bits, E fewer registers)
  T q[E], q1[E], p1[E], g1[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = tid * E + e;
    q[e] = (i < D) ? qs[c * D + i] : (T)0;
  }
  T lp = tg.template eval_wide<E, true>(q, g1, cx);
#pragma unroll
  for (int e = 0; e < E; ++e) q1[e] = q[e];
  long long acc = 0;
  T lus[S];
  for (int s = 0; s < a.n_steps; ++s) {
    const uint64_t st = a.step0 + (uint64_t)s;
    const int k0 = (int)(st % S);
    if (s == 0 || k0 == 0) {  // draw block st/S: momenta to scratch, accept logs to registers
#pragma unroll 1
      for (int e = 0; e < E; ++e) {
        const int i = tid * E + e;
        T z[S];
        momenta_of(draw_block(a.seed, cid, st / S, TAG_MOM, (uint32_t)i), z, bm32[0]);
#pragma unroll
        for (int k = 0; k < S; ++k) zs[k * Dp + i] = (i < D) ? z[k] : (T)0;
      }
      T us[S];
      uniforms_of(draw_block(a.seed, cid, st / S, TAG_ACC, 0u), us);
#pragma unroll
      for (int k = 0; k < S; ++k) lus[k] = glog_unif(us[k]);
    }
    // 1-2. momentum ~ N(0, I) and its kinetic energy
    T kp = (T)0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      p1[e] = zs[k0 * Dp + tid * E + e];
      const T sq = p1[e] * p1[e];
      kp = (e == 0) ? sq : kp + sq;
    }
    const T ke0 = block_sum(kp, cx) * (T)0.5;
    T lnu = lus[0];
#pragma unroll
    for (int k = 1; k < S; ++k) lnu = (k0 == k) ? lus[k] : lnu;
    // 4-5. proposal and leapfrog (q1 = q and g1 = grad(q) here)
    T lp1 = lp;
    for (int l = 0; l < a.L; ++l) {
#pragma unroll
      for (int e = 0; e < E; ++e) p1[e] = gfma(g1[e], half, p1[e]);
#pragma unroll
      for (int e = 0; e < E; ++e) q1[e] = gfma(p1[e], eps, q1[e]);
      if (l + 1 < a.L) tg.template eval_wide<E, false>(q1, g1, cx);
      else lp1 = tg.template eval_wide<E, true>(q1, g1, cx);
#pragma unroll
      for (int e = 0; e < E; ++e) p1[e] = gfma(g1[e], half, p1[e]);
    }
    // 6. proposed kinetic energy
    T kq = (T)0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const T sq = p1[e] * p1[e];
      kq = (e == 0) ? sq : kq + sq;
    }
    const T ke1 = block_sum(kq, cx) * (T)0.5;
    // 7-9. Metropolis accept (NaN log_alpha rejects); block-uniform
    const T log_alpha = (lp1 - lp) + (ke0 - ke1);
    if (log_alpha >= lnu) {
#pragma unroll
      for (int e = 0; e < E; ++e) q[e] = q1[e];
      lp = lp1;
      ++acc;
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) q1[e] = q[e];
      if (a.L > 0) tg.template eval_wide<E, false>(q1, g1, cx);
    }
    if (s >= a.collect_from) {
      T* __restrict__ out = (T*)a.samples + ((a.sample_row0 + (s - a.collect_from)) * a.C + c) * D;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = tid * E + e;
        if (i < D) out[i] = q[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = tid * E + e;
    if (i < D) qs[c * D + i] = q[e];
  }
  if (tid == 0) {
    ((T*)a.logp)[c] = lp;
    a.accepts[c] += acc;
  }
}

}  // namespace gm
