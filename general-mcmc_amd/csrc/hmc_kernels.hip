// hmc_kernels.hip — fused many-chain HMC transition kernel for gfx950.
//
// Replaces BatchedGenericHMC::step + leapfrog (batched_hmc.rs:129-190) and the
// BatchVector ops it calls on Tensor<B,2> (euclidean.rs:447-534): momentum
// draw (484-496), kinetic energy (464-472), add_scaled_assign kick/drift
// (392-394), log-density+gradient (hmc.rs:42-61), accept mask (527-533) and
// masked_assign (474-482).
//
// One launch runs `n_steps` full transitions for every chain; a chain's
// position, momentum and gradient live in VGPRs for the whole launch, so HBM
// sees one read and one write of the state per launch plus the collected
// samples. Arithmetic follows the reference's operation order with no FMA
// contraction (built with -ffp-contract=off):
//   p <- p + g*(0.5*eps);  q <- q + p*eps;  (logp, g) <- target(q);  p <- p + g*(0.5*eps)
//   K = (sum p*p) * 0.5;  log_alpha = (logp' - logp) + (K - K');  accept iff log_alpha >= ln u
// The gradient at the current point is carried across transitions (the
// reference re-evaluates it twice per step, batched_hmc.rs:138,169; same
// values), so a transition costs exactly L target evaluations.
#include "hmc_device.h"
#include "gm_jit.h"
#include "gm_layouts.h"

namespace gm {
hipError_t launch_hmc(gm_dtype dt, const TargetDev& tg, const Layout& lay, const HmcLaunch& a,
                      hipStream_t st, LaunchEvents ev) {
  if (tg.kind == GM_TARGET_CUSTOM) {  // user target, runtime-compiled (gm_jit.cpp)
    HmcLaunch aa = a;
    UserTargetArg ut{tg.params, tg.D};
    void* args[] = {&aa, &ut};
    return with_events(ev, st, [&] {
      return jit_launch(JIT_HMC, dt, tg, (unsigned)((a.C + 255) / 256), 256, 0, st, args);
    });
  }
  if (layout_is_wide(lay)) {
    return dispatch_wide(dt, tg, lay, [&]<class T, int E, class TG>(TG t) -> hipError_t {
      return launch_timed(hmc_wide_kernel<T, E, TG>, dim3((unsigned)a.C), dim3(lay.lanes), 0, st, ev, a, t);
    });
  }
  // (two chains per wave on packed f32 arithmetic, 13 VALU per two
  // chain-leapfrogs instead of 22, bitwise equal, measured no faster: at the
  // 2 waves per SIMD it leaves at 4096 chains the loop is latency-bound,
  // profiles/r04/ab_hmc_packed_and_fma_order.log; not kept)
  return dispatch(dt, tg, lay, [&]<class T, int LPC, int E, class TG>(TG t) -> hipError_t {
    const size_t lds = t.template lds_bytes<LPC, E>();
    const long long threads = a.C * LPC;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    return launch_timed(hmc_kernel<T, LPC, E, TG>, dim3(blocks), dim3(256), lds, st, ev, a, t);
  });
}

}  // namespace gm
