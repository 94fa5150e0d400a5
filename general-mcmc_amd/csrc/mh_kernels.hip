// mh_kernels.hip — many-chain random-walk Metropolis-Hastings for gfx950.
//
// Replaces MHMarkovChain::step (metropolis_hastings.rs:306-318) with an
// IsotropicGaussian proposal (distributions.rs:368-390), run per chain as
// run_chain does (core.rs:95-115). Operation order follows the reference:
//   x' = x + n*std,  n ~ N(0,1)                                   (:372-374)
//   log q(to|from) = sum_i ( -(d_i*d_i) / (2*var) ) - (D*0.5) * ln(var*pi*std*std)
//                    (the reference's constant, :388; symmetric, so the
//                     forward and backward terms are bitwise equal)
//   log_alpha = (lp(x') + log q_b) - (lp(x) + log q_f); accept iff log_alpha > ln u
// The current log-density is carried across steps (the reference recomputes
// it, :308 -- same value).
#include "mh_device.h"
#include "gm_jit.h"
#include "gm_layouts.h"
#include "gm_track.h"

namespace gm {
hipError_t launch_mh(gm_dtype dt, const TargetDev& tg, const Layout& lay, const MhLaunch& a,
                     hipStream_t st, LaunchEvents ev) {
  if (tg.kind == GM_TARGET_CUSTOM) {  // user target, runtime-compiled (gm_jit.cpp)
    MhLaunch aa = a;
    UserTargetArg ut{tg.params, tg.D};
    void* args[] = {&aa, &ut};
    return with_events(ev, st, [&] {
      return jit_launch(JIT_MH, dt, tg, (unsigned)((a.C + 255) / 256), 256, 0, st, args);
    });
  }
  return dispatch(dt, tg, lay, [&]<class T, int LPC, int E, class TG>(TG t) -> hipError_t {
    const long long threads = a.C * LPC;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    const size_t lds = t.template lds_bytes<LPC, E>();
    return launch_timed(mh_kernel<T, LPC, E, TG>, dim3(blocks), dim3(256), lds, st, ev, a, t);
  });
}

}  // namespace gm
