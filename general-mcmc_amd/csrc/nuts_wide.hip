// nuts_wide.hip — the NUTS kernel at the wide layouts: one chain per
// workgroup of lanes/64 waves (nuts_device.h, LPC > 64), for dimensions above
// 256 where a one-wave chain's per-lane state spills (64 x 8 and 64 x 16 f64
// spilled 77-1268 registers, profiles/r04/nuts_resources.txt). The targets
// with a cross-wave evaluation (Rosenbrock's neighbours through LDS, the
// isotropic Gaussian), the identity or diagonal metric (a dense metric is
// capped at dense_max_dim, far below these dimensions; the launcher keeps
// such samplers on the one-wave layouts).
#include "gm_layouts.h"
#include "nuts_device.h"
#include "nuts_launch.h"

// X(LPC, E)
#define GM_NUTS_WIDE_LAYOUTS(X) X(128, 4) X(256, 2) X(256, 4) X(512, 2)

namespace gm {

bool nuts_wide_layout_supported(int lanes, int elems) {
#define GM_NW_OK(L_, E_) \
  if (lanes == L_ && elems == E_) return true;
  GM_NUTS_WIDE_LAYOUTS(GM_NW_OK)
#undef GM_NW_OK
  return false;
}

template <class T, int LPC, int E>
static hipError_t launch_wide(const TargetDev& tg, NutsLaunch& a, hipStream_t st, const NutsLdsBudget& b) {
  auto go = [&]<class TG>(TG t) -> hipError_t {
    const unsigned blocks = (unsigned)a.C;  // one chain per block of LPC threads
    const size_t lds = nuts_size_lds(a, b, blocks, t.template lds_bytes<LPC, E>(), LPC, E, sizeof(T));
    if (a.mass_mode == 1)
      hipLaunchKernelGGL((nuts_kernel<T, LPC, E, TG, 1>), dim3(blocks), dim3(LPC), lds, st, a, t);
    else
      hipLaunchKernelGGL((nuts_kernel<T, LPC, E, TG, 0>), dim3(blocks), dim3(LPC), lds, st, a, t);
    return hipGetLastError();
  };
  if (a.mass_mode == 2) return hipErrorInvalidValue;  // (never: the launcher's layout choice)
  switch (tg.kind) {
    case GM_TARGET_ROSENBROCK: {
      RosenbrockT<T> t;
      t.a = (T)tg.a;
      t.b = (T)tg.b;
      t.b2 = (T)2 * (T)tg.b;
      t.b4 = (T)4 * (T)tg.b;
      t.D = tg.D;
      return go(t);
    }
    case GM_TARGET_ISO_GAUSS: {
      IsoGaussT<T> t;
      t.var = (T)tg.std * (T)tg.std;
      t.D = tg.D;
      return go(t);
    }
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t nuts_launch_wide(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a, hipStream_t st,
                            const NutsLdsBudget& b, bool* found) {
  *found = false;
#define GM_NW_TRY(L_, E_)                                                                         \
  if (lay.lanes == L_ && lay.elems == E_) {                                                       \
    *found = true;                                                                                \
    return dt == GM_F32 ? launch_wide<float, L_, E_>(tg, a, st, b) : launch_wide<double, L_, E_>(tg, a, st, b); \
  }
  GM_NUTS_WIDE_LAYOUTS(GM_NW_TRY)
#undef GM_NW_TRY
  return hipSuccess;
}

}  // namespace gm
