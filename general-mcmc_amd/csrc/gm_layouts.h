// gm_layouts.h — the (lanes-per-chain, elements-per-lane) layouts compiled
// into the sampling kernels, and a dispatcher from runtime values to template
// instantiations.
#pragma once
#include "gm_device.h"
#include "gm_internal.h"

// X(LPC, E)
#define GM_LAYOUT_LIST(X) \
  X(1, 1)                 \
  X(2, 1)                 \
  X(4, 1)                 \
  X(8, 1)                 \
  X(16, 1)                \
  X(32, 1)                \
  X(64, 1)                \
  X(16, 2)                \
  X(32, 2)                \
  X(64, 2)                \
  X(8, 4)                 \
  X(16, 4)                \
  X(32, 4)                \
  X(64, 4)                \
  X(16, 8)                \
  X(32, 8)                \
  X(64, 8)                \
  X(64, 16)

namespace gm {

template <class T, int LPC, int E, class F>
hipError_t dispatch_target(const TargetDev& tg, F& f) {
  switch (tg.kind) {
    case GM_TARGET_ROSENBROCK: {
      RosenbrockT<T> t;
      t.a = (T)tg.a;
      t.b = (T)tg.b;
      t.b2 = (T)2 * (T)tg.b;
      t.b4 = (T)4 * (T)tg.b;
      t.D = tg.D;
      return f.template operator()<T, LPC, E>(t);
    }
    case GM_TARGET_ISO_GAUSS: {
      IsoGaussT<T> t;
      t.var = (T)tg.std * (T)tg.std;
      t.D = tg.D;
      return f.template operator()<T, LPC, E>(t);
    }
    case GM_TARGET_GAUSS: {
      GaussT<T> t;
      t.mu = (const T*)tg.mu;
      t.prec = (const T*)tg.prec;
      t.nc = (T)tg.norm_const;
      t.D = tg.D;
      // LDS staging while it leaves room for >= 4 blocks (16 waves) per CU
      // next to the kernels' static Box-Muller tables (gm_rng.h: BmLds32,
      // 3 KiB, in the f32 HMC kernels; BmLds, 6 KiB, in the f64 MH kernel),
      // or for the matrix-core form (f64 16 x 4 at D <= 64: 41 KiB)
      constexpr size_t bm_static = sizeof(T) == 4 ? 3 * 1024 : 6 * 1024;
      t.use_lds = GaussT<T>::template lds_need<LPC, E>(tg.D) <= 40 * 1024 - bm_static ||
                  (GaussT<T>::template mfma_form<LPC, E>() && tg.D <= 16 * E);
      return f.template operator()<T, LPC, E>(t);
    }
    default:
      return hipErrorInvalidValue;
  }
}

// Calls f.template operator()<T, LPC, E>(target) for the runtime
// (dtype, target kind, layout); hipErrorInvalidValue when not compiled.
template <class F>
hipError_t dispatch(gm_dtype dt, const TargetDev& tg, const Layout& lay, F&& f) {
#define GM_TRY_LAYOUT(L_, E_)                                       \
  if (lay.lanes == L_ && lay.elems == E_) {                         \
    if (dt == GM_F32) return dispatch_target<float, L_, E_>(tg, f); \
    return dispatch_target<double, L_, E_>(tg, f);                  \
  }
  GM_LAYOUT_LIST(GM_TRY_LAYOUT)
#undef GM_TRY_LAYOUT
  return hipErrorInvalidValue;
}

// Wide layouts (one chain per workgroup of lanes/64 waves; HMC, dim > 1024):
// elems in {4, 8, 16, 32} (f64: 4, 8, 16), lanes up to gm_wide_max_threads,
// the targets with a wide evaluation (Rosenbrock, isotropic Gaussian). Calls
// f.template operator()<T, E>(target).
#define GM_WIDE_ELEMS_LIST(X) X(4) X(8) X(16) X(32)
template <class T, int E, class F>
hipError_t dispatch_wide_target(const TargetDev& tg, F& f) {
  switch (tg.kind) {
    case GM_TARGET_ROSENBROCK: {
      RosenbrockT<T> t;
      t.a = (T)tg.a;
      t.b = (T)tg.b;
      t.b2 = (T)2 * (T)tg.b;
      t.b4 = (T)4 * (T)tg.b;
      t.D = tg.D;
      return f.template operator()<T, E>(t);
    }
    case GM_TARGET_ISO_GAUSS: {
      IsoGaussT<T> t;
      t.var = (T)tg.std * (T)tg.std;
      t.D = tg.D;
      return f.template operator()<T, E>(t);
    }
    default:
      return hipErrorInvalidValue;
  }
}
template <class F>
hipError_t dispatch_wide(gm_dtype dt, const TargetDev& tg, const Layout& lay, F&& f) {
  if (lay.lanes % 64 || lay.lanes > gm_wide_max_threads(dt == GM_F32 ? 4 : 8, lay.elems))
    return hipErrorInvalidValue;
#define GM_TRY_WIDE(E_)                                                                     \
  if (lay.elems == E_) {                                                                    \
    if (dt == GM_F32) return dispatch_wide_target<float, E_>(tg, f);                        \
    if constexpr (E_ <= 16) return dispatch_wide_target<double, E_>(tg, f);                 \
    return hipErrorInvalidValue;                                                            \
  }
  GM_WIDE_ELEMS_LIST(GM_TRY_WIDE)
#undef GM_TRY_WIDE
  return hipErrorInvalidValue;
}

}  // namespace gm
