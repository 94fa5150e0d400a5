// nuts_launch.h — launch of the NUTS transition kernel for one compiled
// layout. The (dtype, target, layout) instantiations are spread over the
// translation units nuts_part0.hip ... nuts_part5.hip (three layouts each) so
// that they compile in parallel; nuts_run (nuts_kernels.hip) asks each part in
// turn.
#pragma once
#include <hip/hip_runtime.h>

#include "gm_internal.h"
#include "gm_launch.h"

namespace gm {

// What the LDS sizing of a launch needs to know about the device and the
// sampler (gm_nuts_set_lds_levels).
struct NutsLdsBudget {
  int ncu = 256;                // compute units
  int lds_max = 64 * 1024;      // dynamic LDS per block
  long long lds_cap = -1;       // levels cap (-1: as many as fit)
  int minv_lds = 1;             // dense metric in LDS: 1 packed, 2 full when it fits (else packed), 0 off
                                // (gm_nuts_set_dense_forms)
  int chol_lds = 0;             // its Cholesky factor too (0: off)
};

// LDS of a launch: the target's staging area (tgl bytes), then as many
// subtree-stack levels as fit in the CU's 160 KiB shared by the grid's blocks
// per CU (at most 4 blocks counted) and max_depth; sets a.lds_levels and
// a.lds_stack_off, returns the dynamic LDS size.
inline size_t nuts_size_lds(NutsLaunch& a, const NutsLdsBudget& b, unsigned blocks, size_t tgl, int LPC, int E,
                            size_t tsz) {
  tgl = (tgl + 15) / 16 * 16;
  const int NT = LPC > 64 ? LPC : 256;  // threads per block (one chain per block when wide)
  const size_t per_level = (size_t)3 * NT * E * tsz + (size_t)(NT / LPC) * (tsz + 8);
  long long bpc = ((long long)blocks + b.ncu - 1) / b.ncu;
  bpc = bpc < 1 ? 1 : bpc > 4 ? 4 : bpc;
  if (LPC > 64) {  // the wide kernels' resident blocks per CU (their launch bound)
    const long long rb = (long long)nuts_wide_waves((int)tsz, E) * 4 / (NT / 64);
    bpc = bpc < rb ? bpc : (rb < 1 ? 1 : rb);
  }
  // the dense-metric kernels run GM_DENSE_WAVES (adaptive: one, 512
  // registers per lane, the metric's products and state without scratch
  // spills) or GM_FROZEN_WAVES (frozen) waves per SIMD, i.e. blocks per CU
  if (a.mass_mode == 2) {
    const long long w = a.dense_frozen ? GM_FROZEN_WAVES : GM_DENSE_WAVES;
    bpc = bpc < w ? bpc : w;
  }
  size_t budget = (size_t)(160 * 1024) / (size_t)bpc - 1024;
  if (budget > (size_t)b.lds_max) budget = (size_t)b.lds_max;
  // Dense metric (layout 16 x 2): the block's chains' M^-1 resident in LDS,
  // lower triangles packed (nuts_device.h, minv_packed_lds), when it fits
  // next to the target's staging at the grid's blocks per CU; otherwise the
  // per-chain matrices stream from L2/MALL at every drift and kinetic energy
  // (2 x D*D*s bytes per leapfrog)
  a.minv_lds = 0;
  a.minv_lds_off = 0;
  a.chol_lds = 0;
  a.chol_lds_off = 0;
  if (a.mass_mode == 2 && b.minv_lds && LPC == 16 && E == 2 && a.D <= LPC * E) {
    // the frozen-dense kernel (nuts_device.h MASS 3) takes the packed M^-1
    // only (no full form, no L in LDS)
    const int want = a.dense_frozen ? 1 : b.minv_lds;
    const int want_chol = a.dense_frozen ? 0 : b.chol_lds;
    const size_t dp = (size_t)LPC * E;
    const size_t mb = (size_t)(256 / LPC) * (dp * (dp + 1) / 2) * tsz;
    const size_t mf = (size_t)(256 / LPC) * dp * dp * tsz;
    if (want != 1 && tgl + mf <= budget) {  // the full matrices (no address arithmetic)
      a.minv_lds = 2;
      a.minv_lds_off = (unsigned)tgl;
      tgl += (mf + 15) / 16 * 16;
    } else if (tgl + mb <= budget) {
      a.minv_lds = 1;
      a.minv_lds_off = (unsigned)tgl;
      tgl += (mb + 15) / 16 * 16;
      if (want_chol && tgl + mb <= budget) {
        a.chol_lds = 1;
        a.chol_lds_off = (unsigned)tgl;
        tgl += (mb + 15) / 16 * 16;
      }
    }
  }
  long long kl = budget > tgl ? (long long)((budget - tgl) / per_level) : 0;
  if (kl > a.max_depth) kl = a.max_depth;
  if (b.lds_cap >= 0 && kl > b.lds_cap) kl = b.lds_cap;
  a.lds_levels = (int)kl;
  a.lds_stack_off = (unsigned)tgl;
  return tgl + (size_t)kl * per_level;
}

// Launches nuts_kernel for (dt, tg, lay) when part `part` holds that layout
// (*found = true), else returns hipSuccess with *found = false.
hipError_t nuts_launch_part0(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a, hipStream_t st,
                             const NutsLdsBudget& b, bool* found);
hipError_t nuts_launch_part1(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a, hipStream_t st,
                             const NutsLdsBudget& b, bool* found);
hipError_t nuts_launch_part2(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a, hipStream_t st,
                             const NutsLdsBudget& b, bool* found);
hipError_t nuts_launch_part3(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a, hipStream_t st,
                             const NutsLdsBudget& b, bool* found);
hipError_t nuts_launch_part4(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a, hipStream_t st,
                             const NutsLdsBudget& b, bool* found);
hipError_t nuts_launch_part5(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a, hipStream_t st,
                             const NutsLdsBudget& b, bool* found);
// the wide layouts (lanes > 64, nuts_wide.hip)
hipError_t nuts_launch_wide(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a, hipStream_t st,
                            const NutsLdsBudget& b, bool* found);
bool nuts_wide_layout_supported(int lanes, int elems);

inline hipError_t nuts_launch_layout(gm_dtype dt, const TargetDev& tg, const Layout& lay, NutsLaunch& a,
                                     hipStream_t st, const NutsLdsBudget& b) {
  using Fn = hipError_t (*)(gm_dtype, const TargetDev&, const Layout&, NutsLaunch&, hipStream_t,
                            const NutsLdsBudget&, bool*);
  static const Fn parts[] = {nuts_launch_part0, nuts_launch_part1, nuts_launch_part2, nuts_launch_part3,
                             nuts_launch_part4, nuts_launch_part5, nuts_launch_wide};
  for (Fn f : parts) {
    bool found = false;
    const hipError_t e = f(dt, tg, lay, a, st, b, &found);
    if (found) return e;
  }
  return hipErrorInvalidValue;
}

}  // namespace gm
