"""Where the NUTS lockstep kernel's time goes (cfg3: 8192 chains, dense
Gaussian 32-D f64), from the measurement build abtest/nprof
(tools/ab_variants.sh nprof "-DGM_NUTS_PROF"; nuts_device.h): every wave bins
the shader cycles of each loop iteration by what its chains did in it --
bit 0 a transition start, bit 1 a subtree merge, bit 2 a doubling end, bit 3
a transition end -- and records the evaluation's share.

    GMCMC_LIB=abtest/nprof/libgmcmc.so python tools/probe_nuts_prof.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import general_mcmc_amd as gm  # noqa: E402
from bench_configs import dense_gauss_32  # noqa: E402

NAMES = ["start", "merge", "doubling_end", "transition_end"]


def main():
    chains = int(os.environ.get("CHAINS", 8192))
    layout = os.environ.get("LAYOUT", "")
    s = gm.NUTS(dense_gauss_32(), gm.init_det(chains, 32), 0.8, dtype=np.float64, max_depth=10).set_seed(42)
    if layout:
        s.set_layout(*[int(v) for v in layout.split("x")])
    mass = os.environ.get("MASS", "none")  # diagonal / dense: warm-up metric adaptation
    if mass != "none":
        s.set_mass_adaptation(gm.NUTSMassMatrixConfig(mass))
    s.run_positions(1, 200)  # warm-up, step sizes adapted
    lf0 = s.leapfrog_counts().sum()
    s.run_positions(200, 0)
    lf = int(s.leapfrog_counts().sum() - lf0)
    lib = gm._lib.load()
    lanes, elems = s.layout()
    waves = chains * lanes // 64
    buf = np.zeros((waves, 43), np.uint64)
    f = lib.gm_nuts_prof_read
    f.argtypes = [C.c_void_p, C.c_longlong]
    assert f(buf.ctypes.data, buf.size) == 0
    cnt = buf[:, 0:32:2].astype(np.float64).sum(0)
    cyc = buf[:, 1:32:2].astype(np.float64).sum(0)
    it = float(cnt.sum())
    out = {"chains": chains, "layout": f"{lanes}x{elems}", "waves": waves, "leapfrogs": lf,
           "iterations_per_wave": it / waves, "leapfrogs_per_chain": lf / chains,
           "cycles_per_iteration": float(cyc.sum() / it),
           "eval_cycles_per_iteration": float(buf[:, 32].astype(np.float64).sum() / it),
           "product_cycles_per_iteration": float(buf[:, 34].astype(np.float64).sum() / it), "bins": []}
    for b in range(16):
        if cnt[b] == 0:
            continue
        out["bins"].append({"what": "+".join(NAMES[i] for i in range(4) if b >> i & 1) or "leaf_only",
                            "share_of_iterations": cnt[b] / it, "cycles_mean": cyc[b] / cnt[b],
                            "share_of_cycles": cyc[b] / cyc.sum()})
    # marginal cost of each event: least squares over the bins
    X = np.array([[1.0] + [float(b >> i & 1) for i in range(4)] for b in range(16)])
    w = cnt > 0
    coef, *_ = np.linalg.lstsq(X[w] * np.sqrt(cnt[w])[:, None], (cyc[w] / np.maximum(cnt[w], 1)) * np.sqrt(cnt[w]),
                               rcond=None)
    out["fit_cycles"] = {"base": coef[0], **{NAMES[i]: coef[i + 1] for i in range(4)}}
    seg_names = ["momentum_draw", "kick_drift", "target_eval_part", "kick_kinetic_part", "reduction",
                 "leaf_rules", "merge_climb", "doubling_transition_end"]
    seg = buf[:, 35:43].astype(np.float64).sum(0) / it
    out["segments_cycles_per_iteration"] = {n: float(v) for n, v in zip(seg_names, seg)}
    out["segments_note"] = ("measurement build: an s_waitcnt(0) + s_memtime at each boundary, so memory "
                            "latency is charged to the segment that issued the access")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
