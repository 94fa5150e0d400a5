"""NUTS throughput at high dimension on the default layouts (round 5: the
wide layouts above 256 dimensions, a chain per workgroup; 64 lanes x 4 at
256). One JSON line per (dtype, dim[, layout]):

    GMCMC_LIB=abtest/X/libgmcmc.so python tools/probe_nuts_highdim.py
    PROBE_CASES="f64:1024:256x4,f64:512:128x4" python tools/probe_nuts_highdim.py   # explicit layouts
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import general_mcmc_amd as gm  # noqa: E402


def main():
    chains = int(os.environ.get("PROBE_CHAINS", "2048"))
    cases = [(dt, D, None) for dt in (np.float64, np.float32) for D in (256, 512, 1024)]
    if os.environ.get("PROBE_CASES"):
        cases = []
        for c in os.environ["PROBE_CASES"].split(","):
            d, D, lay = c.split(":")
            cases.append((np.float64 if d == "f64" else np.float32, int(D), tuple(int(v) for v in lay.split("x"))))
    for dt, D, lay in cases:
        if True:
            s = gm.NUTS(gm.IsotropicGaussian(1.0), gm.init_det(chains, D).astype(dt), 0.8, dtype=dt,
                        max_depth=8).set_seed(3)
            if lay:
                s.set_layout(*lay)
            s.run_positions(1, 30)  # step-size warm-up, untimed
            s.reserve(30)
            lib = gm._lib.load()
            lf0 = int(s.leapfrog_counts().sum())
            lib.gm_device_synchronize()
            t0 = time.perf_counter()
            s.run_positions(30, 0)
            lib.gm_device_synchronize()
            t = time.perf_counter() - t0
            lf = int(s.leapfrog_counts().sum()) - lf0
            print(json.dumps({"dtype": np.dtype(dt).name, "dim": D, "chains": chains, "layout": "%dx%d" % s.layout(),
                              "leapfrogs": lf, "seconds": t, "leapfrogs_per_s": lf / t}), flush=True)
            s.close()


if __name__ == "__main__":
    main()
