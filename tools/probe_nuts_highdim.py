"""NUTS throughput at high dimension on the default layouts (64 lanes x E,
E = 4 / 8 / 16): the launch-bound A/B of ADVICE r03 (2 vs 1 waves per SIMD
for E >= 4). One JSON line per (dtype, dim):

    GMCMC_LIB=abtest/X/libgmcmc.so python tools/probe_nuts_highdim.py
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
    for dt in (np.float64, np.float32):
        for D in (256, 512, 1024):
            s = gm.NUTS(gm.IsotropicGaussian(1.0), gm.init_det(chains, D).astype(dt), 0.8, dtype=dt,
                        max_depth=8).set_seed(3)
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
