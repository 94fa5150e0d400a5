"""cfg3 NUTS sampling-phase throughput against the number of subtree-stack
levels kept in LDS (the rest in HBM): 8192 chains x 32-D f64 dense Gaussian,
500 warm-up transitions, then 500 sampling transitions timed."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import general_mcmc_amd as gm  # noqa: E402
from bench_configs import dense_gauss_32  # noqa: E402


def main():
    lib = gm._lib.load()
    out = {}
    for lv in [int(v) for v in os.environ.get("LEVELS", "-1,0,2,4,5,6,10").split(",")]:
        s = gm.NUTS(dense_gauss_32(), gm.init_det(8192, 32), 0.8, dtype=np.float64, max_depth=10).set_seed(42)
        s.set_lds_levels(lv)
        s.run_positions(1, 500)
        lf0 = s.leapfrog_counts().sum()
        lib.gm_device_synchronize()
        t0 = time.perf_counter()
        s.run_positions(500, 0)
        lib.gm_device_synchronize()
        t = time.perf_counter() - t0
        lf = int(s.leapfrog_counts().sum() - lf0)
        out[lv] = {"leapfrogs_per_s": lf / t, "kernel_ms": s.last_run_stats()[0], "leapfrogs": lf}
        print(lv, out[lv], flush=True)
        s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
