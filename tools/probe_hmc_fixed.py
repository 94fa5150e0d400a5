"""Fixed per-launch cost of the HMC kernel at the bench shape (4096 x 64-D
Rosenbrock f32, L = 50): device time (HIP events) of launches of K
transitions, K = 1 ... 100, median of 7 each; fixed = the intercept of the
least-squares line time(K) = fixed + K * per_step.

    python tools/probe_hmc_fixed.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402
from general_mcmc_amd import _lib  # noqa: E402

lib = _lib.load()
_lib.check(lib.gm_set_device(0))
_lib.require_gpu()
x0 = gm.init_with_seed(4096, 64, 42, np.float64).astype(np.float32)
s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
Ks = [1, 2, 4, 8, 12, 20, 40, 100]
s.reserve(max(Ks))
s.run_positions(20, 0)
out = {}
for K in Ks:
    t = []
    for _ in range(7):
        s.run_positions(K, 0)
        t.append(s.last_run_stats()[0] * 1e3)
    out[K] = float(np.median(t))
k = np.array(Ks, float)
v = np.array([out[K] for K in Ks])
A = np.vstack([np.ones_like(k), k]).T
(fixed, per), *_ = np.linalg.lstsq(A, v, rcond=None)
print(json.dumps({"kernel_us_by_K": out, "fixed_us": fixed, "per_step_us": per}))
