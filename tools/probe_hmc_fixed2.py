"""Decomposition of the HMC kernel's per-launch cost at the bench shape
(4096 x 64-D Rosenbrock f32): device time (HIP events, median of 7) of
launches of K transitions with L = 1 and L = 50 leapfrogs, so that
time(K, L) = fixed + K * (t_step + L * t_leapfrog) can be separated.

    python tools/probe_hmc_fixed2.py
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
out = {}
for L in (1, 50):
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, L).set_seed(42)
    s.reserve(40)
    s.run_positions(20, 0)
    for K in (1, 2, 4, 8, 20, 40):
        t = []
        for _ in range(7):
            s.run_positions(K, 0)
            t.append(s.last_run_stats()[0] * 1e3)
        out[f"L{L}_K{K}"] = float(np.median(t))
    s.close()
print(json.dumps(out))
