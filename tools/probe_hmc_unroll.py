"""Leapfrog-loop unroll of the headline HMC kernel (gm_sampler_set_unroll:
1, 2 or 4 leapfrogs per loop trip; identical results) at the bench shape
(4096 x 64-D Rosenbrock f32, L = 50, 20 transitions per launch; CHAINS
and DIM override the shape): device
time per transition (HIP events), interleaved rounds, median.

    python tools/probe_hmc_unroll.py
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402
from general_mcmc_amd import _lib  # noqa: E402

lib = _lib.load()
_lib.check(lib.gm_set_device(0))
_lib.require_gpu()
C_ = int(os.environ.get("CHAINS", "4096"))
D_ = int(os.environ.get("DIM", "64"))
x0 = gm.init_with_seed(C_, D_, 42, np.float64).astype(np.float32)
samplers = {}
for u in (1, 2, 4):
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
    s.set_unroll(u)
    s.reserve(20)
    samplers[u] = s
t_end = time.perf_counter() + 0.1
while time.perf_counter() < t_end:
    for s in samplers.values():
        s.run_positions(20, 0)
res = {u: [] for u in samplers}
for _ in range(int(os.environ.get("ROUNDS", "15"))):
    for u, s in samplers.items():
        s.run_positions(20, 0)
        res[u].append(s.last_run_stats()[0] * 1e3 / 20)
print(json.dumps({"chains": C_, "dim": D_, **{str(u): {"median_us_per_transition": float(np.median(v)), "min": float(np.min(v))}
                  for u, v in res.items()}}))
