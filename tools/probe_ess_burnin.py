"""How far from 1 the split-R-hat of the bench workload (4096 x 64-D
Rosenbrock HMC f32, eps 0.01, L 50, start iid N(0,1)) is after n_discard
transitions, per parameter: quantiles of Stan's R-hat (sqrt(V/W)) over the 64
parameters and the ESS, for burn-in lengths up to 10^5 transitions.

    python tools/probe_ess_burnin.py
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
x0 = gm.init_with_seed(4096, 64, 42, np.float64).astype(np.float32)
for nd in (100, 4000, 20000, 100000):
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
    s.reserve(1000)
    t0 = time.perf_counter()
    ds = s.run_positions(1000, nd)
    _lib.check(lib.gm_device_synchronize())
    ts = time.perf_counter() - t0
    rhat, ess = ds.split_rhat_ess()
    stan = 1.0 / np.asarray(rhat, np.float64)
    q = lambda v, p: float(np.quantile(v, p))
    print(json.dumps({"n_discard": nd, "n_collect": 1000, "sampling_s": ts,
                      "stan_rhat": {"median": q(stan, 0.5), "p90": q(stan, 0.9), "max": float(stan.max()),
                                    "frac_below_1.01": float(np.mean(stan < 1.01)),
                                    "frac_below_1.1": float(np.mean(stan < 1.1)),
                                    "worst_params": [int(i) for i in np.argsort(-stan)[:5]]},
                      "ess": {"median": q(ess, 0.5), "min": float(np.min(ess))}}), flush=True)
    s.close()
