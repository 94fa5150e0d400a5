"""Kernel time per transition as a function of L and of the chain count
(device time from HIP events; interleaved rounds)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402

cases = []
for L in (0, 1, 10, 50, 100):
    cases.append(("L", L, 4096, 64))
for C in (256, 1024, 2048, 4096, 8192, 16384, 65536):
    cases.append(("C", 50, C, 64))
cases.append(("N400", 1, 4096, 64))  # per-launch overhead: 400 transitions per launch
samplers = []
for kind, L, C, D in cases:
    s = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(C, D, 42, np.float32), 0.01, L).set_seed(1)
    s.run_positions(0, 8)
    samplers.append((kind, L, C, D, s))
res = {}
for r in range(5):
    for kind, L, C, D, s in samplers:
        n_steps = 400 if kind == "N400" else 40
        s.run_positions(n_steps, 0)
        ms, n = s.last_run_stats()
        res.setdefault((kind, L, C), []).append(ms * 1e3 / n_steps)
out = [{"kind": k[0], "L": k[1], "C": k[2], "us_per_transition": float(np.median(v)),
        "chain_lf_per_s": k[2] * max(k[1], 1) / (np.median(v) * 1e-6)} for k, v in res.items()]
print(json.dumps(out, indent=0))
