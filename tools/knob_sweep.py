"""Interleaved device time of the bench launch (default 4096 chains x 64-D
RosenbrockND f32, L=50, 100 transitions per launch) across settings of the
kernels' measurement knobs (environment variables read at each launch).

  python tools/knob_sweep.py "GM_HMC_STAGGER=1" "GM_HMC_STAGGER=2,GM_HMC_PHASE_SLEEP=16" ...
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402

C = int(os.environ.get("PROBE_C", "4096"))
D = int(os.environ.get("PROBE_D", "64"))
L = int(os.environ.get("PROBE_L", "50"))
rounds = int(os.environ.get("PROBE_ROUNDS", "7"))
settings = sys.argv[1:] or [""]
s = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(C, D, 42, np.float32), 0.01, L).set_seed(1)
s.reserve(100)
s.run_positions(0, 100)
res = {k: [] for k in settings}
for r in range(rounds):
    for k in settings:
        env = dict(kv.split("=") for kv in k.split(",") if kv)
        old = {n: os.environ.get(n) for n in env}
        os.environ.update(env)
        s.run_positions(100, 0)
        ms, n = s.last_run_stats()
        res[k].append(ms / n)
        for n_, v in old.items():
            if v is None:
                os.environ.pop(n_, None)
            else:
                os.environ[n_] = v
out = {k: {"ms_per_launch_median": float(np.median(v)), "ms_min": float(np.min(v)),
           "chain_lf_per_s": C * L * 100 / (np.median(v) * 1e-3)} for k, v in res.items()}
print(json.dumps({"C": C, "D": D, "L": L, "results": out}, indent=1))
