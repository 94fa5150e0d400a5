"""Interleaved timing of the HMC kernel across lane layouts (one process,
rounds interleaved per cuda rule 24). Prints us per transition (device time)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--chains", type=int, default=4096)
p.add_argument("--dim", type=int, default=64)
p.add_argument("--L", type=int, default=50)
p.add_argument("--steps", type=int, default=100)
p.add_argument("--rounds", type=int, default=5)
p.add_argument("--dtype", default="f32")
p.add_argument("--layouts", default="64x1,32x2,16x4,8x8" )
a = p.parse_args()
dt = np.float32 if a.dtype == "f32" else np.float64
x0 = gm.init_with_seed(a.chains, a.dim, 42, dt)
lays = [tuple(int(v) for v in s.split("x")) for s in a.layouts.split(",")]
samplers = {}
for lay in lays:
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, a.L, dtype=dt).set_seed(42)
    try:
        s.set_layout(*lay)
    except gm.GMError as e:
        print("skip", lay, e)
        continue
    s.run_positions(0, 20)
    samplers[lay] = s
res = {lay: [] for lay in samplers}
for r in range(a.rounds):
    for lay, s in samplers.items():
        s.run_positions(a.steps, 0)
        ms, n = s.last_run_stats()
        res[lay].append(ms * 1e3 / a.steps)
out = {}
for lay, v in res.items():
    out[f"{lay[0]}x{lay[1]}"] = {"us_per_transition_median": float(np.median(v)),
                                  "us_min": float(np.min(v)),
                                  "chain_leapfrogs_per_s": a.chains * a.L / (np.median(v) * 1e-6)}
print(json.dumps({"chains": a.chains, "dim": a.dim, "L": a.L, "dtype": a.dtype, "results": out}, indent=1))
