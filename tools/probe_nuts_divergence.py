"""Lockstep cost of NUTS trees in a wave: per-transition leapfrog counts of
every chain (cfg3: 8192 chains, 32-D dense Gaussian f64, after warm-up), and
the work a wave executes if its G chains run each transition's trees in
lockstep (the max over the group) versus their mean."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import general_mcmc_amd as gm  # noqa: E402
from bench_configs import dense_gauss_32  # noqa: E402  (bench_configs runs its own measurements on import)

C = 8192
s = gm.NUTS(dense_gauss_32(), gm.init_det(C, 32), 0.8, dtype=np.float64, max_depth=10).set_seed(42)
s.run_positions(1, 500)
counts = []
prev = s.leapfrog_counts().copy()
for t in range(40):
    s.run_positions(1, 0) if t == 0 else s.run_positions(2, 0)
    cur = s.leapfrog_counts().copy()
    counts.append(cur - prev)
    prev = cur
n = np.array(counts, dtype=np.float64)  # [T, C] (first row: 0 or 1 transitions, rest 1)
n = n[1:]
out = {"mean_leapfrogs_per_chain_transition": float(n.mean())}
for G in (1, 2, 4, 8, 16):
    g = n.reshape(n.shape[0], C // G, G)
    out[f"lockstep_overhead_G{G}"] = float(g.max(axis=2).mean() / g.mean())
hist = np.bincount(n.astype(int).ravel())
out["hist_nonzero"] = {int(k): int(v) for k, v in enumerate(hist) if v}
print(json.dumps(out, indent=1))
