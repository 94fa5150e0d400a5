"""One NUTS workload for profiling: cfg3-shaped (8192 x 32-D f64) by default.
    python tools/probe_nuts_one.py [--target dense|iso] [--layout 32x1] [--steps 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import general_mcmc_amd as gm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--target", default="dense")
ap.add_argument("--layout", default="")
ap.add_argument("--chains", type=int, default=8192)
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--adapt", type=int, default=100)
a = ap.parse_args()
D = 32
if a.target == "dense":
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((D, D)))
    cov = q @ np.diag(np.logspace(-1, 1, D)) @ q.T
    tg = gm.DenseGaussian(np.zeros(D), 0.5 * (cov + cov.T))
else:
    tg = gm.IsotropicGaussian(1.0)
s = gm.NUTS(tg, gm.init_det(a.chains, D), 0.8, dtype=np.float64, max_depth=10).set_seed(42)
if a.layout:
    s.set_layout(*[int(v) for v in a.layout.split("x")])
s.run_positions(1, a.adapt)
lib = gm._lib.load()
lf0 = s.leapfrog_counts().sum()
lib.gm_device_synchronize()
t0 = time.perf_counter()
s.run_positions(a.steps, 0)
lib.gm_device_synchronize()
t = time.perf_counter() - t0
lf = s.leapfrog_counts().sum() - lf0
print(json.dumps({"target": a.target, "layout": "%dx%d" % s.layout(), "s": t, "lf_per_s": lf / t,
                  "mean_tree": lf / (a.chains * a.steps)}))
