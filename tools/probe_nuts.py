"""NUTS cost breakdown on one GPU: leapfrogs/s of the cfg3 workload
(8192 chains, 32-D f64) for the dense-Gaussian target and, as a control with
the same tree logic but an O(D) gradient, the isotropic Gaussian; per layout.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import general_mcmc_amd as gm  # noqa: E402


def dense_gauss_32():
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((32, 32)))
    cov = q @ np.diag(np.logspace(-1, 1, 32)) @ q.T
    return gm.DenseGaussian(np.zeros(32), 0.5 * (cov + cov.T))


def run(target, layout, C=8192, D=32, dtype=np.float64, steps=200):
    s = gm.NUTS(target, gm.init_det(C, D), 0.8, dtype=dtype, max_depth=10).set_seed(42)
    if layout:
        s.set_layout(*layout)
    s.run_positions(1, 200)  # adapt
    lib = gm._lib.load()
    lf0 = s.leapfrog_counts().sum()
    lib.gm_device_synchronize()
    t0 = time.perf_counter()
    s.run_positions(steps, 0)
    lib.gm_device_synchronize()
    t = time.perf_counter() - t0
    lf = s.leapfrog_counts().sum() - lf0
    return {"layout": "%dx%d" % s.layout(), "s": t, "lf_per_s": lf / t, "mean_tree": lf / (C * steps)}


targets = {"dense": dense_gauss_32(), "iso": gm.IsotropicGaussian(1.0)}
for name, tg in targets.items():
    for lay in [None, (16, 2), (8, 4), (4, 8) if False else None]:
        if lay is None and name == "iso" and False:
            continue
        try:
            r = run(tg, lay)
        except Exception as e:  # layout not compiled
            r = {"layout": str(lay), "error": str(e)}
        r["target"] = name
        print(json.dumps(r), flush=True)
