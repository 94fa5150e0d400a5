"""Where the HMC launch's fixed cost comes from: device time (HIP events) of
1- and 2-transition launches of the bench's kernel (64-D Rosenbrock f32,
L = 50, layout 64x1) at several chain counts, median of 9 each, after a
clock warm-up. A fixed cost that does not grow with the chains is serial
latency (prologue / epilogue); one that grows is dispatch or bandwidth.

    python tools/probe_hmc_prologue.py
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
out = {}
for C in (64, 1024, 4096, 16384):
    x0 = gm.init_with_seed(C, 64, 42, np.float64).astype(np.float32)
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
    s.reserve(20)
    t_end = time.perf_counter() + 0.05
    while time.perf_counter() < t_end:
        s.run_positions(20, 0)
    row = {}
    for K in (1, 2, 20):
        t = []
        for _ in range(9):
            s.run_positions(K, 0)
            t.append(s.last_run_stats()[0] * 1e3)
        row[K] = float(np.median(t))
    row["per_step"] = (row[20] - row[2]) / 18
    row["fixed"] = row[2] - 2 * row["per_step"]
    out[C] = row
    s.close()
print(json.dumps(out))
