"""The bench's timed region as the driver runs it (a fresh process, W warm-up
transitions, one timed run of K), then the same call repeated: how much of the
first timed call's wall time is first-call cost, and what a warm-up that
collects into the reserved sample buffer changes.

    python tools/probe_bench_first.py [--warm-collect] [--steps 20 --warmup 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402
from general_mcmc_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--warm-collect", action="store_true")
ap.add_argument("--repeat", type=int, default=8)
ap.add_argument("--extra-warm", type=int, default=0, help="untimed run_positions(steps) calls after the warm-up")
ap.add_argument("--scratch-warm", type=int, default=0,
                help="untimed run_positions(steps) calls on a second sampler of the same shape after the warm-up")
ap.add_argument("--scratch-first", action="store_true",
                help="run the scratch-sampler launches before the measured sampler's warm-up")
ap.add_argument("--sleep-ms", type=float, default=0.0, help="idle time before each timed call")
a = ap.parse_args()
lib = _lib.load()
_lib.check(lib.gm_set_device(0))
lib = _lib.require_gpu()
x0 = gm.init_with_seed(4096, 64, 42, np.float64).astype(np.float32)
def scratch_warm():
    w = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(7)
    w.reserve(a.steps)
    for _ in range(a.scratch_warm):
        w.run_positions(a.steps, 0)
    return w


s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
s.reserve(a.steps)
if a.scratch_first and a.scratch_warm:
    w0 = scratch_warm()
if a.warm_collect:
    s.run_positions(a.warmup, 0)
else:
    s.run_positions(0, a.warmup)
for _ in range(a.extra_warm):
    s.run_positions(a.steps, 0)
if a.scratch_warm and not a.scratch_first:
    w = scratch_warm()
walls, kerns, calls = [], [], []
for i in range(1 + a.repeat):
    _lib.check(lib.gm_device_synchronize())
    if a.sleep_ms:
        time.sleep(a.sleep_ms * 1e-3)
    t0 = time.perf_counter()
    s.run_positions(a.steps, 0)
    t1 = time.perf_counter()
    _lib.check(lib.gm_device_synchronize())
    walls.append((time.perf_counter() - t0) * 1e6)
    calls.append((t1 - t0) * 1e6)
    kerns.append(s.last_run_stats()[0] * 1e3)
print(json.dumps({"lib": os.environ.get("GMCMC_LIB", "default"), "warm_collect": a.warm_collect,
                  "extra_warm": a.extra_warm, "scratch_warm": a.scratch_warm, "scratch_first": a.scratch_first, "sleep_ms": a.sleep_ms, "calls": [round(c, 1) for c in calls],
                  "first_wall_us": walls[0], "first_kernel_us": kerns[0],
                  "repeat_wall_us_median": float(np.median(walls[1:])),
                  "repeat_kernel_us_median": float(np.median(kerns[1:])),
                  "walls": [round(w, 1) for w in walls], "kernels": [round(k, 1) for k in kerns]}))
