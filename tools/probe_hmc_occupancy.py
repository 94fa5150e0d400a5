"""Kernel time of the bench launch (4096 chains x 64-D RosenbrockND f32, L=50,
100 transitions per launch) against a dynamic-LDS pad that caps the
workgroups resident per CU (GM_HMC_LDS_PAD, a measurement knob): tests
whether the hardware dispatcher spreads the 1024 workgroups evenly."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402

C = int(os.environ.get("PROBE_C", "4096"))
pads = [int(v) for v in os.environ.get("PROBE_PADS", "0,20000,36000,50000,70000").split(",")]
s = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(C, 64, 42, np.float32), 0.01, 50).set_seed(1)
s.set_steps_per_launch(100) if hasattr(s, "set_steps_per_launch") else None
s.run_positions(0, 100)
res = {}
for r in range(7):
    for pad in pads:
        os.environ["GM_HMC_LDS_PAD"] = str(pad)
        s.run_positions(100, 0)
        ms, n = s.last_run_stats()
        res.setdefault(pad, []).append(ms / n)
out = {str(p): {"ms_per_launch_median": float(np.median(v)), "ms_min": float(np.min(v)),
                "chain_lf_per_s": C * 50 * 100 / (np.median(v) * 1e-3)} for p, v in res.items()}
print(json.dumps({"C": C, "results": out}, indent=1))
