"""A/B device time of the bench launch for libgmcmc variants (GMCMC_LIB),
alternating processes in one GPU call: python tools/ab_run.py A.so B.so ..."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sys.argv[1:]
rounds = int(os.environ.get("AB_ROUNDS", "4"))
extra = os.environ.get("AB_ARGS", "--layouts 64x1 --rounds 3").split()
res = {l: [] for l in libs}
for r in range(rounds):
    for l in libs:
        env = dict(os.environ, GMCMC_LIB=os.path.abspath(l))
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sweep_hmc.py")] + extra,
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(out.stderr[-2000:])
            sys.exit(out.returncode)
        d = json.loads(out.stdout[out.stdout.index("{"):])
        for k, v in d["results"].items():
            res[l].append(v["us_per_transition_median"])
        print(l, r, [v["us_per_transition_median"] for v in d["results"].values()], flush=True)
print(json.dumps({l: {"median_us": float(np.median(v)), "min_us": float(np.min(v))} for l, v in res.items()}, indent=1))
