"""A/B of NUTS cfg3 throughput for libgmcmc variants (GMCMC_LIB), alternating
processes in one GPU call:  python tools/ab_nuts.py A.so B.so ...
(variants from tools/ab_build_unit.sh)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sys.argv[1:]
rounds = int(os.environ.get("AB_ROUNDS", "3"))
res = {l: [] for l in libs}
for r in range(rounds):
    for l in libs:
        env = dict(os.environ, GMCMC_LIB=os.path.abspath(l))
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_configs.py"), "--which", "3"] + os.environ.get("AB_ARGS", "").split(),
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(out.stderr[-2000:])
            sys.exit(out.returncode)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res[l].append(d["leapfrog_per_s"])
        print(l, r, d["leapfrog_per_s"], d["ess_mean"], flush=True)
print(json.dumps({l: {"median": float(np.median(v)), "max": float(np.max(v))} for l, v in res.items()}, indent=1))
