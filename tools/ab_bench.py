"""A/B of the driver-timed headline (bench.py --steps 20 --warmup 5, the
headline only: no config legs, CPU baselines or long ESS leg) for libgmcmc
variants (GMCMC_LIB), alternating processes in one GPU call:

    AB_ROUNDS=4 python tools/ab_bench.py A.so B.so ...
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sys.argv[1:]
rounds = int(os.environ.get("AB_ROUNDS", "4"))
args = ["--steps", "20", "--warmup", "5", "--configs", "", "--cpu-seconds", "0", "--cpu-config-seconds", "0",
        "--ess-long-discard", "0", "--no-north-star"]
res = {l: {"value": [], "kernel_ms": []} for l in libs}
for r in range(rounds):
    for l in libs:
        env = dict(os.environ, GMCMC_LIB=os.path.abspath(l))
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                             text=True, timeout=300)
        if out.returncode:
            print(out.stderr[-2000:])
            sys.exit(out.returncode)
        d = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
        res[l]["value"].append(d["value"])
        res[l]["kernel_ms"].append(d["timing"]["kernel_ms"])
        print(l, r, d["value"], d["timing"]["kernel_ms"], d["timing"]["wall_ms"], flush=True)
print(json.dumps({l: {"median_value": float(np.median(v["value"])), "max_value": float(np.max(v["value"])),
                      "median_kernel_ms": float(np.median(v["kernel_ms"]))} for l, v in res.items()}, indent=1))
