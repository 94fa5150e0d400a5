"""The bench's timed launch after device warm-ups of different lengths (GPU
clock ramp): each trial idles IDLE s, runs scratch launches of the timed
shape for WARM ms, the W = 5 warm-up transitions of the measured sampler,
then the timed 20-transition call; wall and HIP-event kernel time per trial.
Prints one JSON object (medians per warm-up length)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import general_mcmc_amd as gm  # noqa: E402


def main():
    K, W = 20, 5
    idle = float(os.environ.get("IDLE", 0.5))
    warms = [float(v) for v in os.environ.get("WARMS", "0,0.2,1,3,10,30,100").split(",")]
    reps = int(os.environ.get("REPS", 5))
    lib = gm._lib.load()
    gm._lib.check(lib.gm_set_device(0))
    x0 = gm.init_with_seed(4096, 64, 42, np.float64).astype(np.float32)
    scratch = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(7)
    scratch.reserve(K)
    scratch.run_positions(K, 0)
    res = {w: {"wall_us": [], "kernel_us": []} for w in warms}
    for _ in range(reps):
        for w in warms:
            s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
            s.reserve(K)
            lib.gm_device_synchronize()
            time.sleep(idle)
            t_end = time.perf_counter() + w * 1e-3
            n = 0
            while n < 2 or time.perf_counter() < t_end:
                scratch.run_positions(K, 0)
                n += 1
            s.run_positions(W, 0)
            lib.gm_device_synchronize()
            t0 = time.perf_counter()
            s.run_positions(K, 0)
            lib.gm_device_synchronize()
            t = time.perf_counter() - t0
            res[w]["wall_us"].append(t * 1e6)
            res[w]["kernel_us"].append(s.last_run_stats()[0] * 1e3)
            s.close()
    out = {"K": K, "W": W, "idle_s": idle, "reps": reps}
    for w, v in res.items():
        out[f"warm_{w}ms"] = {"wall_us_median": float(np.median(v["wall_us"])),
                              "kernel_us_median": float(np.median(v["kernel_us"])),
                              "wall_us": [round(x, 1) for x in v["wall_us"]]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
