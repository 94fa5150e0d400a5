"""The bench's timed call repeated: the headline shape (4096 x 64 f32, L 50,
20 transitions per call) in bench.py's order -- scratch launches for 50 ms,
5 warm-up transitions, then (device sync, timed run_positions + device sync)
REPS times -- printing each call's wall and HIP-event kernel time, so the
first timed call can be compared with the steady state. Variants per rep:
the plain sequence, and one with a 200 us host spin right before t0.

    python tools/probe_timed_call.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import general_mcmc_amd as gm  # noqa: E402


def main():
    reps = int(os.environ.get("REPS", 12))
    lib = gm._lib.load()
    gm._lib.check(lib.gm_set_device(0))
    x0 = gm.init_with_seed(4096, 64, 42, np.float64).astype(np.float32)
    out = {}
    for variant in ("plain", "spin200us"):
        s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
        scratch = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
        s.reserve(20)
        scratch.reserve(20)
        t_end = time.perf_counter() + 0.05
        while time.perf_counter() < t_end:
            scratch.run_positions(20, 0)
        s.run_positions(5, 0)
        walls, kerns = [], []
        for _ in range(reps):
            gm._lib.check(lib.gm_device_synchronize())
            if variant == "spin200us":
                t_spin = time.perf_counter() + 2e-4
                while time.perf_counter() < t_spin:
                    pass
            t0 = time.perf_counter()
            s.run_positions(20, 0)
            gm._lib.check(lib.gm_device_synchronize())
            walls.append((time.perf_counter() - t0) * 1e6)
            kerns.append(s.last_run_stats()[0] * 1e3)
        out[variant] = {"wall_us": [round(w, 2) for w in walls], "kernel_us": [round(k, 2) for k in kerns],
                        "first_minus_median_wall_us": round(walls[0] - float(np.median(walls[1:])), 2)}
        s.close()
        scratch.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
