"""Host path of the bench's timed call at the driver's shape (4096 x 64 f32,
L 50, 20 transitions): wall time of variants of "run + wait", interleaved in
one process after the bench's warm-up, with the run's HIP-event kernel time.

  V1 run_positions (waits on its stream) + gm_device_synchronize   (r02 bench)
  V2 async run_positions + gm_device_synchronize                    (one wait)
  V3 V2 through the bare ctypes entry (no Python facade)
  V4 run_positions alone (stream wait only)
  E  gm_device_synchronize on an idle device
Prints one JSON object."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import general_mcmc_amd as gm  # noqa: E402


def main():
    K, reps = int(os.environ.get("K", 20)), int(os.environ.get("REPS", 40))
    lib = gm._lib.load()
    gm._lib.check(lib.gm_set_device(0))
    x0 = gm.init_with_seed(4096, 64, 42, np.float64).astype(np.float32)
    A = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
    B = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42).set_async(True)
    for s in (A, B):
        s.reserve(K)
        for _ in range(3):
            s.run_positions(K, 0)
    lib.gm_device_synchronize()
    p = C.c_void_p()
    sync = lib.gm_device_synchronize
    run = lib.gm_run_device
    hb = B._h

    def v1():
        A.run_positions(K, 0)
        sync()

    def v2():
        B.run_positions(K, 0)
        sync()

    def v3():
        run(hb, K, 0, C.byref(p))
        sync()

    def v4():
        A.run_positions(K, 0)

    def e():
        sync()
    variants = {"V1": (v1, A), "V2": (v2, B), "V3": (v3, B), "V4": (v4, A), "E": (e, None)}
    res = {k: {"wall_us": [], "kernel_us": []} for k in variants}
    for _ in range(reps):
        for k, (fn, smp) in variants.items():
            sync()
            t0 = time.perf_counter()
            fn()
            t = time.perf_counter() - t0
            res[k]["wall_us"].append(t * 1e6)
            if smp is not None:
                sync()
                res[k]["kernel_us"].append(smp.last_run_stats()[0] * 1e3)
    out = {"K": K, "reps": reps}
    for k, v in res.items():
        w = np.array(v["wall_us"])
        out[k] = {"wall_us_median": float(np.median(w)), "wall_us_min": float(w.min())}
        if v["kernel_us"]:
            out[k]["kernel_us_median"] = float(np.median(v["kernel_us"]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
