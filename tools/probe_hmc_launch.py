"""Where the bench's wall time goes at the driver's shape (4096 x 64-D
Rosenbrock, f32, L = 50): device time per launch against transitions per
launch (intercept = fixed per-launch cost in the kernel), the host cost of a
run_positions call around it, and a bare ctypes round trip.

    python tools/probe_hmc_launch.py [--out gpurun_out/probe_launch.json]
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


def med(v):
    return float(np.median(v))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--chains", type=int, default=4096)
    ap.add_argument("--quick", action="store_true", help="kernel-vs-K fit only")
    a = ap.parse_args()
    lib = _lib.load()
    _lib.check(lib.gm_set_device(0))
    C, D, L = a.chains, 64, 50
    s = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(C, D, 42, np.float64).astype(np.float32), 0.01, L).set_seed(42)
    s.reserve(200)
    s.run_positions(0, 5)
    res = {"shape": f"{C}x{D} f32 L={L}"}
    # device time per launch vs K
    ks = [1, 2, 5, 10, 20, 50, 100, 200]
    dev = {}
    for _ in range(3):
        for k in ks:
            s.run_positions(k, 0)
            ms, n = s.last_run_stats()
            dev.setdefault(k, []).append(ms * 1e3)
    res["kernel_us_by_K"] = {k: med(v) for k, v in dev.items()}
    x = np.array(ks, dtype=float)
    y = np.array([res["kernel_us_by_K"][k] for k in ks])
    slope, icpt = np.polyfit(x, y, 1)
    res["fit_us_per_transition"] = float(slope)
    res["fit_us_per_launch_fixed"] = float(icpt)
    if a.quick:
        print(json.dumps(res))
        if a.out:
            json.dump(res, open(a.out, "w"), indent=1)
        return
    # host wall of the timed region at K = 20 (run + device synchronize)
    walls, kern = [], []
    for _ in range(a.reps):
        _lib.check(lib.gm_device_synchronize())
        t0 = time.perf_counter()
        s.run_positions(20, 0)
        _lib.check(lib.gm_device_synchronize())
        walls.append((time.perf_counter() - t0) * 1e6)
        kern.append(s.last_run_stats()[0] * 1e3)
    res["K20_wall_us"] = med(walls)
    res["K20_kernel_us"] = med(kern)
    res["K20_host_overhead_us"] = med(np.array(walls) - np.array(kern))
    # zero-transition call (no launch) and a bare ctypes round trip
    z = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        s.run_positions(0, 0)
        z.append((time.perf_counter() - t0) * 1e6)
    res["run0_us"] = med(z)
    import ctypes as Ct
    li, el = Ct.c_int32(), Ct.c_int32()
    b = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        lib.gm_sampler_layout(s._h, Ct.byref(li), Ct.byref(el))
        b.append((time.perf_counter() - t0) * 1e6)
    res["ctypes_call_us"] = med(b)
    sy = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        lib.gm_device_synchronize()
        sy.append((time.perf_counter() - t0) * 1e6)
    res["idle_device_sync_us"] = med(sy)
    # L = 0: the per-transition cost outside the leapfrog loop
    s0 = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(C, D, 42, np.float64).astype(np.float32), 0.01, 0).set_seed(1)
    s0.reserve(200)
    s0.run_positions(0, 5)
    l0 = {}
    for _ in range(3):
        for k in (20, 100, 200):
            s0.run_positions(k, 0)
            l0.setdefault(k, []).append(s0.last_run_stats()[0] * 1e3)
    res["L0_kernel_us_by_K"] = {k: med(v) for k, v in l0.items()}
    res["env"] = {k: os.environ.get(k) for k in ("GM_SYNC_SPIN", "HIP_FORCE_DEV_KERNARG")}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
