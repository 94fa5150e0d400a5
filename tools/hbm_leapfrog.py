"""The per-leapfrog design on the HBM roofline: gm_bv_leapfrog (one kernel
per leapfrog, q, p, g and logp round-tripping HBM) timed at an HBM-resident
size (default 2^20 chains x 64-D f32 = 256 MiB per array, SURVEY.md §7 "Roofline
honesty") and at the bench's 4096 chains, against B_alg = (6D+1)*sizeof(T)
bytes per chain-leapfrog and the 8 TB/s HBM peak.

    python tools/hbm_leapfrog.py [--chains 1048576] [--dim 64] [--reps 20]
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
from general_mcmc_amd import batch_vector as bv  # noqa: E402

HBM_PEAK_GBS = 8000.0


def measure(C, D, dtype, reps):
    lib = _lib.require_gpu()
    x0 = gm.init_with_seed(C, D, 42, np.float64).astype(dtype)
    t = bv.BatchTarget(gm.RosenbrockND(), D, dtype)
    q = bv.DeviceMatrix.from_host(x0)
    p = bv.DeviceMatrix.from_host(np.zeros_like(x0))
    g = bv.DeviceMatrix.like(q)
    lp = t.logp_and_grad(q, g)
    for _ in range(3):
        t.leapfrog(q, p, g, lp, 1e-4)
    _lib.check(lib.gm_device_synchronize())
    t0 = time.perf_counter()
    for _ in range(reps):
        t.leapfrog(q, p, g, lp, 1e-4)
    _lib.check(lib.gm_device_synchronize())
    dt = (time.perf_counter() - t0) / reps
    s = np.dtype(dtype).itemsize
    gbs = (6 * D + 1) * s * C / dt / 1e9
    return {"chains": C, "dim": D, "dtype": np.dtype(dtype).name, "us_per_leapfrog": dt * 1e6,
            "chain_leapfrogs_per_s": C / dt, "achieved_gbs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS,
            "bytes_per_chain_leapfrog": (6 * D + 1) * s, "note": "wall time per launch (back-to-back launches)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=1 << 20)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    out = [measure(a.chains, a.dim, np.float32, a.reps), measure(4096, a.dim, np.float32, a.reps * 10)]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
