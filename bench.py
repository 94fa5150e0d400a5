"""Benchmark: many-chain HMC on RosenbrockND, 64 dims, f32 (BASELINE.json
configs[1]: 4096 chains per GPU; eps 0.01, L = 50, the reference's own
high-dimensional Rosenbrock settings, hmc.rs:763-780).

A "step" is one HMC transition of every chain (L leapfrogs each). The timed
region runs --steps transitions with every state collected on the device,
bracketed by a barrier and a device synchronize on both sides; the time is
the maximum over ranks. Then the split-R-hat / ESS of the collected draws is
computed on the GPUs (RCCL all-gather of per-split-chain summaries when N > 1).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
VALU_F32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--chains", type=int, default=4096, help="chains per GPU")
    p.add_argument("--dim", type=int, default=64)
    p.add_argument("--leapfrog", type=int, default=50)
    p.add_argument("--eps", type=float, default=0.01)
    p.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    p.add_argument("--layout", default="", help="lanes,elems override")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="target CPU time of the oracle baseline sample (0 disables)")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--north-star", action="store_true",
                   help="also time BASELINE.json north_star's 16384-chain shape (off by default, so that "
                        "every hmc_kernel launch of the default run has the bench's shape)")
    return p.parse_args()


def main():
    a = parse()
    import general_mcmc_amd as gm
    from general_mcmc_amd import _lib
    from general_mcmc_amd.distributed import Comm, ControlPlane, shard

    cp = ControlPlane()  # gloo control plane when launched by torchrun
    world, rank = cp.world, cp.rank
    lib = _lib.load()
    _lib.check(lib.gm_set_device(cp.local_rank))
    lib = _lib.require_gpu()

    dtype = np.float32 if a.dtype == "f32" else np.float64
    s_bytes = np.dtype(dtype).itemsize
    D, L = a.dim, a.leapfrog
    C_glob = a.chains * world
    offset, C_loc = shard(C_glob, world, rank)
    x0 = gm.init_with_seed(C_glob, D, 42, np.float64)[offset:offset + C_loc].astype(dtype)
    sampler = gm.HMC(gm.RosenbrockND(), x0, a.eps, L, dtype=dtype, chain_offset=offset).set_seed(42)
    if a.layout:
        sampler.set_layout(*[int(v) for v in a.layout.split(",")])
    lanes, elems = sampler.layout()
    comm = Comm(cp, lib) if world > 1 else None

    def barrier_sync():
        _lib.check(lib.gm_device_synchronize())
        cp.barrier()

    # the sample buffer is resident before the clock starts, like the state
    sampler.reserve(a.steps)
    # warmup = burn-in transitions (untimed)
    if a.warmup > 0:
        sampler.run_positions(0, a.warmup)
    barrier_sync()
    t0 = time.perf_counter()
    ds = sampler.run_positions(a.steps, 0)
    # each rank's clock stops at its own device synchronize; the closing
    # barrier follows, so its (gloo, host-network) latency is not charged to
    # the GPU time, and the max over ranks below is the slowest rank's time
    _lib.check(lib.gm_device_synchronize())
    t_local = time.perf_counter() - t0
    cp.barrier()
    kernel_ms, launches = sampler.last_run_stats()
    t_max, launch_ms = cp.max([t_local, kernel_ms / max(launches, 1)])

    # diagnostics on the collected draws (device; RCCL all-gather when N > 1)
    td0 = time.perf_counter()
    if a.steps >= 4:
        rhat, ess = comm.split_rhat_ess(ds) if comm is not None else ds.split_rhat_ess()
    else:
        rhat = ess = np.full(D, np.nan, dtype=np.float32)
    t_diag = time.perf_counter() - td0

    # throughput: chain-leapfrogs per second over the whole job
    value = C_glob * L * a.steps / t_max
    # roofline of the dominant kernel: algorithmic bytes per launch (BASELINE.md
    # "Roofline accounting"): per transition and chain
    #   B_step = L (6D+1) s + (4D+2) s + D s (collected)
    b_step = (L * (6 * D + 1) + (4 * D + 2) + D) * s_bytes
    steps_per_launch = a.steps / max(launches, 1)
    bytes_per_launch = b_step * C_loc * steps_per_launch
    achieved_gbs = bytes_per_launch / (launch_ms * 1e-3) / 1e9
    flops_lf = 15 * (D - 1) + 6 * D  # RosenbrockND logp+grad and kick/drift/kick per chain-leapfrog
    achieved_tflops = flops_lf * C_loc * L * steps_per_launch / (launch_ms * 1e-3) / 1e12

    # PMC-derived figures of this exact launch shape (profiles/, from the
    # rocprofv3 passes of tools/profile_bench.sh and tools/pmc_sq.sh)
    key = f"C{C_loc}_D{D}_L{L}_K{a.steps}_{a.dtype}"

    def pmc(name):
        path = os.path.join(ROOT, "profiles", name)
        try:
            return json.load(open(path)).get(key) if os.path.exists(path) else None
        except Exception:
            return None

    tr = pmc("pmc_traffic.json")
    traffic = tr["hbm_bytes_per_launch"] if tr else None
    vi = pmc("pmc_valu.json")
    valu_issue = None if not vi else {
        "frac": vi["issue_frac"], "frac_at_2p4ghz": vi["issue_frac_at_2p4ghz"],
        "valu_insts_per_wave": vi["valu_insts_per_wave"], "clock_ghz": vi["clock_ghz"],
        "note": "SQ_INSTS_VALU x 2 cycles (wave64 on SIMD-32) / (1024 SIMDs x kernel cycles)"}

    copy_gbs = copy_ceiling(lib) if rank == 0 else None
    ns = north_star_check(gm, a, dtype) if rank == 0 and world == 1 and a.north_star else None
    host_out = host_output_rate(lib, sampler, a) if rank == 0 and world == 1 else None
    per_lf = per_leapfrog_hbm(a, dtype) if rank == 0 and world == 1 else None

    cpu = None
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        cpu = cpu_baseline(gm, a, dtype, x0, lanes, elems)

    if rank == 0:
        line = {
            "metric": "leapfrog steps/sec (whole node) + ESS/sec, 64-dim Rosenbrock HMC at 1/2/4/8 GPUs",
            "value": value,
            "unit": "chain-leapfrog steps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": t_max * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic (init: iid N(0,1) Philox seed 42; target RosenbrockND a=1 b=100)",
            "config": {"workload": f"HMC RosenbrockND dim={D}, {C_loc} chains/GPU ({C_glob} total), "
                                   f"eps={a.eps}, n_leapfrog={L}, all {a.steps} transitions collected",
                       "chains_per_gpu": C_loc, "dim": D, "n_leapfrog": L, "step_size": a.eps,
                       "layout": f"{lanes}x{elems}", "parallelism": f"chains sharded x{world}"},
            "ess_per_sec": fin(np.mean(ess) / t_max),
            "ess_min_per_sec": fin(np.min(ess) / t_max),
            "ess": {"min": fin(np.min(ess)), "mean": fin(np.mean(ess))},
            "rhat": {"min": fin(np.min(rhat)), "max": fin(np.max(rhat))},
            "diag_seconds": t_diag,
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "hmc_kernel", "launch_ms": launch_ms,
                         "note": "achieved = SURVEY 8(d) algorithmic bytes (q, p, g round-trip HBM every "
                                 "leapfrog) / launch time; the fused kernel keeps the state in VGPRs "
                                 "(traffic = the PMC bytes it moves, mostly the collected samples), so "
                                 "frac > 1; its real bound is VALU issue (valu); the HBM-bound "
                                 "per-leapfrog formulation is per_leapfrog_hbm",
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "valu": {"achieved_tflops": achieved_tflops,
                                  "peak_tflops": VALU_F32_PEAK_TFLOPS,
                                  "frac": achieved_tflops / VALU_F32_PEAK_TFLOPS,
                                  "issue": valu_issue},
                         "copy_ceiling_gbs": copy_gbs,
                         "per_leapfrog_hbm": per_lf},
            "cpu_baseline": cpu,
            "north_star_check": ns,
            "host_output": host_out,
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    sampler.close()
    cp.close()


def per_leapfrog_hbm(a, dtype, chains=1 << 20, reps=20):
    """The unfused, per-leapfrog design the HBM roofline is written for
    (SURVEY.md §8(d)): gm_bv_leapfrog, one kernel per leapfrog with q, p, g
    and logp in HBM, at an HBM-resident size (2^20 chains: 256 MiB per
    array); achieved = B_alg (6D+1)*s per chain-leapfrog x chains / time."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        from hbm_leapfrog import measure
        r = measure(chains, a.dim, dtype, reps)
    except Exception as e:  # reported, never fatal to the bench line
        return {"error": str(e)}
    return {"kernel": "leapfrog_hbm_kernel", "chains": chains, "achieved": r["achieved_gbs"],
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": r["hbm_frac"], "us_per_leapfrog": r["us_per_leapfrog"],
            "chain_leapfrogs_per_s": r["chain_leapfrogs_per_s"]}


def host_output_rate(lib, sampler, a):
    """The same transitions through gm_run (HMC::run, hmc.rs:164-181): the
    [C, N, D] sample returned in a host array (device transpose + D2H into
    pageable memory). The PCIe-inclusive rate; never `value`."""
    from general_mcmc_amd import _lib
    sampler.run(a.steps, 0)  # warm (host array, staging buffers)
    _lib.check(lib.gm_device_synchronize())
    t0 = time.perf_counter()
    out = sampler.run(a.steps, 0)
    t = time.perf_counter() - t0
    C, N, D = out.shape
    return {"chain_leapfrogs_per_s": C * a.leapfrog * N / t, "seconds": t,
            "sample_bytes": int(out.nbytes), "d2h_gbs_incl_sampling": out.nbytes / t / 1e9}


def north_star_check(gm, a, dtype, chains=16384):
    """BASELINE.json north_star's target shape: >= 10^4 chains of 64-D
    Rosenbrock HMC on one GPU (same eps, L and collection as the bench; device
    time of one launch). Reported beside the headline, never as `value`."""
    D, L, n = a.dim, a.leapfrog, 100
    s = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(chains, D, 43, np.float64).astype(dtype),
               a.eps, L, dtype=dtype).set_seed(43)
    try:
        s.reserve(n)
        s.run_positions(0, 20)
        s.run_positions(n, 0)
        ms, launches = s.last_run_stats()
    finally:
        s.close()
    sb = np.dtype(dtype).itemsize
    b_step = (L * (6 * D + 1) + (4 * D + 2) + D) * sb
    gbs = b_step * chains * n / (ms * 1e-3) / 1e9
    return {"chains": chains, "chain_leapfrogs_per_s": chains * L * n / (ms * 1e-3),
            "launch_ms": ms / max(launches, 1), "hbm_equiv_gbs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS,
            "target": ">= 1e4 chains at >= 50% of the HBM-read roofline (BASELINE.json north_star)"}


def fin(v):
    """float, or None where undefined (diagnostics need >= 4 draws): keeps the
    JSON line strict."""
    v = float(v)
    return v if np.isfinite(v) else None


def copy_ceiling(lib, nbytes=1 << 30, reps=5):
    """Empirical HBM ceiling on this box: a 1 GiB
    device-to-device copy, read + write bytes over the median time."""
    import ctypes as C
    from general_mcmc_amd import _lib
    src, dst = C.c_void_p(), C.c_void_p()
    try:
        _lib.check(lib.gm_malloc(C.byref(src), nbytes))
        _lib.check(lib.gm_malloc(C.byref(dst), nbytes))
        ts = []
        for _ in range(reps + 1):
            _lib.check(lib.gm_device_synchronize())
            t0 = time.perf_counter()
            _lib.check(lib.gm_memcpy_dtod(dst, src, nbytes))
            _lib.check(lib.gm_device_synchronize())
            ts.append(time.perf_counter() - t0)
        return 2 * nbytes / float(np.median(ts[1:])) / 1e9
    except Exception:
        return None
    finally:
        for p in (src, dst):
            if p.value:
                lib.gm_free(p)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(gm, a, dtype, x0, lanes, elems):
    """The CPU oracle (plain-C restatement of batched_hmc.rs, multithreaded over
    chains like the reference's rayon par_iter) timed on a bounded sample of the
    same workload: all chains, a few transitions."""
    from tests import _oracle
    ora = _oracle.load()
    threads = a.cpu_threads or min(16, os.cpu_count() or 1)
    t = _oracle.Target(1, a.dim, a=1.0, b=100.0)
    q = np.array(x0, copy=True)
    t0 = time.perf_counter()
    ora.hmc_run(t, q, a.eps, a.leapfrog, 42, 0, 1, 1, lanes, elems, threads=threads)
    one = time.perf_counter() - t0
    steps = max(1, int(a.cpu_seconds / max(one, 1e-6)))
    t0 = time.perf_counter()
    ora.hmc_run(t, q, a.eps, a.leapfrog, 42, 1, steps, steps, lanes, elems, threads=threads)
    dt = time.perf_counter() - t0
    # one thread on a slice of the chains (the reference's per-core rate)
    n1 = max(1, x0.shape[0] // threads)
    q1 = np.array(x0[:n1], copy=True)
    t0 = time.perf_counter()
    ora.hmc_run(t, q1, a.eps, a.leapfrog, 42, 1, steps, steps, lanes, elems, threads=1)
    dt1 = time.perf_counter() - t0
    return {"value": x0.shape[0] * a.leapfrog * steps / dt, "unit": "chain-leapfrog steps/s",
            "cores": threads, "kind": "port",
            "sample": f"{x0.shape[0]} chains x {steps} transitions x {a.leapfrog} leapfrogs "
                      f"(oracle/gm_oracle.c, {threads} threads, {dt:.1f}s)",
            "one_thread_value": n1 * a.leapfrog * steps / dt1,
            "host": {"cpu_model": _cpu_model(), "nproc": os.cpu_count()}}


if __name__ == "__main__":
    main()
