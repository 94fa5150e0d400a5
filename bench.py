"""Benchmark: many-chain HMC on RosenbrockND, 64 dims, f32 (BASELINE.json
configs[1]: 4096 chains per GPU; eps 0.01, L = 50, the reference's own
high-dimensional Rosenbrock settings, hmc.rs:763-780).

A "step" is one HMC transition of every chain (L leapfrogs each). The timed
region runs --steps transitions with every state collected on the device,
bracketed by a barrier and a device synchronize on both sides; the time is
the maximum over ranks. The split-R-hat / ESS of those draws follows (RCCL
all-gather of per-split-chain summaries when N > 1), and a separately timed
ESS leg runs cfg2's own schedule (n_discard 100, n_collect 100; hmc.rs:763-780)
from the same start, so that ESS/s does not depend on --steps/--warmup.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints one JSON line (rank 0). Every field of the N = 1 line is also in the
N > 1 line: the rank-0-only measurements (copy ceiling, per-leapfrog HBM
kernel, host-output path, CPU baseline) run on rank 0 after the timed region
while the other ranks wait at the closing barrier.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
VALU_F32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (MI355X_MICROARCH.md, spec)
VALU_F64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (MI355X_MICROARCH.md, spec)
METRIC = "leapfrog steps/sec (whole node) + ESS/sec, 64-dim Rosenbrock HMC at 1/2/4/8 GPUs"
PMC_FILE = os.path.join(ROOT, "profiles", "r06", "pmc_hmc.json")
PMC_CONFIGS_FILE = os.path.join(ROOT, "profiles", "r06", "pmc_configs.json")  # tools/profile_r06.sh


def parse(argv=None):
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
    p.add_argument("--ess-discard", type=int, default=100, help="ESS leg burn-in (cfg2: 100)")
    p.add_argument("--ess-collect", type=int, default=100, help="ESS leg draws (cfg2: 100)")
    p.add_argument("--ess-long-discard", type=int, default=4000,
                   help="second ESS leg: long burn-in toward stationarity (0 disables)")
    p.add_argument("--ess-long-collect", type=int, default=1000)
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="target CPU time of each CPU-baseline sample (0 disables)")
    p.add_argument("--cpu-threads", type=int, default=0, help="0: every core available to this process")
    p.add_argument("--cpu-config-seconds", type=float, default=3.0,
                   help="target CPU time of each config leg's CPU-baseline sample (0 disables)")
    p.add_argument("--device-warmup-ms", type=float, default=50.0,
                   help="untimed scratch launches of the timed shape for this long before the W warm-up "
                        "transitions: the GPU clock ramps to its peak within ~10-30 ms of load "
                        "(tools/probe_warmup.py, profiles/r03/warmup_probe.json)")
    p.add_argument("--no-north-star", dest="north_star", action="store_false",
                   help="skip the north_star 16384-chain shape (timed by default after the bench line's "
                        "measurements)")
    p.add_argument("--configs", default="cfg3,cfg3_dense,cfg4,cfg5",
                   help="BASELINE.json config legs timed after the headline (comma list, '' for none)")
    return p.parse_args(argv)


def _build_info():
    """The library's embedded source digest against this tree's (the loader
    refuses a mismatch; recorded so the line names the sources it measured)."""
    try:
        import general_mcmc_amd as gm
        return gm._lib.build_info()
    except Exception as e:  # the CPU-stubbed CLI tests have no library
        return {"error": str(e)}


def dense_gauss_32():
    """configs[2]'s target: mean 0, Sigma = Q diag(logspace(-1, 1,
    32)) Q^T with Q from the QR of a seed-42 N(0,1) 32x32 matrix."""
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((32, 32)))
    cov = q @ np.diag(np.logspace(-1, 1, 32)) @ q.T
    return np.zeros(32), 0.5 * (cov + cov.T)


# The BASELINE.json configs other than the headline, each a leg of its own
# (per-GPU share; chains sharded over the ranks like the headline, R-hat/ESS
# over every rank's chains through the RCCL all-gather when N > 1).
CONFIG_LEGS = {
    # configs[2]: NUTS, DenseGaussian 32-D f64, 8192 chains per GPU; NUTS::run
    # (nuts.rs:214-259) of 500 collected after 500 warm-up transitions
    "cfg3": dict(kind="nuts", chains=8192, dim=32, dtype="f64", n_discard=500, n_collect=500,
                 target_accept=0.8, max_depth=10),
    # the same with GenericNUTS::new_with_mass_matrix's dense metric adaptation
    # during the warm-up (generic_nuts.rs:33-359)
    "cfg3_dense": dict(kind="nuts", chains=8192, dim=32, dtype="f64", n_discard=500, n_collect=500,
                       target_accept=0.8, max_depth=10, mass="dense"),
    # configs[3]: batched HMC, RosenbrockND 128-D f32, 65,536 chains over 8 GPUs
    "cfg4": dict(kind="hmc", chains=8192, dim=128, dtype="f32", n_discard=100, n_collect=100,
                 eps=0.01, L=50),
    # configs[4]: MH IsotropicGaussian(1) 256-D f64, proposal sd 2.38/16,
    # 131,072 chains over 8 GPUs
    "cfg5": dict(kind="mh", chains=16384, dim=256, dtype="f64", n_discard=1000, n_collect=100,
                 proposal_std=2.38 / 16),
}


def f_alg_rosenbrock(D):
    """RosenbrockND logp+grad ~15 flops per coupled pair, two
    kicks and a drift 6 per coordinate: flops per chain-leapfrog."""
    return 15 * (D - 1) + 6 * D


def b_step(D, L, s_bytes):
    """SURVEY 8(d) / BASELINE.md algorithmic bytes per chain-transition of
    the per-leapfrog (state in HBM) formulation, collected step."""
    return (L * (6 * D + 1) + (4 * D + 2) + D) * s_bytes


# --------------------------------------------------------------------------
# The GPU side (libgmcmc through the Python facade). The test suite replaces
# this class with a stub to run main()'s aggregation and JSON assembly under
# gloo with world_size 2 on the CPU (tests/test_bench_cpu.py).
class GpuBench:
    def __init__(self, a, cp):
        import general_mcmc_amd as gm
        from general_mcmc_amd import _lib
        self.gm, self._lib, self.a, self.cp = gm, _lib, a, cp
        lib = _lib.load()
        import ctypes
        n_dev = ctypes.c_int(0)
        _lib.check(lib.gm_device_count(ctypes.byref(n_dev)))
        if cp.local_rank >= n_dev.value:
            raise SystemExit(f"bench.py: rank {cp.rank} needs GPU {cp.local_rank} but {n_dev.value} "
                             f"device(s) are visible (--gpus {a.gpus})")
        _lib.check(lib.gm_set_device(cp.local_rank))
        self.lib = _lib.require_gpu()
        self.dtype = np.float32 if a.dtype == "f32" else np.float64

    def init_positions(self, n, offset, count):
        return self.gm.init_with_seed(count, self.a.dim, 42, np.float64, row0=offset).astype(self.dtype)

    def config_leg(self, name, cfg, offset, comm):
        """One BASELINE config on this rank's share: the run timed between
        device synchronizes (warm-up transitions included, as the reference's
        run(n_collect, n_discard)), the kernels' HIP-event time, the work
        counted on the device, then the device diagnostics of the collected
        draws (the RCCL all-gather when N > 1). Returns this rank's figures;
        main() aggregates."""
        gm = self.gm
        dt = np.float32 if cfg["dtype"] == "f32" else np.float64
        C, D = cfg["chains"], cfg["dim"]
        x0 = gm.init_with_seed(C, D, 42, np.float64, row0=offset).astype(dt)
        s = self._same_kind(cfg, dt, x0, offset, 42)
        try:
            # untimed: one transition of the same kernel on a scratch copy of the
            # sampler (its own chains and buffers), so that the timed run does
            # not include the kernel's first-launch cost (code-object load; 3-4
            # ms on the cfg5 MH leg before this warm-up, profiles/r03/final)
            w = self._same_kind(cfg, dt, x0, offset, 7)
            try:
                w.set_layout(*s.layout())
                w.run_positions(1, 0)
                self.sync()
            finally:
                w.close()
            s.reserve(cfg["n_collect"])
            lf0 = int(s.leapfrog_counts().sum())
            self.sync()
            self.cp.barrier()
            t0 = time.perf_counter()
            warm = None
            if cfg["kind"] == "nuts":
                # NUTS::run(n_collect, n_discard) as its two phases: run(1,
                # n_discard) adapts the step size over the n_discard warm-up
                # transitions, then run(n_collect, 0) takes the n_collect - 1
                # sampling transitions at eps_bar (row 0 = the warm-up's end
                # state): the same 999 transitions and rows as the single
                # call (nuts.rs:232-257; generic_nuts.rs:882-924), with the
                # sampling phase timed on its own
                s.run_positions(1, cfg["n_discard"])
                self.sync()
                t_w = time.perf_counter() - t0
                kms_w, _ = s.last_run_stats()
                lf_w = int(s.leapfrog_counts().sum()) - lf0
                warm = {"warmup_s": t_w, "warmup_kernel_ms": kms_w, "warmup_leapfrogs": lf_w}
                lf0 += lf_w
                t0 = time.perf_counter()
                ds = s.run_positions(cfg["n_collect"], 0)
            else:
                ds = s.run_positions(cfg["n_collect"], cfg["n_discard"])
            self.sync()
            t_run = time.perf_counter() - t0
            kernel_ms, launches = s.last_run_stats()
            leapfrogs = int(s.leapfrog_counts().sum()) - lf0
            accept = float(s.accept_counts().mean())
            self.cp.barrier()
            t0 = time.perf_counter()
            rhat, ess = self.diagnostics(ds, comm)
            t_diag = time.perf_counter() - t0
        finally:
            s.close()
        out = {"run_s": t_run, "kernel_ms": kernel_ms, "launches": launches, "leapfrogs": leapfrogs,
               "accepts_per_chain": accept, "diag_s": t_diag, "rhat": rhat, "ess": ess}
        if warm:
            out.update(warm)
        return out

    def _same_kind(self, cfg, dt, x0, offset, seed):
        """A sampler of the config's kind, dtype and shape (BASELINE.json configs)."""
        gm = self.gm
        if cfg["kind"] == "nuts":
            mean, cov = dense_gauss_32()
            s = gm.NUTS(gm.DenseGaussian(mean, cov), x0, cfg["target_accept"], dtype=dt,
                        max_depth=cfg["max_depth"], chain_offset=offset).set_seed(seed)
            if cfg.get("mass"):
                s.set_mass_adaptation(gm.NUTSMassMatrixConfig(cfg["mass"]))
            return s
        if cfg["kind"] == "hmc":
            return gm.HMC(gm.RosenbrockND(), x0, cfg["eps"], cfg["L"], dtype=dt, chain_offset=offset).set_seed(seed)
        return gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(cfg["proposal_std"]),
                                     x0, dtype=dt, chain_offset=offset).seed(seed)

    def sampler(self, x0, offset):
        a = self.a
        s = self.gm.HMC(self.gm.RosenbrockND(), x0, a.eps, a.leapfrog, dtype=self.dtype,
                        chain_offset=offset).set_seed(42)
        if a.layout:
            s.set_layout(*[int(v) for v in a.layout.split(",")])
        return s

    def sync(self):
        self._lib.check(self.lib.gm_device_synchronize())

    def comm(self):
        from general_mcmc_amd.distributed import Comm
        return Comm(self.cp, self.lib) if self.cp.world > 1 else None

    def diagnostics(self, ds, comm):
        return comm.split_rhat_ess(ds) if comm is not None else ds.split_rhat_ess()

    def copy_ceiling(self, nbytes=1 << 30, reps=5):
        """Empirical HBM ceiling on this box: a 1 GiB
        device-to-device copy by the engine's 16-byte copy kernel
        (gm_memcpy_dtod, util_kernels.hip copy16_kernel), read + write bytes
        over the median time."""
        import ctypes as C
        lib, _lib = self.lib, self._lib
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

    def per_leapfrog_hbm(self, chains=1 << 20, reps=20):
        """The unfused, per-leapfrog design the HBM roofline is written for
        (SURVEY.md 8(d)): gm_bv_leapfrog, one kernel per leapfrog with q, p,
        g and logp in HBM, at an HBM-resident size (2^20 chains: 256 MiB per
        array); achieved = B_alg (6D+1)*s per chain-leapfrog x chains / time."""
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        try:
            from hbm_leapfrog import measure
            r = measure(chains, self.a.dim, self.dtype, reps)
        except Exception as e:  # reported, never fatal to the bench line
            return {"error": str(e)}
        return {"kernel": "leapfrog_hbm_kernel", "chains": chains, "achieved": r["achieved_gbs"],
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": r["hbm_frac"],
                "us_per_leapfrog": r["us_per_leapfrog"], "chain_leapfrogs_per_s": r["chain_leapfrogs_per_s"]}

    def host_output(self, sampler):
        """The same transitions through gm_run (HMC::run, hmc.rs:164-181):
        the [C, N, D] sample returned in a host array (device transpose + D2H
        into pageable memory). The PCIe-inclusive rate; never `value`."""
        a = self.a
        sampler.run(a.steps, 0)  # warm (host array, staging buffers)
        self.sync()
        t0 = time.perf_counter()
        out = sampler.run(a.steps, 0)
        t = time.perf_counter() - t0
        C, N, D = out.shape
        return {"chain_leapfrogs_per_s": C * a.leapfrog * N / t, "seconds": t,
                "sample_bytes": int(out.nbytes), "d2h_gbs_incl_sampling": out.nbytes / t / 1e9}

    def ess_leg(self, x0, offset, comm, n_discard, n_collect):
        """cfg2's schedule from the bench's start: a fresh sampler,
        run_positions(n_collect, n_discard) timed (burn-in included, as the
        reference's run(100, 100)), then the device diagnostics timed on
        their own. Returns this rank's times; the caller takes the max."""
        s = self.sampler(x0, offset)
        try:
            s.reserve(n_collect)
            self.sync()
            self.cp.barrier()
            t0 = time.perf_counter()
            ds = s.run_positions(n_collect, n_discard)
            self.sync()
            t_sample = time.perf_counter() - t0
            self.cp.barrier()
            t0 = time.perf_counter()
            rhat, ess = self.diagnostics(ds, comm)
            t_diag = time.perf_counter() - t0
        finally:
            s.close()
        return t_sample, t_diag, rhat, ess

    def north_star_check(self, chains=16384, offset=0):
        """BASELINE.json north_star's target shape: >= 10^4 chains of 64-D
        Rosenbrock HMC on one GPU (device time of one launch)."""
        a, gm = self.a, self.gm
        D, L, n = a.dim, a.leapfrog, 100
        s = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(chains, D, 43, np.float64, row0=offset).astype(self.dtype),
                   a.eps, L, dtype=self.dtype, chain_offset=offset).set_seed(43)
        try:
            s.reserve(n)
            s.run_positions(0, 20)
            s.run_positions(n, 0)
            ms, launches = s.last_run_stats()
        finally:
            s.close()
        flops = f_alg_rosenbrock(D) * chains * L * n / (ms * 1e-3) / 1e12
        return {"chains": chains, "chain_leapfrogs_per_s": chains * L * n / (ms * 1e-3),
                "launch_ms": ms / max(launches, 1), "valu_tflops": flops,
                "valu_frac": flops / VALU_F32_PEAK_TFLOPS}

    def cpu_baseline(self, x0, lanes, elems):
        return cpu_baseline(self.a, self.dtype, x0, lanes, elems)


# --------------------------------------------------------------------------
def available_cores():
    """Cores this process may use, with the evidence: the affinity mask and
    the cgroup v2 (or v1) CPU quota; the smaller bounds the thread count."""
    ev = {}
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    ev["sched_getaffinity"] = aff
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            ev["cgroup_cpu_max"] = f"{q} {per}"
            if q != "max":
                quota = float(q) / float(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            ev["cgroup_v1_cfs"] = f"{q} {per}"
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    ev["cgroup_quota_cores"] = quota
    ev["os_cpu_count"] = os.cpu_count()
    ev["OMP_NUM_THREADS"] = os.environ.get("OMP_NUM_THREADS")
    n = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    return n, ev


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(a, dtype, x0, lanes, elems):
    """The reference's CPU path timed on this host's available cores, on a
    bounded sample of the same workload (all chains, as many transitions as
    fit in about --cpu-seconds each):
      * value: oracle/cpu_hmc.c, a restatement of batched_hmc.rs's step with
        the reference's operation structure (one pass per BatchVector op over
        a chain block, left-to-right sums, euclidean.rs:392-394/447-534),
        gcc -O3 -march=native, threads over chain blocks like rayon's
        par_iter (core.rs:221-225). Not bit-matching (its own momentum
        stream: xoshiro256++ + Box-Muller, the reference's SmallRng family).
      * oracle: the bit-matching C oracle (gcc -O2 -ffp-contract=off, the
        engine's 64-lane summation order), for context."""
    from tests import _oracle
    threads, ev = available_cores()
    if a.cpu_threads:
        threads = a.cpu_threads
    C = x0.shape[0]
    out = {"unit": "chain-leapfrog steps/s", "cores": threads, "kind": "port",
           "host": {"cpu_model": _cpu_model(), **ev}}
    fast = _oracle.cpu_hmc()
    if fast is not None and dtype == np.float32:
        q = np.array(x0, copy=True)
        fast.run(q, a.eps, a.leapfrog, 1, 42, threads)
        t0 = time.perf_counter()
        fast.run(q, a.eps, a.leapfrog, 1, 42, threads)
        one = time.perf_counter() - t0
        steps = max(1, int(a.cpu_seconds / max(one, 1e-6)))
        t0 = time.perf_counter()
        fast.run(q, a.eps, a.leapfrog, steps, 43, threads)
        dt = time.perf_counter() - t0
        out["value"] = C * a.leapfrog * steps / dt
        out["sample"] = (f"{C} chains x {steps} transitions x {a.leapfrog} leapfrogs, oracle/cpu_hmc.c "
                         f"(-O3 -march=native, reference op structure), {threads} threads, {dt:.1f}s")
        # the same restatement on one core (BASELINE.md section 3 asks for 1 thread and all cores)
        t0 = time.perf_counter()
        fast.run(q, a.eps, a.leapfrog, 1, 44, 1)
        one1 = time.perf_counter() - t0
        steps1 = max(1, int(0.5 * a.cpu_seconds / max(one1, 1e-6)))
        t0 = time.perf_counter()
        fast.run(q, a.eps, a.leapfrog, steps1, 45, 1)
        dt1 = time.perf_counter() - t0
        out["one_thread"] = {"value": C * a.leapfrog * steps1 / dt1, "cores": 1,
                             "sample": f"{C} chains x {steps1} transitions x {a.leapfrog} leapfrogs, "
                                       f"oracle/cpu_hmc.c, 1 thread, {dt1:.1f}s"}
    ora = _oracle.load()
    t = _oracle.Target(1, a.dim, a=1.0, b=100.0)
    q = np.array(x0, copy=True)
    t0 = time.perf_counter()
    ora.hmc_run(t, q, a.eps, a.leapfrog, 42, 0, 1, 1, lanes, elems, threads=threads)
    one = time.perf_counter() - t0
    steps = max(1, int(a.cpu_seconds / max(one, 1e-6)))
    t0 = time.perf_counter()
    ora.hmc_run(t, q, a.eps, a.leapfrog, 42, 1, steps, steps, lanes, elems, threads=threads)
    dt = time.perf_counter() - t0
    out["oracle"] = {"value": C * a.leapfrog * steps / dt, "threads": threads,
                     "sample": f"{C} chains x {steps} transitions, oracle/gm_oracle.c (-O2, bit-matching), {dt:.1f}s"}
    if "value" not in out:
        out["value"] = out["oracle"]["value"]
        out["sample"] = out["oracle"]["sample"]
    return out


def _timed_scaled(run_once, seconds):
    """Time run_once(k) (k units of work, returns the work done) at a k
    calibrated so that the timed call takes about `seconds`."""
    k, work = 1, None
    while True:
        t0 = time.perf_counter()
        work = run_once(k)
        dt = time.perf_counter() - t0
        if dt >= 0.2 * seconds or k >= 1 << 20:
            break
        k = max(k + 1, int(k * min(64.0, 0.5 * seconds / max(dt, 1e-4))))
    if dt < 0.5 * seconds:
        k = max(k + 1, int(k * seconds / max(dt, 1e-4)))
        t0 = time.perf_counter()
        work = run_once(k)
        dt = time.perf_counter() - t0
    return k, work, dt


def config_cpu_baseline(name, cfg, threads, seconds):
    """The reference's CPU path for one BASELINE config leg, timed on this
    host at `threads` threads and at 1 thread on a bounded sample (about
    `seconds` each): the C restatements in oracle/ (gm_oracle.c, bit-matching,
    threads over chain blocks as rayon's par_iter over chains, core.rs:221-225
    and generic_nuts.rs:404-412), in the leg's own unit.
      NUTS (cfg3): NUTS::step after step-size warm-up, generic_nuts.rs:755-925;
      NUTS dense (cfg3_dense): GenericNUTS::new_with_mass_matrix's whole run,
        dense warm-up included (the leg's whole_run rate);
      HMC (cfg4): oracle/cpu_hmc.c (batched_hmc.rs:129-190 op structure, -O3);
      MH (cfg5): metropolis_hastings.rs:306-318."""
    from tests import _oracle
    ora = _oracle.load()
    D = cfg["dim"]
    dt = np.float32 if cfg["dtype"] == "f32" else np.float64
    out = {"kind": "port", "cores": threads}

    def both(run, unit, what):
        res = {}
        for th in (threads, 1):
            k, work, secs = _timed_scaled(lambda k: run(k, th), seconds)
            res[th] = (work / secs, k, secs)
        v, k, secs = res[threads]
        out.update(value=v, unit=unit, sample=what(k, threads, secs))
        v1, k1, s1 = res[1]
        out["one_thread"] = {"value": v1, "cores": 1, "sample": what(k1, 1, s1)}
        return out

    if cfg["kind"] == "nuts":
        mean, cov = dense_gauss_32()
        prec = np.linalg.inv(cov)
        t = _oracle.Target(3, D, mean=mean, prec=prec, norm_const=0.0)
        lanes, elems = 16, 2
        if cfg.get("mass"):
            nd = 500  # the leg's warm-up: the default windows end at 450 (generic_nuts.rs:81-359)

            def run(k, th):
                C_ = k * th
                x0 = np.random.default_rng(1).standard_normal((C_, D)).astype(dt)
                st = ora.nuts_state(C_, dt)
                mass = ora.nuts_mass(2, C_, D, dt)
                _, _, _, nlf = ora.nuts_mass_run(t, x0, st, mass, cfg["target_accept"], cfg["max_depth"], 42, 0,
                                                 20, nd, False, lanes, elems, threads=th)
                return float(nlf.sum())
            return both(run, "leapfrog steps/s (whole run, dense warm-up included)",
                        lambda k, th, s: f"{k * th} chains x run(20, {nd}) with dense mass-matrix adaptation, "
                                         f"oracle/gm_oracle.c or_nuts_mass_run, {th} thread(s), {s:.1f}s")
        C_ = 4 * threads
        x0 = np.random.default_rng(1).standard_normal((C_, D)).astype(dt)
        st = ora.nuts_state(C_, dt)
        q, _, _, _ = ora.nuts_run(t, x0, st, cfg["target_accept"], cfg["max_depth"], 42, 0, 1, 100, False,
                                  lanes, elems, threads=threads)  # step-size warm-up (untimed)

        def run(k, th):
            s2 = {kk: np.array(v, copy=True) for kk, v in st.items()}
            _, _, nlf = ora.nuts_step(t, q, s2, cfg["target_accept"], cfg["max_depth"], 42, 1000, k, 100, 100,
                                      lanes, elems, threads=th)
            return float(nlf.sum())
        return both(run, "leapfrog steps/s (sampling phase)",
                    lambda k, th, s: f"{C_} chains x {k} sampling transitions after 100 warm-up, "
                                     f"oracle/gm_oracle.c or_nuts_step, {th} thread(s), {s:.1f}s")
    if cfg["kind"] == "hmc":
        fast = _oracle.cpu_hmc()
        C_ = cfg["chains"]
        q = np.random.default_rng(1).standard_normal((C_, D)).astype(np.float32)

        def run(k, th):
            fast.run(q, cfg["eps"], cfg["L"], k, 42, th)
            return float(C_ * cfg["L"] * k)
        return both(run, "chain-leapfrog steps/s",
                    lambda k, th, s: f"{C_} chains x {k} transitions x {cfg['L']} leapfrogs, oracle/cpu_hmc.c "
                                     f"(-O3, reference op structure), {th} thread(s), {s:.1f}s")
    C_ = cfg["chains"]
    x0 = np.random.default_rng(1).standard_normal((C_, D)).astype(dt)
    t = _oracle.Target(2, D, std=1.0)

    def run(k, th):
        ora.mh_run(t, x0, cfg["proposal_std"], 42, 0, k, k, 64, 4, threads=th)
        return float(C_ * k)
    return both(run, "chain-steps/s",
                lambda k, th, s: f"{C_} chains x {k} steps, oracle/gm_oracle.c or_mh_run (f64, bit-matching), "
                                 f"{th} thread(s), {s:.1f}s")


def load_pmc(C, D, L, dtype, steps):
    """PMC figures of the timed hmc_kernel launch from profiles/r02
    (tools/pmc_hmc.py over rocprofv3 passes of the driver's command). A
    launch of K transitions moves fixed + K x per-transition bytes; figures
    for a K that was not profiled are scaled on that line and marked so."""
    try:
        d = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None, None
    e = d.get(f"C{C}_D{D}_L{L}_{dtype}")
    if not e:
        return None, None
    byk = {int(k): v for k, v in e.get("by_steps", {}).items()}
    traffic = issue = None
    if steps in byk:
        r = byk[steps]
        traffic = {"bytes": r["hbm_bytes_per_launch"], "source": r["source"], "scaled": False}
        issue = dict(r.get("valu", {}), scaled=False) if r.get("valu") else None
        if issue is not None and r.get("pmc_flops") and r.get("launch_us_traced"):
            issue["executed"] = pmc_executed(r, VALU_F32_PEAK_TFLOPS, "fp32_lane_flops")
    elif "fit" in e:
        f = e["fit"]
        traffic = {"bytes": f["fixed_bytes"] + f["bytes_per_transition"] * steps,
                   "source": f["source"], "scaled": True}
    if issue is None and byk:
        k = min(byk, key=lambda k: abs(k - steps))
        if byk[k].get("valu"):
            issue = dict(byk[k]["valu"], scaled=True, measured_at_steps=k)
    return traffic, issue


def fin(v):
    """float, or None where undefined (diagnostics need >= 4 draws)."""
    v = float(v)
    return v if np.isfinite(v) else None


def rhat_block(rhat):
    """Both orientations, and Stan's over the parameters: the maximum is
    parameter 0 on RosenbrockND, whose chains settle in the x0 = +1 or the
    x0 = -1 basin and stay there (R-hat ~ 11 at any burn-in length,
    tools/probe_ess_burnin.py); the median is the mixing of the rest."""
    r = np.asarray(rhat, dtype=np.float64)
    stan = 1.0 / r
    ok = np.isfinite(stan)
    q = (lambda p: fin(np.quantile(stan[ok], p))) if ok.any() else (lambda p: None)
    return {"reference_sqrt_W_over_V": {"min": fin(np.min(r)), "max": fin(np.max(r))},
            "stan_sqrt_V_over_W": {"min": fin(np.min(stan)), "max": fin(np.max(stan)),
                                   "median": q(0.5), "p90": q(0.9),
                                   "frac_below_1p01": float(np.mean(stan[ok] < 1.01)) if ok.any() else None,
                                   "argmax": int(np.argmax(np.where(ok, stan, -np.inf))) if ok.any() else None},
            "max_abs_dev_from_1": fin(np.max(np.abs(stan - 1.0)))}


def f_alg_mh(D):
    """Algorithmic flops of one MH chain-step on the isotropic Gaussian
    (metropolis_hastings.rs:306-318; distributions.rs:378-406): the proposal
    x' = x + sd z (2D), the target's sum of squares and scale (2D + 2), the
    proposal's forward and backward log-densities (3D + 2 each). The D
    normals and the accept uniform are RNG work, counted separately
    (SURVEY 8(d))."""
    return 10 * D + 6


def pmc_executed(r, peak, key):
    """The hardware's own flop count of a profiled dispatch (SQ_INSTS_VALU_
    FLOPS_FP32/FP64 x 64: every lane-flop the VALU executed, FMA as 2, the RNG
    and bookkeeping included, padded lanes excluded) over its traced time,
    against the vector peak: the executed-flop fraction, beside the F_alg
    fraction that counts only the algorithm's flops."""
    fl = r["pmc_flops"][key]
    tf = fl / (r["launch_us_traced"] * 1e-6) / 1e12
    return {"lane_flops_per_launch": fl, "tflops": tf, "frac": tf / peak,
            "note": "SQ_INSTS_VALU_FLOPS x 64 of the profiled dispatch / its traced duration, vs the vector peak"}


def load_pmc_config(name):
    """PMC figures of a config leg's dispatch (profiles/r04/pmc_configs.json,
    tools/profile_r04.sh), or None."""
    try:
        e = json.load(open(PMC_CONFIGS_FILE)).get(name)
    except (OSError, ValueError):
        return None
    if not e or not e.get("by_steps"):
        return None
    k, r = next(iter(e["by_steps"].items()))
    v = r.get("valu", {})
    ex = None
    if r.get("pmc_flops") and r.get("launch_us_traced"):
        f64 = r["pmc_flops"].get("fp64_lane_flops", 0.0) > 0
        ex = pmc_executed(r, VALU_F64_PEAK_TFLOPS if f64 else VALU_F32_PEAK_TFLOPS,
                          "fp64_lane_flops" if f64 else "fp32_lane_flops")
    return {"transitions_per_launch": int(k), "launch_us_traced": r.get("launch_us_traced"),
            "executed_flops": ex,
            "hbm_bytes_per_launch": r.get("hbm_bytes_per_launch"), "issue_frac": v.get("issue_frac"),
            "valu_insts_per_wave": v.get("valu_insts_per_wave"), "salu_per_valu": v.get("salu_per_valu"),
            "wave_wait_frac": v.get("wave_wait_frac"), "clock_ghz": v.get("clock_ghz"), "source": r.get("source")}


def config_summary(name, cfg, figs, world, rhat, ess):
    """Aggregate one config leg over the ranks (max time, summed work) with
    its own roofline: the FP64/FP32 vector peak for NUTS / HMC (F_alg of
    SURVEY 8(d)), the HBM-equivalent bytes for MH (its unit there)."""
    t = max(f["run_s"] for f in figs)
    kms = max(f["kernel_ms"] for f in figs)
    D = cfg["dim"]
    chains = cfg["chains"] * world
    s_bytes = 4 if cfg["dtype"] == "f32" else 8
    total = cfg["n_collect"] + cfg["n_discard"] - (1 if cfg["kind"] == "nuts" else 0)
    out = {"workload": None, "chains_total": chains, "chains_per_gpu": cfg["chains"], "dim": D,
           "dtype": cfg["dtype"], "n_discard": cfg["n_discard"], "n_collect": cfg["n_collect"],
           "transitions": total, "wall_s": t, "kernel_ms": kms,
           "launches": max(f["launches"] for f in figs), "diag_s": max(f["diag_s"] for f in figs),
           "accepts_per_chain": float(np.mean([f["accepts_per_chain"] for f in figs]))}
    if cfg["kind"] == "nuts":
        lf = sum(f["leapfrogs"] for f in figs)
        lf_w = sum(f.get("warmup_leapfrogs", 0) for f in figs)
        t_w = max(f.get("warmup_s", 0.0) for f in figs)
        n_samp = cfg["n_collect"] - 1
        # the target's GEMV and the kicks/drift, 2D^2 + 8D; under
        # a dense metric each leaf adds the ONE M^-1 product the engine does
        # (of the new gradient: M^-1 p is carried by linearity, DESIGN.md §3,
        # where the reference's formulation takes two, generic_nuts.rs:255-273,
        # 1396-1418) and the carried velocity's 4D (the products at transition
        # starts are not counted)
        fa = 2 * D * D + 8 * D + (2 * D * D + 4 * D if cfg.get("mass") == "dense" else 0)
        tf = fa * (lf / world) / (kms * 1e-3) / 1e12
        mass = f", {cfg['mass']} mass-matrix adaptation" if cfg.get("mass") else ""
        out.update(workload=f"NUTS DenseGaussian dim={D} f64, {chains} chains, target_accept "
                            f"{cfg['target_accept']}, max_depth {cfg['max_depth']}{mass}, run({cfg['n_collect']}, "
                            f"{cfg['n_discard']}) as run(1, {cfg['n_discard']}) + run({cfg['n_collect']}, 0)",
                   metric="leapfrog steps/s (sampling phase)", value=lf / t, value_kernel=lf / (kms * 1e-3),
                   leapfrogs=lf, mean_tree_leapfrogs=lf / (chains * n_samp),
                   sampling_transitions=n_samp, sampling_s=t,
                   warmup={"transitions": cfg["n_discard"], "wall_s": t_w, "leapfrogs": lf_w,
                           "kernel_ms": max(f.get("warmup_kernel_ms", 0.0) for f in figs),
                           "leapfrogs_per_s": lf_w / t_w if t_w > 0 else None},
                   whole_run={"wall_s": t + t_w, "leapfrogs_per_s": (lf + lf_w) / (t + t_w)},
                   roofline={"bound": "valu_f64", "kernel": "nuts_kernel", "achieved": tf,
                             "peak": VALU_F64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / VALU_F64_PEAK_TFLOPS,
                             "flops_per_leapfrog": fa,
                             "note": "F = 2D^2 + 8D per leapfrog (SURVEY 8(d)), + 2D^2 + 4D under a dense "
                                     "metric (the leaf's one M^-1 product and the carried M^-1 p), x leapfrogs "
                                     "counted on the device / the run's HIP-event kernel time (per GPU)"})
    elif cfg["kind"] == "hmc":
        work = chains * cfg["L"] * total
        fa = f_alg_rosenbrock(D)
        tf = fa * (work / world) / (kms * 1e-3) / 1e12
        out.update(workload=f"HMC RosenbrockND dim={D} {cfg['dtype']}, {chains} chains, eps {cfg['eps']}, "
                            f"L {cfg['L']}, run({cfg['n_collect']}, {cfg['n_discard']})",
                   metric="chain-leapfrog steps/s", value=work / t, value_kernel=work / (kms * 1e-3),
                   roofline={"bound": "valu", "kernel": "hmc_kernel", "achieved": tf, "peak": VALU_F32_PEAK_TFLOPS,
                             "unit": "TFLOP/s", "frac": tf / VALU_F32_PEAK_TFLOPS, "flops_per_chain_leapfrog": fa})
    else:
        work = chains * total
        b = (2 * D + 2) * s_bytes
        gbs = b * (work / world) / (kms * 1e-3) / 1e9
        fa = f_alg_mh(D)
        tf = fa * (work / world) / (kms * 1e-3) / 1e12
        out.update(workload=f"MH IsotropicGaussian(1) dim={D} f64, proposal sd {cfg['proposal_std']:.5f}, "
                            f"{chains} chains, run({cfg['n_collect']}, {cfg['n_discard']})",
                   metric="chain-steps/s", value=work / t, value_kernel=work / (kms * 1e-3),
                   roofline={"bound": "valu_f64", "kernel": "mh_kernel", "achieved": tf,
                             "peak": VALU_F64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / VALU_F64_PEAK_TFLOPS,
                             "flops_per_chain_step": fa,
                             "rng_normals_per_s": D * (work / world) / (kms * 1e-3),
                             "hbm_equivalent": {"achieved_gbs": gbs, "peak_gbs": HBM_PEAK_GBS,
                                                "frac": gbs / HBM_PEAK_GBS, "bytes_per_chain_step": b},
                             "note": "achieved = F_alg (10D+6 per chain-step: proposal, target and the two "
                                     "proposal log-densities, f_alg_mh) x chain-steps / the run's HIP-event "
                                     "kernel time (per GPU), against the FP64 vector peak. The D Philox/"
                                     "Box-Muller normals per chain-step are RNG work outside F_alg (SURVEY "
                                     "8(d)) and take most of the VALU issue (pmc.issue_frac); the "
                                     "HBM-equivalent is SURVEY 8(d)'s (2D+2)s bytes per chain-step"})
    pm = load_pmc_config(name)
    if pm is not None:
        out["roofline"]["pmc"] = pm
    out["ess_mean"] = fin(np.mean(ess))
    out["ess_min"] = fin(np.min(ess))
    out["ess_per_sec"] = fin(np.mean(ess) / t)
    out["ess_min_per_sec"] = fin(np.min(ess) / t)
    out["rhat"] = rhat_block(rhat)
    out["mixing_note"] = LEG_NOTES.get(name)
    return out


# What the legs' ESS and R-hat say, so that a reader does not take a
# property of the target, the schedule or the reference's metric convention
# for a kernel defect.
LEG_NOTES = {
    "cfg3": "identity metric on the 32-D Gaussian: R-hat within 0.002 of 1 after 500 warm-up transitions",
    "cfg3_dense": "the reference's dense adaptation sets the MASS matrix to the regularised sample covariance "
                  "C (M = C: kinetic p^T C^-1 p / 2, momentum p ~ N(0, C), drift C^-1 p; generic_nuts.rs:209-224, "
                  "255-303, 975-989), the inverse of Stan's convention (M^-1 = C). The drift then scales the "
                  "target's directions by Sigma^-1 instead of Sigma, so this leg mixes worse than the identity "
                  "metric (lower ESS, longer trees) by the reference's own design, reproduced bit for bit; "
                  "pinned by tests/test_gpu_nuts_mass.py::test_dense_metric_convention_is_reference_M_equals_cov",
    "cfg4": "RosenbrockND: the chains settle in the x0 = +1 or x0 = -1 basin and HMC with trajectory length 0.5 "
            "does not cross, so parameter 0's R-hat stays large at any burn-in (a target property, pinned by "
            "tests/test_gpu_statistical.py); 100 + 100 transitions is the configured schedule",
    "cfg5": "random-walk MH with sd 2.38/16 in 256-D: a step moves each coordinate by ~0.15 sd and is accepted "
            "~23 % of the time, so a chain's 100 collected draws span a small part of the target and the "
            "between-chain variance dominates: R-hat ~ 5 on every parameter is the configured schedule's "
            "property (the starts are already N(0, I) draws), not a sampler defect",
}


def pin_host_thread(rank: int, world: int):
    """A single rank's host thread on the CPU it runs on, from the device
    warm-up to the end of the timed region, so that the timed call's launch
    and spin-wait do not migrate between cores: median host path 12.2 ->
    10.8 us, headline +1.8 % over 5 alternating rounds
    (profiles/r06/ab_bench_pin.jsonl, the first allowed CPU); the current
    CPU, 13.7 -> 11.1 us, +3 % (ab_bench_pin_current_cpu.jsonl). Returns the
    previous affinity (restored before the CPU-baseline legs, whose threads
    need every core); BENCH_PIN_CPU=0 turns it off."""
    # (one rank only: several ranks would need their GPUs' NUMA-near cores,
    # which the first allowed CPUs need not be)
    if os.environ.get("BENCH_PIN_CPU", "1") != "1" or world != 1 or not hasattr(os, "sched_setaffinity"):
        return None
    prev = os.sched_getaffinity(0)
    cpu = sorted(prev)[0]
    try:  # the CPU it runs on now (no migration, warm caches)
        import ctypes
        now = ctypes.CDLL(None).sched_getcpu()
        if now in prev:
            cpu = now
    except (OSError, AttributeError):
        pass
    os.sched_setaffinity(0, {cpu})
    return prev


def main(argv=None, backend=None):
    a = parse(argv)
    from general_mcmc_amd.distributed import ControlPlane, shard

    cp = ControlPlane()  # gloo control plane when launched by torchrun
    world, rank = cp.world, cp.rank
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s) "
                         f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')})")
    be = (backend or GpuBench)(a, cp)
    s_bytes = 4 if a.dtype == "f32" else 8
    D, L = a.dim, a.leapfrog
    C_glob = a.chains * world
    offset, C_loc = shard(C_glob, world, rank)
    x0 = be.init_positions(C_glob, offset, C_loc)
    sampler = be.sampler(x0, offset)
    # the measured sampler's runs are asynchronous: run_positions returns once
    # the launch is enqueued, and the timed region's closing device
    # synchronize is its one wait (0.7 us less host path than a stream wait
    # followed by it, profiles/r06/host_path_probe.log V1 vs V2)
    if hasattr(sampler, "set_async"):
        sampler.set_async(True)
    lanes, elems = sampler.layout()
    comm = be.comm()
    if world > 1 and (comm is None or comm.info()["nranks"] != world):
        raise SystemExit(f"bench.py: the RCCL communicator does not span the {world} ranks")

    def barrier_sync():
        be.sync()
        cp.barrier()

    # the sample buffer is resident before the clock starts, like the state;
    # the W warm-up transitions collect into it (untimed)
    sampler.reserve(max(a.steps, a.warmup))
    # device warm-up (untimed): launches of the timed shape on a scratch
    # sampler with its own chains and buffers for --device-warmup-ms (at
    # least two), then the W warm-up transitions of the measured sampler right
    # before the timed call. The GPU clock ramps to its peak only after ~10-30
    # ms of load: after 0.2 ms of warm-up launches the timed 20-transition
    # launch takes 103 us (2.26 GHz), after 30-100 ms 89.5 us
    # (tools/probe_warmup.py, profiles/r03/warmup_probe.json); without the
    # scratch launches the first call of a process is slower still
    # (profiles/r02/first_call/). The measured chains are exactly W
    # transitions from the start.
    affinity = pin_host_thread(rank, world)
    scratch = be.sampler(x0, offset)
    scratch.reserve(a.steps)
    t_warm_end = time.perf_counter() + a.device_warmup_ms * 1e-3
    n_scratch = 0
    while n_scratch < 2 or time.perf_counter() < t_warm_end:
        scratch.run_positions(a.steps, 0)
        n_scratch += 1
    if a.warmup > 0:
        sampler.run_positions(a.warmup, 0)
    barrier_sync()
    t0 = time.perf_counter()
    ds = sampler.run_positions(a.steps, 0)
    # each rank's clock stops at its own device synchronize; the closing
    # barrier follows, so its (gloo) latency is not charged to the GPU time,
    # and the max over ranks below is the slowest rank's time
    be.sync()
    t_local = time.perf_counter() - t0
    if affinity is not None:
        os.sched_setaffinity(0, affinity)
    cp.barrier()
    scratch.close()
    kernel_ms, launches = sampler.last_run_stats()
    ranks = cp.gather({"rank": rank, "wall_ms": t_local * 1e3, "kernel_ms": kernel_ms, "launches": launches})
    t_max = max(r["wall_ms"] for r in ranks) * 1e-3
    kmax = max(r["kernel_ms"] for r in ranks)
    launch_ms = max(r["kernel_ms"] / max(r["launches"], 1) for r in ranks)

    # diagnostics of the timed draws (device; RCCL all-gather when N > 1)
    td0 = time.perf_counter()
    if a.steps >= 4:
        rhat, ess = be.diagnostics(ds, comm)
    else:
        rhat = ess = np.full(D, np.nan, dtype=np.float32)
    t_diag = time.perf_counter() - td0

    # ESS legs on their own schedules (every rank; diagnostics over all chains)
    legs = {}
    for name, nd, nc in (("cfg2_schedule", a.ess_discard, a.ess_collect),
                         ("long", a.ess_long_discard, a.ess_long_collect)):
        if nc < 4 or (name == "long" and nd <= 0):
            continue
        ts, tdg, rh, es = be.ess_leg(x0, offset, comm, nd, nc)
        ts, tdg = cp.max([ts, tdg])
        legs[name] = {"n_discard": nd, "n_collect": nc, "sampling_s": float(ts), "diag_s": float(tdg),
                      "ess_mean": fin(np.mean(es)), "ess_min": fin(np.min(es)),
                      "ess_per_sec_sampling": fin(np.mean(es) / ts),
                      "ess_min_per_sec_sampling": fin(np.min(es) / ts),
                      "ess_per_sec_end_to_end": fin(np.mean(es) / (ts + tdg)),
                      "rhat": rhat_block(rh)}
    # the other BASELINE configs (every rank, its share; diagnostics over all)
    configs = {}
    for name in [c for c in a.configs.split(",") if c]:
        cfg = CONFIG_LEGS[name]
        off, _ = shard(cfg["chains"] * world, world, rank)
        figs = be.config_leg(name, cfg, off, comm)
        rh, es = figs.pop("rhat"), figs.pop("ess")
        configs[name] = config_summary(name, cfg, cp.gather(figs), world, rh, es)
    comm_info = comm.info() if comm is not None else None

    # rank-0-only measurements; the other ranks wait at the closing barrier
    extra = {}
    if rank == 0:
        extra["copy_ceiling_gbs"] = be.copy_ceiling()
        extra["per_leapfrog_hbm"] = be.per_leapfrog_hbm()
        extra["host_output"] = be.host_output(sampler)
        extra["north_star_check"] = be.north_star_check(offset=offset) if a.north_star else None
        extra["cpu_baseline"] = be.cpu_baseline(x0, lanes, elems) if a.cpu_seconds > 0 else None
        if a.cpu_config_seconds > 0:
            threads = a.cpu_threads or available_cores()[0]
            for name in configs:
                configs[name]["cpu_baseline"] = config_cpu_baseline(name, CONFIG_LEGS[name], threads,
                                                                    a.cpu_config_seconds)
    cp.barrier()

    line = None
    if rank == 0:
        value = C_glob * L * a.steps / t_max
        steps_per_launch = a.steps / max(launches, 1)
        fa = f_alg_rosenbrock(D)
        achieved_tf = fa * C_loc * L * steps_per_launch / (launch_ms * 1e-3) / 1e12
        hbm_bytes = b_step(D, L, s_bytes) * C_loc * steps_per_launch
        hbm_gbs = hbm_bytes / (launch_ms * 1e-3) / 1e9
        traffic, issue = load_pmc(C_loc, D, L, a.dtype, a.steps)
        line = {
            "metric": METRIC,
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
            "timing": {"wall_ms": t_max * 1e3, "kernel_ms": kmax, "launches": launches,
                       "host_overhead_ms": t_max * 1e3 - kmax, "per_rank": ranks,
                       "device_warmup": f"{n_scratch} untimed launches of the timed shape on a scratch sampler (own "
                                        f"chains and buffers) for {a.device_warmup_ms:g} ms (GPU clock ramp), then "
                                        "the W warm-up transitions of the measured sampler",
                       "note": "wall = barrier-bracketed timed region (max over ranks); kernel = HIP events "
                               "around the run's launches on the sampler's stream; host_overhead = wall - kernel"},
            "ess_per_sec": legs.get("cfg2_schedule", {}).get("ess_per_sec_sampling"),
            "ess": legs,
            "timed_draws_diagnostics": {"ess_mean": fin(np.mean(ess)), "ess_min": fin(np.min(ess)),
                                        "rhat": rhat_block(rhat), "diag_s": t_diag,
                                        "note": "the --steps draws of the timed region, started "
                                                "--warmup transitions from N(0,1): not a mixing figure"},
            "roofline": {"bound": "valu", "achieved": achieved_tf, "peak": VALU_F32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved_tf / VALU_F32_PEAK_TFLOPS,
                         "traffic": traffic["bytes"] if traffic else None,
                         "kernel": "hmc_kernel", "launch_ms": launch_ms,
                         "flops_per_chain_leapfrog": fa,
                         "algorithmic_flops_per_launch": fa * C_loc * L * steps_per_launch,
                         "note": "achieved = F_alg (15(D-1)+6D per chain-leapfrog, SURVEY 8(d)) x chain-"
                                 "leapfrogs per launch / the launch's HIP-event time; the fused kernel keeps "
                                 "q, p, g in VGPRs, so VALU issue, not HBM, bounds it (traffic = PMC HBM bytes "
                                 "of the launch: the collected samples plus one state read/write)",
                         "traffic_source": traffic,
                         "valu_issue": issue,
                         "pmc_flops_frac": (issue or {}).get("executed", {}).get("frac"),
                         "hbm_equivalent": {"achieved_gbs": hbm_gbs, "peak_gbs": HBM_PEAK_GBS,
                                            "hbm_equivalent_frac": hbm_gbs / HBM_PEAK_GBS,
                                            "algorithmic_bytes_per_launch": hbm_bytes,
                                            "note": "BASELINE.md's per-leapfrog algorithmic bytes (q, p, g "
                                                    "round-trip HBM every leapfrog) over the fused launch's "
                                                    "time: a comparison with the unfused design, not a "
                                                    "roofline fraction"},
                         "copy_ceiling_gbs": extra.get("copy_ceiling_gbs"),
                         "per_leapfrog_hbm": extra.get("per_leapfrog_hbm")},
            "cpu_baseline": extra.get("cpu_baseline"),
            "configs": configs,
            "rccl": comm_info,
            "north_star_check": extra.get("north_star_check"),
            "host_output": extra.get("host_output"),
            "build": _build_info(),
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    sampler.close()
    cp.close()
    return line


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(argv, n: int) -> int:
    """`bench.py --gpus N` (N > 1) started as one plain process: start the N
    ranks as `torch.distributed.run` children (one process per GPU, rendezvous
    on 127.0.0.1) and return their exit status. Nothing here touches the GPU
    or imports the engine, so the children are the only HIP processes; rank 0
    prints the line to the inherited stdout."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd).returncode


def backend_from_env():
    """GMCMC_BENCH_BACKEND=module:factory replaces GpuBench (CPU tests of the
    CLI path, tests/test_bench_cpu.py); unset in every real run."""
    spec = os.environ.get("GMCMC_BENCH_BACKEND")
    if not spec:
        return None
    import importlib
    mod, fn = spec.split(":")
    return getattr(importlib.import_module(mod), fn)()


if __name__ == "__main__":
    _args = parse()
    if _args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if _args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], _args.gpus))
    main(backend=backend_from_env())
