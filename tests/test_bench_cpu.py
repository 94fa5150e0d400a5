"""bench.py's aggregation and JSON assembly, run on the CPU with the GPU calls
stubbed (the GpuBench class replaced): at world_size 2 under gloo -- the path
that produces the driver's multi-GPU SCALE lines -- rank 0 must emit every
field of the world_size 1 line, take the max over ranks, and carry each rank's
timing, the communicator's rank count and the CPU baseline."""
import json
import os
import socket

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGV = ["--steps", "8", "--warmup", "2", "--chains", "128", "--cpu-seconds", "0.05", "--cpu-config-seconds", "0.05",
        "--ess-discard", "4", "--ess-collect", "8", "--ess-long-discard", "4", "--ess-long-collect", "8"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Samples:
    def __init__(self, n, c, d):
        self.n_collect, self.n_chains, self.dim = n, c, d


class _Sampler:
    def __init__(self, x0, rank):
        self.C, self.D, self.rank = x0.shape[0], x0.shape[1], rank

    def layout(self):
        return 64, 1

    def reserve(self, n):
        return self

    def run_positions(self, n, nd):
        return _Samples(n, self.C, self.D)

    def last_run_stats(self):  # rank 1 is the slower one
        return (2.0 if self.rank == 1 else 1.0), 1

    def close(self):
        pass


class _Comm:
    def __init__(self, cp):
        self.cp = cp

    def info(self):
        return {"nranks": self.cp.world, "rank": self.cp.rank, "device": self.cp.local_rank}

    def close(self):
        pass


def stub_backend():
    import bench

    class StubBench:
        def __init__(self, a, cp):
            self.a, self.cp = a, cp

        def init_positions(self, n, offset, count):
            return np.random.default_rng(offset).standard_normal((count, self.a.dim)).astype(np.float32)

        def sampler(self, x0, offset):
            return _Sampler(x0, self.cp.rank)

        def sync(self):
            pass

        def comm(self):
            return _Comm(self.cp) if self.cp.world > 1 else None

        def diagnostics(self, ds, comm):
            return np.full(ds.dim, 0.99, np.float32), np.full(ds.dim, 100.0 * ds.n_chains, np.float32)

        def ess_leg(self, x0, offset, comm, nd, nc):
            r, e = self.diagnostics(_Samples(nc, x0.shape[0], x0.shape[1]), comm)
            return 0.01 * (1 + self.cp.rank), 0.001, r, e

        def copy_ceiling(self):
            return 5000.0

        def per_leapfrog_hbm(self):
            return {"achieved": 5000.0, "frac": 0.625}

        def host_output(self, sampler):
            return {"chain_leapfrogs_per_s": 1.0}

        def north_star_check(self, offset=0):
            return None

        def config_leg(self, name, cfg, offset, comm):
            r, e = self.diagnostics(_Samples(cfg["n_collect"], cfg["chains"], cfg["dim"]), comm)
            k = 1 + self.cp.rank  # rank 1 is the slower one
            out = {"run_s": 0.1 * k, "kernel_ms": 50.0 * k, "launches": 1, "leapfrogs": 1000 * cfg["chains"],
                   "accepts_per_chain": 10.0, "diag_s": 0.01, "rhat": r, "ess": e}
            if cfg["kind"] == "nuts":
                out.update(warmup_s=0.05 * k, warmup_kernel_ms=40.0 * k, warmup_leapfrogs=900 * cfg["chains"])
            return out

        def cpu_baseline(self, x0, lanes, elems):
            return bench.cpu_baseline(self.a, np.float32, x0, lanes, elems)

    return StubBench


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import bench
    line = bench.main(ARGV + ["--gpus", str(world)], backend=stub_backend())
    if rank == 0:
        with open(os.path.join(outdir, f"line{world}.json"), "w") as f:
            json.dump(line, f)
    else:
        assert line is None


def _cli(args, extra_env=None, timeout=300):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(GMCMC_BENCH_BACKEND="tests.test_bench_cpu:stub_backend", **(extra_env or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_cli_gpus2_launches_two_ranks():
    """The driver's own command form, `python bench.py --gpus 2`, started as
    one plain process: bench.py must start two ranks itself (torch.distributed
    .run children) and rank 0's line must describe a 2-rank job."""
    r = _cli(ARGV + ["--gpus", "2"])
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert [p["rank"] for p in line["timing"]["per_rank"]] == [0, 1]
    assert line["rccl"]["nranks"] == 2
    assert line["configs"]["cfg3"]["chains_total"] == 2 * 8192
    assert line["config"]["parallelism"] == "chains sharded x2"


def test_bench_cli_rank_count_mismatch_fails():
    """A launcher that started fewer ranks than --gpus asks for is an error,
    never a silent N = 1 line."""
    r = _cli(ARGV + ["--gpus", "2"], extra_env={"WORLD_SIZE": "1"})
    assert r.returncode != 0
    assert "--gpus 2" in r.stderr and not [l for l in r.stdout.splitlines() if l.startswith("{")]


def _keys(d, prefix=""):
    out = set()
    for k, v in d.items():
        out.add(prefix + k)
        if isinstance(v, dict) and k not in ("ess", "per_rank"):
            out |= _keys(v, prefix + k + ".")
    return out


def test_bench_line_world1_and_world2(tmp_path):
    for world in (1, 2):
        mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                           start_method="spawn", join=True)
    l1 = json.load(open(tmp_path / "line1.json"))
    l2 = json.load(open(tmp_path / "line2.json"))
    # the N = 2 line carries every field of the N = 1 line
    missing = _keys(l1) - _keys(l2)
    assert not missing, missing
    assert l2["n_gpus"] == 2 and l1["n_gpus"] == 1
    # whole-job value over the slowest rank's time; per-rank timing kept
    assert len(l2["timing"]["per_rank"]) == 2
    assert l2["roofline"]["launch_ms"] == 2.0  # the slower rank's kernel
    assert l2["rccl"] == {"nranks": 2, "rank": 0, "device": 0}
    assert l1["rccl"] is None
    for line in (l1, l2):
        assert line["roofline"]["bound"] == "valu" and 0 < line["roofline"]["frac"]
        cb = line["cpu_baseline"]
        assert cb["cores"] >= 1 and cb["value"] > 0 and "sched_getaffinity" in cb["host"]
        assert cb["one_thread"]["cores"] == 1 and cb["one_thread"]["value"] > 0
        assert set(line["ess"]) == {"cfg2_schedule", "long"}
        assert line["ess"]["cfg2_schedule"]["rhat"]["stan_sqrt_V_over_W"]["max"] > 1.0
    # the ESS legs time the slowest rank
    assert l2["ess"]["cfg2_schedule"]["sampling_s"] == 0.02
    # the config legs: every rank's share, the slowest rank's time, work summed
    for line, world in ((l1, 1), (l2, 2)):
        assert set(line["configs"]) == {"cfg3", "cfg3_dense", "cfg4", "cfg5"}
        assert "dense mass-matrix adaptation" in line["configs"]["cfg3_dense"]["workload"]
        c3 = line["configs"]["cfg3"]
        assert c3["chains_total"] == 8192 * world and c3["leapfrogs"] == 1000 * 8192 * world
        assert c3["wall_s"] == 0.1 * world and c3["value"] == c3["leapfrogs"] / c3["wall_s"]
        assert c3["roofline"]["bound"] == "valu_f64" and c3["roofline"]["frac"] > 0
        assert c3["warmup"]["leapfrogs"] == 900 * 8192 * world and c3["warmup"]["wall_s"] == 0.05 * world
        c5 = line["configs"]["cfg5"]
        assert c5["value"] == 16384 * world * 1100 / (0.1 * world)
        assert c5["roofline"]["hbm_equivalent"]["frac"] > 0
        assert line["configs"]["cfg4"]["transitions"] == 200
        # a CPU baseline beside every config leg, at all cores and at 1 thread
        for name, unit in (("cfg3", "leapfrog steps/s (sampling phase)"),
                           ("cfg3_dense", "leapfrog steps/s (whole run, dense warm-up included)"),
                           ("cfg4", "chain-leapfrog steps/s"), ("cfg5", "chain-steps/s")):
            cb = line["configs"][name]["cpu_baseline"]
            assert cb["unit"] == unit and cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
            assert cb["one_thread"]["cores"] == 1 and cb["one_thread"]["value"] > 0
