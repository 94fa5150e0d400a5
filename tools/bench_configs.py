"""Per-GPU measurements of the other BASELINE.json configs (parity-test
workloads, not the bench line): throughput of each sampler kernel at its
config size, with ESS from the device diagnostics.

  cfg3  NUTS, DenseGaussian 32-D f64 (Sigma = Q diag(logspace(-1,1,32)) Q^T,
        Q from QR of a seed-42 N(0,1) matrix), 8192 chains
  cfg4  HMC RosenbrockND 128-D f32, 65536 chains / 8 GPUs = 8192 per GPU
  cfg5  MH IsotropicGaussian(1) 256-D f64, proposal sd 2.38/sqrt(256),
        131072 chains / 8 GPUs = 16384 per GPU
  10k   the reference's test_bench_10000d (6 chains x 10,000-D, wide layout)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import general_mcmc_amd as gm  # noqa: E402


def dense_gauss_32():
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((32, 32)))
    cov = q @ np.diag(np.logspace(-1, 1, 32)) @ q.T
    cov = 0.5 * (cov + cov.T)
    return gm.DenseGaussian(np.zeros(32), cov)


def timed(fn):
    gm._lib.load().gm_device_synchronize()
    t0 = time.perf_counter()
    r = fn()
    gm._lib.load().gm_device_synchronize()
    return r, time.perf_counter() - t0


def cfg3(a):
    C, D = a.nuts_chains, 32
    s = gm.NUTS(dense_gauss_32(), gm.init_det(C, D), 0.8, dtype=np.float64, max_depth=10).set_seed(42)
    if a.nuts_mass != "none":  # GenericNUTS::new_with_mass_matrix's warm-up metric adaptation
        s.set_mass_adaptation(gm.NUTSMassMatrixConfig(a.nuts_mass))
    if a.nuts_layout:
        s.set_layout(*[int(v) for v in a.nuts_layout.split("x")])
    if a.nuts_lds_levels >= 0:
        s.set_lds_levels(a.nuts_lds_levels)
    if a.nuts_dense_forms:
        mi, ch = (int(v) for v in a.nuts_dense_forms.split(","))
        s.set_dense_forms(mi, ch)
    # warm-up (step-size adaptation) then sampling, as NUTS::run_progress
    _, tw = timed(lambda: s.run_positions(1, a.nuts_discard))
    lf0 = s.leapfrog_counts().sum()
    ds, ts = timed(lambda: s._run_progress_device(a.nuts_collect, 0) if hasattr(s, "_run_progress_device") else s.run_positions(a.nuts_collect, 0))
    lf = s.leapfrog_counts().sum() - lf0
    rhat, ess = ds.split_rhat_ess()
    eps, _ = s.step_sizes()
    return {"config": "cfg3 NUTS DenseGaussian32 f64", "chains": C, "layout": "%dx%d" % s.layout(),
            "mass_adaptation": a.nuts_mass,
            "warmup_s": tw, "sample_s": ts, "leapfrogs": int(lf), "leapfrog_per_s": lf / ts,
            "mean_tree_leapfrogs": lf / (C * a.nuts_collect), "plan": s.launch_plan() if hasattr(s._lib, "gm_nuts_get_plan") else None, "eps_median": float(np.median(eps)),
            "ess_mean": float(ess.mean()), "ess_min": float(ess.min()), "rhat_max": float(rhat.max()),
            "ess_per_s": float(ess.mean()) / ts}


def cfg4(a):
    C, D, L = a.hmc128_chains, 128, 50
    s = gm.HMC(gm.RosenbrockND(), gm.init_det(C, D, np.float32), 0.01, L).set_seed(42)
    if a.hmc128_layout:
        s.set_layout(*[int(v) for v in a.hmc128_layout.split("x")])
    if a.hmc128_unroll:
        s.set_unroll(a.hmc128_unroll)
    s.run_positions(0, 100)
    ds, t = timed(lambda: s.run_positions(100, 0))
    rhat, ess = ds.split_rhat_ess()
    return {"config": "cfg4 HMC Rosenbrock128 f32 (per GPU share)", "chains": C, "layout": "%dx%d" % s.layout(),
            "sample_s": t, "chain_leapfrog_per_s": C * L * 100 / t, "ess_mean": float(ess.mean()),
            "ess_per_s": float(ess.mean()) / t}


def cfg5(a):
    C, D = a.mh_chains, 256
    s = gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(2.38 / 16.0),
                              gm.init_det(C, D), dtype=np.float64).seed(42)
    if a.mh_layout:
        s.set_layout(*[int(v) for v in a.mh_layout.split("x")])
    _, tw = timed(lambda: s.run_positions(0, 100))  # warm (module load, clocks)
    # the config's run(100, 1000), timed whole (1100 transitions, ~20 ms)
    ds, t = timed(lambda: s.run_positions(100, 1000))
    rhat, ess = ds.split_rhat_ess()
    return {"config": "cfg5 MH IsoGauss256 f64 (per GPU share)", "chains": C, "layout": "%dx%d" % s.layout(),
            "burnin_s": tw, "sample_s": t, "chain_steps_per_s": C * 1100 / t,
            "hbm_alg_GBs": C * 1100 * (2 * D + 2) * 8 / t / 1e9, "accept": float(s.accept_counts().mean() / 1200),
            "ess_mean": float(ess.mean()), "ess_per_s": float(ess.mean()) / t}


def ref10k(a):
    """test_bench_10000d (hmc.rs:757-791): 6 chains x 10,000-D RosenbrockND
    f32, eps 0.01, L 50, run(100, 100) -- the reference's own HMC benchmark."""
    dim, n = 10000, 6
    x0 = np.repeat(gm.init_with_seed(1, dim, 42, np.float32), n, axis=0)
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
    s.run_positions(1, 0)  # warm (module load)
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
    out, t = timed(lambda: s.run(100, 100))
    assert out.shape == (n, 100, dim)
    return {"config": "ref test_bench_10000d HMC Rosenbrock10000 f32 6 chains run(100,100)",
            "chains": n, "layout": "%dx%d" % s.layout(), "wall_s": t,
            "chain_leapfrog_per_s": n * 200 * 50 / t, "includes": "D2H of the [6,100,10000] sample"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--which", default="3,4,5,10k")
    p.add_argument("--nuts-mass", default="none", choices=["none", "diagonal", "dense"],
                   help="cfg3 with the warm-up metric adaptation (new_with_mass_matrix)")
    p.add_argument("--nuts-chains", type=int, default=8192)
    p.add_argument("--nuts-lds-levels", type=int, default=-1, help="cap on the subtree-stack levels held in LDS")
    p.add_argument("--nuts-dense-forms", default="", help="minv_lds,chol_lds (gm_nuts_set_dense_forms)")
    p.add_argument("--nuts-discard", type=int, default=500)
    p.add_argument("--nuts-collect", type=int, default=500)
    p.add_argument("--nuts-layout", default="")
    p.add_argument("--hmc128-chains", type=int, default=8192)
    p.add_argument("--hmc128-layout", default="")
    p.add_argument("--hmc128-unroll", type=int, default=0)
    p.add_argument("--mh-chains", type=int, default=16384)
    p.add_argument("--mh-layout", default="")
    a = p.parse_args()
    for w in a.which.split(","):
        r = {"3": cfg3, "4": cfg4, "5": cfg5, "10k": ref10k}[w](a)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
