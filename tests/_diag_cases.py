"""Config-size cases of the split-R-hat/ESS diagnostic (stats.rs:439-573)
shared by tests/test_gpu_diag_fullsize.py and tools/diag_fullsize.py.

Each case samples a BASELINE.json configuration on the GPU (the bench's own
sampler and schedule), computes the diagnostic on the device exactly as the
bench / the 8-GPU all-gather does, and returns it next to

* the oracle (tests/_oracle.py, the C restatement of stats.rs: f32 throughout,
  sequential f32 sum of the autocovariances over split chains, stats.rs:535),
  on the same f32-cast sample; and
* an f64 evaluation of the same formulas (NumPy, the Gram-matrix form of the
  lag sums), the "exact" value that tells which side drifts at large chain
  counts.

Test infrastructure only (imports the oracle)."""
from __future__ import annotations

import os

import numpy as np

# BASELINE.json configs / SURVEY.md §8(d)
CFG2 = dict(C=4096, D=64, L=50, eps=0.01, n_collect=100, n_discard=100)
CFG4 = dict(R=8, C=8192, D=128, L=50, eps=0.01, n_collect=100, n_discard=100)
CFG5 = dict(R=8, C=16384, D=256, prop=2.38 / 16, n_collect=100, n_discard=1000)


def threads() -> int:
    # the GPU box grants 16 cores (cgroup quota); this container 8
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def exact_f64(x32: np.ndarray):
    """split_rhat_mean_ess's formulas in f64 on an f32
    [C, N, P] sample. Sum over lags via the Gram matrix G = Y^T Y of the
    centred split chains: sum_k acov_k[l] = (1/h) sum_t G[t, t+l]."""
    C, N, P = x32.shape
    h = N // 2
    K = 2 * C
    rhat = np.empty(P)
    ess = np.empty(P)
    for p in range(P):
        y = np.concatenate([x32[:, :h, p], x32[:, N - h:, p]]).astype(np.float64)  # [K, h]
        cm = y.mean(axis=1)
        b = ((cm - cm.mean()) ** 2).sum() * h / (K - 1)
        yc = y - cm[:, None]
        w = ((yc * yc).sum(axis=1) / h).mean()
        v = (h - 1) / h * w + b / h
        rhat[p] = np.sqrt(w / v)
        g = yc.T @ yc
        avg = np.array([np.trace(g, offset=l) for l in range(h)]) / h / K
        rho = 1.0 - (w - avg) / v
        mn = rho[0] + rho[1] if h >= 2 else 0.0
        out = 0.0
        for i in range(h // 2):
            pt = rho[2 * i] + rho[2 * i + 1]
            if pt <= 0.0:
                break
            pt = min(pt, mn)
            mn = pt
            out += pt
        ess[p] = K * h / (-1.0 + 2.0 * out)
    return rhat, ess


def compare(gpu, orc, exact) -> dict:
    (gr, ge), (orr, oe), (xr, xe) = gpu, orc, exact
    gr, ge, orr, oe = (np.asarray(a, np.float64) for a in (gr, ge, orr, oe))
    rel = lambda a, b: np.abs(a - b) / np.abs(b)  # noqa: E731
    return {
        "n_params": int(gr.size),
        "rhat_gpu_vs_oracle_max_abs": float(np.max(np.abs(gr - orr))),
        "ess_gpu_vs_oracle_max_rel": float(np.max(rel(ge, oe))),
        "ess_gpu_vs_oracle_n_over_1e-3": int(np.sum(rel(ge, oe) > 1e-3)),
        "rhat_gpu_vs_exact_max_abs": float(np.max(np.abs(gr - xr))),
        "rhat_oracle_vs_exact_max_abs": float(np.max(np.abs(orr - xr))),
        "ess_gpu_vs_exact_max_rel": float(np.max(rel(ge, xe))),
        "ess_oracle_vs_exact_max_rel": float(np.max(rel(oe, xe))),
        "rhat_range": [float(gr.min()), float(gr.max())],
        "ess_range": [float(ge.min()), float(ge.max())],
    }


def cfg2(gm, oracle):
    """configs[1]: HMC 4096 x 64-D Rosenbrock f32, run_positions(100, 100)
    (the bench's ess.cfg2_schedule sample)."""
    c = CFG2
    x0 = gm.init_det(c["C"], c["D"], np.float32)
    s = gm.HMC(gm.RosenbrockND(), x0, c["eps"], c["L"]).set_seed(42)
    ds = s.run_positions(c["n_collect"], c["n_discard"])
    gpu = ds.split_rhat_ess()
    host = ds.to_host()
    orc = oracle.split_rhat_ess(host, threads=threads())
    res = compare(gpu, orc, exact_f64(host))
    s.close()
    return res


def _sharded(gm, make, R, C, D, n_collect, n_discard, dtype, params=None):
    from general_mcmc_amd.distributed import split_rhat_ess_shards
    samplers, shards, host = [], [], []
    for r in range(R):
        s = make(r)
        samplers.append(s)
        shards.append(s.run_positions(n_collect, n_discard))
    gr, ge = split_rhat_ess_shards(shards)  # the all-gather layout [R][P][2C], [R][h][P]
    for d in shards:
        x = d.to_host()
        if params is not None:
            x = np.ascontiguousarray(x[:, :, params])
        host.append(x.astype(np.float32))  # the reference's cast (stats.rs:443)
        del x
    host = np.concatenate(host)
    for s in samplers:
        s.close()
    if params is not None:
        gr, ge = gr[params], ge[params]
    return (gr, ge), host


def cfg4(gm, oracle):
    """configs[3]: HMC 65,536 x 128-D Rosenbrock f32 as 8 shards of 8192
    chains (chain_offset r*8192, global Philox ids), diagnostics through the
    8-rank all-gather assembly on one GPU."""
    c = CFG4
    x0 = gm.init_det(c["R"] * c["C"], c["D"], np.float32)

    def make(r):
        off = r * c["C"]
        return gm.HMC(gm.RosenbrockND(), x0[off:off + c["C"]], c["eps"], c["L"],
                      chain_offset=off).set_seed(42)
    gpu, host = _sharded(gm, make, c["R"], c["C"], c["D"], c["n_collect"], c["n_discard"], np.float32)
    orc = oracle.split_rhat_ess(host, threads=threads())
    return compare(gpu, orc, exact_f64(host))


CFG5_PARAMS = np.arange(0, 256, 4)  # 64 of 256 parameters, all 131,072 chains


def cfg5(gm, oracle):
    """configs[4]: MH 131,072 x 256-D f64 IsotropicGaussian (proposal sigma
    2.38/16) as 8 shards of 16,384; the device computes all 256 parameters,
    the oracle checks every 4th over all chains (parameters are independent,
    stats.rs:463-466, 545-548)."""
    c = CFG5
    x0 = gm.init_det(c["R"] * c["C"], c["D"], np.float64)
    prop = gm.IsotropicGaussian(c["prop"])

    def make(r):
        off = r * c["C"]
        return gm.MetropolisHastings(gm.IsotropicGaussian(1.0), prop, x0[off:off + c["C"]],
                                     chain_offset=off).seed(42)
    gpu, host = _sharded(gm, make, c["R"], c["C"], c["D"], c["n_collect"], c["n_discard"], np.float64,
                         params=CFG5_PARAMS)
    orc = oracle.split_rhat_ess(host, threads=threads())
    return compare(gpu, orc, exact_f64(host))
