"""The kernels' arithmetic tied to the reference's op structure at the
configs' sizes, on the GPU.

* HMC (cfg2: RosenbrockND 64-D f32, 4096 chains, eps 0.01, L 50). The fused
  kernel's kicks and drift are fused multiply-adds; the reference's
  add_scaled_assign rounds the product and the sum separately
  (batched_hmc.rs:166-190, euclidean.rs:392-394), which the tier-2 composed
  step reproduces (bitwise the oracle's form 1, tests/test_gpu_bv.py).
  Stated tolerances: one transition from identical positions and momenta,
  per-chain proposal deviation rel = max |dq'| / max |q'|:
    from the stationary regime (200 transitions in): rel <= 5e-6 for every
      chain;
    from the bench's iid N(0, 1) start (steep valley walls: 50 leapfrogs
      amplify the ulp-level differences of each kick): median <= 1e-5,
      99th percentile <= 1e-4, <= 1e-3 for every chain either form accepts
      (rejected unstable trajectories are unbounded in both forms);
  at most 0.1 % of the accept decisions differ; over run(100, 100) the
  per-coordinate means and variances agree within 5 Monte-Carlo standard
  errors (chains as the independent units).
* Dense-metric NUTS (cfg3_dense: the 32-D Gaussian, f64, dense adaptation).
  The kernel (carried M^-1 p, fma-chain products; bitwise the oracle's form
  0) against the oracle's form 1 (generic_nuts.rs:244-273, 1357-1418 as
  written) over 512 chains, run(500, 500): per-chain final step size, tree
  length, accept count and per-coordinate mean and variance within 5 standard
  errors. The per-leapfrog bounds of the two forms are in
  tests/test_oracle_nuts_forms.py.
* Identity-metric NUTS (cfg3's target) and MH (cfg5's shape): the kernels'
  canonical-order sums and exp/ln against the oracle's form 1, the reference
  text (left-to-right kinetic, U-turn, proposal and target sums, the C
  library's exp/ln/pow; tests/test_oracle_ref_forms.py). NUTS: 512 chains,
  run(500, 500), the statistics above within 5 standard errors. MH: 4096
  chains, run(100, 1000); along the kernel's trajectory |d log alpha| <=
  1e-13 |lp'| and <= 2e-12 with <= 0.1 % of decisions differing, and means,
  variances and accept rates within 5 standard errors."""
import numpy as np
import pytest

from tests._oracle import Target
from tests.test_oracle_nuts_forms import _mc_close

pytestmark = pytest.mark.gpu


def _one_transition(gm, x0, seed):
    """one transition of both forms from x0 with the same momenta: per-chain
    relative deviation of the proposals q' (max |dq'| / max |q'|), accept
    masks of both, and the engine form's proposals"""
    bv = gm.batch_vector
    eps, L = 0.01, 50
    ref = bv.BatchedGenericHMC(gm.RosenbrockND(), x0, eps, L, seed=seed)                       # reference ops
    eng = bv.BatchedGenericHMC(gm.RosenbrockND(), x0, eps, L, seed=seed, fused_leapfrog=True)  # kernel's bits
    ref.step()
    eng.step()
    qa, qb = eng.proposal_pos.to_host(), ref.proposal_pos.to_host()
    rel = np.max(np.abs(qa - qb), axis=1) / np.max(np.abs(qb), axis=1)
    acc_a = np.all(eng.positions() == qa, axis=1)
    acc_b = np.all(ref.positions() == qb, axis=1)
    return rel, acc_a, acc_b, eng


@pytest.mark.parametrize("start", ["init", "stationary"])
def test_hmc_cfg2_fused_vs_reference_structure_one_transition(gm, start):
    """From the bench's start (iid N(0, 1), far out in the Rosenbrock valley's
    walls, where a few trajectories are unstable and rejected) and from the
    stationary regime (after 200 transitions): per-chain proposal deviation
    and accept flips within the bounds of the module docstring."""
    C_, D, eps, L = 4096, 64, 0.01, 50
    x0 = gm.init_with_seed(C_, D, 42, np.float32)
    if start == "stationary":
        warm = gm.HMC(gm.RosenbrockND(), x0, eps, L).set_seed(3)
        warm.run(1, 200)
        x0 = warm.positions()
    rel, acc_a, acc_b, eng = _one_transition(gm, x0, 7)
    flips = float(np.mean(acc_a != acc_b))
    kept = acc_a | acc_b
    print(f"\ncfg2 one transition from {start}: q' per-chain rel deviation median {np.median(rel):.2e} "
          f"p99 {np.percentile(rel, 99):.2e} max(accepted) {rel[kept].max():.2e} max(all) {rel.max():.2e}; "
          f"accept {acc_a.mean():.4f}, decisions differing {flips:.2e}")
    assert flips <= 1e-3, flips
    if start == "init":
        assert np.median(rel) <= 1e-5 and np.percentile(rel, 99) <= 1e-4 and rel[kept].max() <= 1e-3
    else:
        assert 0 < rel.max() <= 5e-6
    # the fused sampler's transition is the one-kernel leapfrog's, bitwise
    fused = gm.HMC(gm.RosenbrockND(), x0, eps, L).set_seed(7)
    np.testing.assert_array_equal(fused.run(1, 0)[:, 0], eng.positions())
    np.testing.assert_array_equal(fused.accept_counts(), acc_a.astype(np.int64))


def test_hmc_cfg2_fused_vs_reference_structure_run_100_100(gm):
    bv = gm.batch_vector
    C_, D, eps, L = 4096, 64, 0.01, 50
    x0 = gm.init_with_seed(C_, D, 43, np.float32)
    fused = gm.HMC(gm.RosenbrockND(), x0, eps, L).set_seed(8)
    a = fused.run(100, 100)                                   # [C, N, D]
    ref = bv.BatchedGenericHMC(gm.RosenbrockND(), x0, eps, L, seed=8)
    b = ref.run(100, 100)
    assert not np.array_equal(a, b)  # the two arithmetics really differ
    assert _mc_close(a.mean(axis=1), b.mean(axis=1)) < 5.0
    assert _mc_close(a.var(axis=1), b.var(axis=1)) < 5.0
    acc_b = np.mean(np.any(np.diff(b, axis=1) != 0, axis=2), axis=1)
    acc_a = np.mean(np.any(np.diff(a, axis=1) != 0, axis=2), axis=1)
    assert _mc_close(acc_a, acc_b) < 5.0


def test_dense_nuts_kernel_vs_reference_form_512_chains(gm, oracle):
    D, C_ = 32, 512
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((D, D)))
    cov = q @ np.diag(np.logspace(-1, 1, D)) @ q.T
    cov = 0.5 * (cov + cov.T)
    t = gm.DenseGaussian(np.zeros(D), cov)
    x0 = gm.init_with_seed(C_, D, 12, np.float64)
    s = gm.NUTS.new_with_mass_matrix(t, x0, 0.8, gm.NUTSMassMatrixConfig("dense"), dtype=np.float64).set_seed(13)
    out = s.run(500, 500)                                     # [C, N, D]
    lanes, elems = s.layout()
    st = oracle.nuts_state(C_, np.float64)
    om = oracle.nuts_mass(2, C_, D, np.float64, form=1)
    _, smp, acc, nlf = oracle.nuts_mass_run(Target.from_product(t, D), x0, st, om, 0.8, 10, 13, 0, 500, 500,
                                            False, lanes, elems, threads=16)
    ref = smp.transpose(1, 0, 2)
    assert np.all(s.mass_matrix().kind == 2) and np.all(om.kind == 2)
    assert not np.array_equal(out, ref)
    _, bar = s.step_sizes()
    assert _mc_close(bar, st["eps_bar"]) < 5.0
    assert _mc_close(s.leapfrog_counts() / 999.0, nlf / 999.0) < 5.0
    assert _mc_close(s.accept_counts(), acc) < 5.0
    assert _mc_close(out.mean(axis=1), ref.mean(axis=1)) < 5.0
    assert _mc_close(out.var(axis=1), ref.var(axis=1)) < 5.0


def test_nuts_identity_kernel_vs_reference_form_512_chains(gm, oracle):
    """cfg3's 32-D dense Gaussian under the identity metric (the BASELINE NUTS
    config's sampler), f64, 512 chains, run(500, 500): the kernel (canonical
    sums, the engine's exp/ln; bitwise the oracle's form 0) against the
    oracle's form 1 (left-to-right kinetic and U-turn dots, the C library's
    exp/ln/pow: generic_nuts.rs:230-235, 882-893, 1369-1377): final step size,
    tree length, accept count and per-coordinate mean and variance within 5
    standard errors (tests/test_oracle_ref_forms.py pins form 1 to the
    reference text)."""
    D, C_ = 32, 512
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((D, D)))
    cov = q @ np.diag(np.logspace(-1, 1, D)) @ q.T
    cov = 0.5 * (cov + cov.T)
    t = gm.DenseGaussian(np.zeros(D), cov)
    x0 = gm.init_with_seed(C_, D, 14, np.float64)
    s = gm.NUTS(t, x0, 0.8, dtype=np.float64, max_depth=10).set_seed(15)
    out = s.run(500, 500)                                     # [C, N, D]
    lanes, elems = s.layout()
    st = oracle.nuts_state(C_, np.float64)
    _, smp, acc, nlf = oracle.nuts_run(Target.from_product(t, D), x0, st, 0.8, 10, 15, 0, 500, 500, False,
                                       lanes, elems, threads=16, form=1)
    ref = smp.transpose(1, 0, 2)
    assert not np.array_equal(out, ref)
    _, bar = s.step_sizes()
    z = {"eps_bar": _mc_close(bar, st["eps_bar"]),
         "tree": _mc_close(s.leapfrog_counts() / 999.0, nlf / 999.0),
         "accept": _mc_close(s.accept_counts(), acc),
         "mean": _mc_close(out.mean(axis=1), ref.mean(axis=1)),
         "var": _mc_close(out.var(axis=1), ref.var(axis=1))}
    print(f"\ncfg3 identity NUTS kernel vs form 1, max z per statistic: {z}")
    assert max(z.values()) < 5.0, z


def test_mh_cfg5_kernel_vs_reference_form(gm, oracle):
    """cfg5's shape (IsotropicGaussian(1) 256-D f64, proposal sd 2.38/16),
    4096 chains, run(100, 1000) in blocks of 100: along the kernel's own
    trajectory, every step of the first block from identical states -- the
    oracle's form 0 decides exactly the kernel's moves, form 1 (the reference
    text, metropolis_hastings.rs:306-318, distributions.rs:378-406) gives
    |d log alpha| <= 1e-13 |lp'| and <= 2e-12, and <= 0.1 % of the decisions
    differ; over the run, per-coordinate means, variances and accept rates of
    the kernel and of form 1 within 5 standard errors."""
    C_, D, sd, seed = 4096, 256, 2.38 / 16, 21
    t = Target(2, D, std=1.0)
    x0 = gm.init_with_seed(C_, D, 22, np.float64)
    s = gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(sd), x0).seed(seed)
    lanes, elems = s.layout()
    q = x0
    ka = np.zeros((2, C_, D))
    kb = np.zeros((2, C_, D))
    acc_b = np.zeros(C_)
    worst_rel = worst_abs = 0.0
    flips = n = 0
    for blk in range(10):
        out = s.run(100, 100 if blk == 0 else 0)                         # [C, 100, D]
        step0, n_steps, coll = (0, 200, 100) if blk == 0 else (200 + 100 * (blk - 1), 100, 0)
        q, smp, acc = oracle.mh_run(t, q, sd, seed, step0, n_steps, coll, lanes, elems, threads=16, form=1)
        acc_b += acc
        ka += np.stack([out.sum(axis=1), (out * out).sum(axis=1)])
        kb += np.stack([smp.sum(axis=0), (smp * smp).sum(axis=0)])
        if blk == 0:
            for k in range(99):
                x = np.ascontiguousarray(out[:, k])
                la0, lp0, lnu0 = oracle.mh_terms(t, x, sd, seed, 101 + k, lanes, elems, 0, threads=16)
                la1, lp1, lnu1 = oracle.mh_terms(t, x, sd, seed, 101 + k, lanes, elems, 1, threads=16)
                moved = np.any(out[:, k + 1] != out[:, k], axis=1)
                np.testing.assert_array_equal(la0 > lnu0, moved)           # form 0 is the kernel
                d = np.abs(la0 - la1)
                worst_abs = max(worst_abs, float(d.max()))
                worst_rel = max(worst_rel, float((d / np.abs(lp1)).max()))
                flips += int(np.sum((la0 > lnu0) != (la1 > lnu1)))
                n += C_
    print(f"\ncfg5 MH kernel vs form 1: |d log alpha| max {worst_abs:.2e} (rel {worst_rel:.2e}), "
          f"decisions differing {flips} of {n}")
    assert worst_rel <= 1e-13 and worst_abs <= 2e-12
    assert flips <= 1e-3 * n
    ma, mb = ka[0] / 1000.0, kb[0] / 1000.0
    va, vb = ka[1] / 1000.0 - ma * ma, kb[1] / 1000.0 - mb * mb
    z = {"mean": _mc_close(ma, mb), "var": _mc_close(va, vb),
         "accept": _mc_close(s.accept_counts() / 1100.0, acc_b / 1100.0)}
    print(f"cfg5 MH kernel vs form 1, max z per statistic: {z}")
    assert max(z.values()) < 5.0, z
