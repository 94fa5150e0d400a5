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
  tests/test_oracle_nuts_forms.py."""
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
