"""BASELINE.json config sizes (spot-checked against the oracle through the
global-chain keying: any subset of chains can be replayed on the CPU) and
edge cases the reference exercises (empty runs, 1 chain, 1 dim, odd draw
counts, NaN targets, bad shapes)."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu


def _spot(oracle, t, x0, dim, lay, fn_gpu, fn_oracle, chains):
    out = fn_gpu()
    for c in chains:
        ref = fn_oracle(x0[c:c + 1], c)
        np.testing.assert_array_equal(out[c], ref[:, 0, :], err_msg=f"chain {c}")
    return out


def test_cfg2_hmc_rosenbrock64_full_size(gm, oracle):
    """configs[1]: 4096 chains x 64-D f32, eps 0.01, L 50 -- every chain's
    trajectory keyed by its id; 12 chains replayed bit-exactly on the CPU."""
    C, D, L = 4096, 64, 50
    x0 = gm.init_with_seed(C, D, 42, np.float32)
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, L).set_seed(42)
    lay = s.layout()
    out = s.run(4, 2)
    assert np.all(np.isfinite(out))
    t = Target(1, D)
    for c in [0, 1, 63, 64, 1000, 2047, 2048, 3001, 4032, 4093, 4094, 4095]:
        _, smp, _ = oracle.hmc_run(t, x0[c:c + 1], 0.01, L, 42, 0, 6, 2, *lay, chain_offset=c)
        np.testing.assert_array_equal(out[c], smp[:, 0, :], err_msg=f"chain {c}")


def test_cfg4_hmc_rosenbrock128_per_gpu_share(gm, oracle):
    """configs[3] per-GPU share: 8192 chains x 128-D f32, shard 3 of 8
    (chain_offset 24576) -- identical to the same chains of an unsharded run."""
    C, D, L = 8192, 128, 50
    x0 = gm.init_with_seed(C * 8, D, 42, np.float32)[3 * C:4 * C]
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, L, chain_offset=3 * C).set_seed(42)
    lay = s.layout()
    out = s.run(3, 1)
    t = Target(1, D)
    for c in [0, 5, 4097, 8191]:
        _, smp, _ = oracle.hmc_run(t, x0[c:c + 1], 0.01, L, 42, 0, 4, 1, *lay, chain_offset=3 * C + c)
        np.testing.assert_array_equal(out[c], smp[:, 0, :], err_msg=f"chain {c}")


def test_cfg5_mh_isogauss256_per_gpu_share(gm, oracle):
    """configs[4] per-GPU share: 16384 chains x 256-D f64 MH."""
    C, D = 16384, 256
    x0 = gm.init_with_seed(C, D, 9, np.float64)
    prop = gm.IsotropicGaussian(2.38 / 16)
    s = gm.MetropolisHastings(gm.IsotropicGaussian(1.0), prop, x0).seed(5)
    lay = s.layout()
    out = s.run(5, 5)
    acc = s.accept_counts() / 10.0
    assert 0.05 < acc.mean() < 0.6
    t = Target(2, D, std=1.0)
    for c in [0, 777, 16383]:
        _, smp, _ = oracle.mh_run(t, x0[c:c + 1], prop.std, 5, 0, 10, 5, *lay, chain_offset=c)
        np.testing.assert_array_equal(out[c], smp[:, 0, :], err_msg=f"chain {c}")


def test_cfg3_nuts_dense32_f64_full_size(gm, oracle):
    """configs[2]: 8192 chains x 32-D f64 dense Gaussian NUTS."""
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((32, 32)))
    cov = q @ np.diag(np.logspace(-1, 1, 32)) @ q.T
    cov = 0.5 * (cov + cov.T)
    t = gm.DenseGaussian(np.zeros(32), cov)
    C = 8192
    x0 = gm.init_det(C, 32)
    s = gm.NUTS(t, x0, 0.8, dtype=np.float64).set_seed(42)
    lay = s.layout()
    out = s.run(3, 3)
    ot = Target.from_product(t, 32)
    for c in [0, 4095, 8191]:
        st = oracle.nuts_state(1, np.float64)
        _, smp, _, _ = oracle.nuts_run(ot, x0[c:c + 1], st, 0.8, 10, 42, 0, 3, 3, False, *lay,
                                       chain_offset=c)
        np.testing.assert_array_equal(out[c], smp[:, 0, :], err_msg=f"chain {c}")


def test_empty_and_zero_runs(gm):
    x0 = gm.init_det(5, 3, np.float32)
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 5)
    assert s.run(0, 0).shape == (5, 0, 3)        # hmc.rs:168-171
    assert s.run(0, 3).shape == (5, 0, 3)
    n = gm.NUTS(gm.IsotropicGaussian(1.0), x0, 0.8)
    assert n.run(0, 4).shape == (5, 0, 3)        # nuts.rs:220-229
    np.testing.assert_array_equal(n.run(1, 0)[:, 0], n.positions())


def test_one_chain_one_dim(gm, oracle):
    x0 = np.array([[0.3]], dtype=np.float64)
    t = gm.IsotropicGaussian(2.0)
    s = gm.HMC(t, x0, 0.2, 3).set_seed(1)
    out = s.run(7, 2)
    _, smp, _ = oracle.hmc_run(Target(2, 1, std=2.0), x0, 0.2, 3, 1, 0, 9, 2, 1, 1)
    np.testing.assert_array_equal(out[0], smp[:, 0, :])


def test_zero_leapfrog_always_accepts(gm):
    """L = 0: the proposal is the current state; log_alpha = 0 >= ln u."""
    s = gm.HMC(gm.RosenbrockND(), gm.init_det(16, 4, np.float32), 0.01, 0).set_seed(3)
    x = s.run(5, 0)
    assert np.all(s.accept_counts() == 5)
    np.testing.assert_array_equal(x[:, 0], x[:, -1])


def test_nan_target_rejects(gm):
    """A NaN log-density never satisfies the accept predicate
    (euclidean.rs:527-533 greater_equal; metropolis_hastings.rs:314)."""
    x0 = np.full((8, 2), np.nan, dtype=np.float64)
    s = gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(1.0), x0).seed(1)
    s.run(3, 0)
    assert np.all(s.accept_counts() == 0)
    h = gm.HMC(gm.IsotropicGaussian(1.0), x0, 0.1, 2).set_seed(1)
    h.run(3, 0)
    assert np.all(h.accept_counts() == 0)


def test_odd_draw_count_and_two_draws(gm, oracle):
    """splitcat drops the middle draw of an odd chain (stats.rs:419-425)."""
    rng = np.random.default_rng(3)
    for n in (2, 3, 5, 101, 257):
        x = rng.standard_normal((3, n, 2)).astype(np.float32)
        r, e = gm.split_rhat_mean_ess(x)
        orr, oe = oracle.split_rhat_ess(x)
        np.testing.assert_allclose(r, orr, atol=1e-3, err_msg=str(n))
        np.testing.assert_allclose(e, oe, rtol=1e-3, atol=1e-3, err_msg=str(n))


def test_single_chain_diagnostics(gm, oracle):
    x = np.cumsum(np.random.default_rng(1).standard_normal((1, 400, 3)), axis=1)
    r, e = gm.split_rhat_mean_ess(x)
    orr, oe = oracle.split_rhat_ess(x)
    np.testing.assert_allclose(r, orr, atol=1e-3)
    np.testing.assert_allclose(e, oe, rtol=1e-3)


def test_bad_arguments_raise(gm):
    x0 = gm.init_det(4, 3)
    with pytest.raises(ValueError):
        gm.HMC(gm.DiffableGaussian2D([0, 0], np.eye(2)), x0, 0.1, 2)  # dim assert (distributions.rs:267)
    s = gm.HMC(gm.RosenbrockND(), x0, 0.1, 2)
    with pytest.raises(gm.GMError):
        s.set_layout(2, 1)  # does not cover dim
    with pytest.raises(gm.GMError):
        s.set_layout(3, 1)  # not compiled
    with pytest.raises(gm.GMError):  # beyond the wide path (f32 16384, f64 8192)
        gm.HMC(gm.RosenbrockND(), gm.init_det(2, 16385, np.float32), 0.1, 2)
    with pytest.raises(gm.GMError):
        gm.split_rhat_mean_ess(np.zeros((2, 1, 3)))


def test_reserve_and_host_output_match_device_samples(gm):
    """gm_sampler_reserve pre-sizes the sample buffer (no allocation inside the
    bench's timed region) without changing results; gm_run's host [C,N,D]
    array is the transpose of the device [N,C,D] samples of the same run."""
    C, D, L = 128, 64, 10
    x0 = gm.init_with_seed(C, D, 5, np.float32)
    a = gm.HMC(gm.RosenbrockND(), x0, 0.01, L).set_seed(9)
    b = gm.HMC(gm.RosenbrockND(), x0, 0.01, L).set_seed(9)
    b.reserve(40)
    b.reserve(3)  # grow-only: a smaller request keeps the buffer
    da = a.run_positions(6, 2).to_host()
    db = b.run_positions(6, 2).to_host()
    np.testing.assert_array_equal(da, db)
    ha = a.run(5, 0)
    ds = b.run_positions(5, 0)
    np.testing.assert_array_equal(ha, ds.to_host())
    rows = ds.block(0, 5, 0, C)  # the device layout, [N, C, D]
    np.testing.assert_array_equal(ha, np.ascontiguousarray(rows.transpose(1, 0, 2)))
    with pytest.raises(gm.GMError):
        b.reserve(-1)


def test_host_output_multi_chunk_staging(gm):
    """gm_run's host array goes through two 16 MiB pinned staging slots; a
    sample of 2.5 chunks plus a ragged tail (41 MB) arrives intact: equal to
    the device rows of the same run, transposed to [C, N, D]."""
    C, D, N = 4099, 50, 50  # 4099*50*50*4 B = 41 MB, not a multiple of the chunk
    x0 = gm.init_with_seed(C, D, 11, np.float32)
    a = gm.HMC(gm.RosenbrockND(), x0, 0.01, 2).set_seed(3)
    b = gm.HMC(gm.RosenbrockND(), x0, 0.01, 2).set_seed(3)
    ha = a.run(N, 1)
    assert ha.shape == (C, N, D)
    rows = b.run_positions(N, 1).block(0, N, 0, C)
    np.testing.assert_array_equal(ha, np.ascontiguousarray(rows.transpose(1, 0, 2)))
    hb = a.run(1, 0)  # a small copy after a large one (one partial chunk)
    np.testing.assert_array_equal(hb[:, 0, :], b.run_positions(1, 0).block(0, 1, 0, C)[0])
