"""The RCCL path of the diagnostic exchange on one GPU (a 1-rank
communicator runs the same all-gather code as the 8-GPU bench)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_single_rank_diagnostic_matches_local(gm, monkeypatch):
    from general_mcmc_amd.distributed import Comm, ControlPlane
    monkeypatch.setenv("WORLD_SIZE", "1")
    cp = ControlPlane()
    comm = Comm(cp)
    s = gm.HMC(gm.RosenbrockND(), gm.init_det(512, 16, np.float32), 0.02, 10).set_seed(4)
    ds = s.run_positions(64, 16)
    r1, e1 = comm.split_rhat_ess(ds)
    r0, e0 = ds.split_rhat_ess()
    np.testing.assert_array_equal(r1, r0)
    np.testing.assert_array_equal(e1, e0)
    host = ds.to_host()
    r2, e2 = gm.split_rhat_mean_ess(host)
    np.testing.assert_array_equal(r2, r0)
    np.testing.assert_array_equal(e2, e0)
    comm.close()


def test_run_progress_stats_match_host_diagnostics(gm):
    s = gm.NUTS(gm.IsotropicGaussian(1.0), gm.init_det(64, 4), 0.8).set_seed(3)
    sample, stats = s.run_progress(50, 20)
    r, e = gm.split_rhat_mean_ess(sample)
    assert stats.ess.min == pytest.approx(float(e.min()))
    assert stats.rhat.max == pytest.approx(float(r.max()))


@pytest.mark.parametrize("n_collect", [100, 300])  # h = 50 (matrix-core series), h = 150 (direct lags)
def test_multi_shard_assembly_matches_whole_sample(gm, oracle, n_collect):
    """The N > 1 exchange without RCCL: four samplers own contiguous chain
    shards (chain_offset, global Philox ids) like four bench ranks; their
    summaries assembled in the all-gather's [R][P][2C] layout give the
    diagnostics of the whole sample (stats.rs:439-450): against the
    single-shard device result up to summation order, and within 1e-3 of the
    oracle's restatement (the north star's R-hat bar)."""
    from general_mcmc_amd.distributed import shard, split_rhat_ess_shards
    R, C_glob, D = 4, 512, 8
    x = gm.init_with_seed(C_glob, D, 42, np.float64).astype(np.float32)
    samplers, shards = [], []
    for r in range(R):
        off, n = shard(C_glob, R, r)
        s = gm.HMC(gm.RosenbrockND(), x[off:off + n], 0.05, 8, chain_offset=off).set_seed(7)
        samplers.append(s)
        shards.append(s.run_positions(n_collect, 10))
    whole = gm.HMC(gm.RosenbrockND(), x, 0.05, 8).set_seed(7)
    host = whole.run(n_collect, 10)
    np.testing.assert_array_equal(np.concatenate([d.to_host() for d in shards]), host)
    r4, e4 = split_rhat_ess_shards(shards)
    r1, e1 = gm.split_rhat_mean_ess(host)
    np.testing.assert_allclose(r4, r1, rtol=1e-5)
    np.testing.assert_allclose(e4, e1, rtol=1e-4)
    ro, eo = oracle.split_rhat_ess(host)
    np.testing.assert_allclose(r4, ro, atol=1e-3)
    np.testing.assert_allclose(e4, eo, rtol=1e-3)
    with pytest.raises(ValueError):
        split_rhat_ess_shards([shards[0], whole.run_positions(3, 0)])
    for s in samplers + [whole]:
        s.close()
