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
