"""run_progress statistics on the device (stats.rs:24-339): the
MultiChainTracker kernels and the ChainTracker fused into the MH and NUTS
kernels, bit-exact against the oracle's restatement; the progress callback;
samples unchanged by tracking."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))


@pytest.mark.parametrize("case", range(3))
def test_mct_device_kat(gm, case):
    """stats.rs:734-783 (test_rhat_*): R-hat after two steps of 3x4 data."""
    k = KAT["mct_rhat"]
    steps = np.array(k["cases"][case]["steps"], dtype=np.float64)
    t = gm.MultiChainTracker(*steps.shape[1:])
    for x in steps:
        t.step(x)
    r = t.rhat()
    assert np.max(np.abs(r - np.array(k["cases"][case]["expected"], dtype=np.float32))) < k["tol"]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_mct_device_matches_oracle(gm, oracle, dtype):
    rng = np.random.default_rng(7)
    steps = rng.standard_normal((9, 300, 5)).astype(dtype)
    steps[4, 17] = steps[3, 17]
    t = gm.MultiChainTracker(300, 5)
    for x in steps:
        t.step(x)
    np.testing.assert_array_equal(t.rhat(), oracle.mct_rhat(steps.astype(np.float32)))
    assert t.p_accept == oracle.mct_p_accept(steps)
    r = oracle.mct_rhat(steps.astype(np.float32))
    assert t.max_rhat() == np.float32(np.max(r))


def _states(x0_sampler_factory, total):
    s = x0_sampler_factory()
    return s.run(total, 0).transpose(1, 0, 2)


def test_mh_chain_trackers_fused(gm, oracle):
    """core.rs:132-176: each chain's tracker steps after every transition,
    burn-in included; chain_stats and the progress R-hat equal the oracle's
    trackers replayed over the same states."""
    C, D, nc, nd = 40, 3, 12, 5
    x0 = gm.init_with_seed(C, D, 2, np.float64)
    mk = lambda: gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(0.7), x0).seed(3)
    reports = []
    s = mk()
    out, stats = s.run_progress(nc, nd, progress=reports.append, interval=0.0)
    states = _states(mk, nc + nd)
    np.testing.assert_array_equal(out, states[nd:].transpose(1, 0, 2))  # samples unchanged
    st = s.chain_stats()
    p, m, q = oracle.chain_trackers(x0, states)
    assert st.n == nc + nd
    np.testing.assert_array_equal(st.p_accept, p)
    np.testing.assert_array_equal(st.mean, m)
    n = np.float32(nc + nd)
    np.testing.assert_array_equal(st.sm2, ((q - m * m) * n / (n - np.float32(1))).astype(np.float32))
    assert reports and reports[-1].done == reports[-1].total == nc + nd
    r = oracle.collect_rhat(nc + nd, m, q)
    assert reports[-1].max_rhat == np.float32(np.nanmax(r))
    ps = np.float32(0)
    for v in p:
        ps = np.float32(ps + v)
    assert reports[-1].p_accept == np.float32(ps / np.float32(C))
    assert [r_.done for r_ in reports] == sorted(r_.done for r_ in reports)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_nuts_chain_trackers_fused(gm, oracle, dtype):
    """generic_nuts.rs:675-716: NUTS run_progress (n_collect + n_discard
    transitions) with per-step trackers."""
    C, D, nc = 16, 4, 9
    x0 = gm.init_with_seed(C, D, 5, dtype)
    s = gm.NUTS(gm.IsotropicGaussian(1.0), x0, 0.8, dtype=dtype).set_seed(8)
    out, _ = s.run_progress(nc, 0, progress=lambda p: None, interval=0.0)
    st = s.chain_stats()
    p, m, q = oracle.chain_trackers(x0, out.transpose(1, 0, 2))
    np.testing.assert_array_equal(st.p_accept, p)
    np.testing.assert_array_equal(st.mean, m)


def test_hmc_progress_multichain_tracker(gm, oracle):
    """hmc.rs:252-290: burn-in, then a MultiChainTracker stepped with the
    positions at each sync point; interval 0 and n_collect <= 32 make every
    collected state a sync point, so the tracker saw exactly the sample."""
    C, D, nc, nd = 64, 6, 10, 4
    x0 = gm.init_with_seed(C, D, 1, np.float32)
    reports = []
    s = gm.HMC(gm.RosenbrockND(), x0, 0.02, 5).set_seed(4)
    out, stats = s.run_progress(nc, nd, progress=reports.append, interval=0.0)
    twin = gm.HMC(gm.RosenbrockND(), x0, 0.02, 5).set_seed(4)
    np.testing.assert_array_equal(out, twin.run(nc, nd))
    assert [r.done for r in reports] == list(range(1, nc + 1))
    steps = out.transpose(1, 0, 2)
    assert reports[-1].p_accept == oracle.mct_p_accept(steps)
    assert reports[-1].max_rhat == np.float32(np.max(oracle.mct_rhat(steps)))
    assert stats is not None and np.isfinite(stats.ess.mean)


def test_progress_printer_and_silent_default(gm, capsys):
    s = gm.HMC(gm.RosenbrockND(), gm.init_det(8, 3, np.float32), 0.02, 3)
    s.run_progress(4, 0)  # silent
    assert capsys.readouterr().err == ""
    s.run_progress(4, 0, progress=True, interval=0.0)
    err = capsys.readouterr().err
    assert "HMC" in err and "4/4" in err and "p(accept)" in err and "max(rhat)" in err
