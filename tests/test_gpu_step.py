"""step() of every sampler (hmc.rs:316-330, core.rs:81, nuts.rs:431-433 ->
generic_nuts.rs:755-925) against the oracle, bit for bit: on a fresh sampler
and after a run. A NUTS step continues the last run's adaptation counter and
does not re-run init_chain_state; on a fresh sampler it therefore integrates
with the initial epsilon = -1, as the reference's step() does."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu


def _x0(gm, n, d, dtype):
    return (gm.init_with_seed(n, d, 5, np.float64) * 0.5).astype(dtype)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_nuts_step_fresh_and_after_run(gm, oracle, dtype):
    n, d, lay = 12, 32, (16, 2)
    rng = np.random.default_rng(3)
    a = rng.standard_normal((d, d))
    t = gm.DenseGaussian(rng.standard_normal(d), a @ a.T / d + np.eye(d))
    ot = Target.from_product(t, d)
    x0 = _x0(gm, n, d, dtype)
    s = gm.NUTS(t, x0, 0.8, dtype=dtype, max_depth=6).set_seed(4)
    s.set_layout(*lay)
    # fresh sampler: two steps, nothing collected, no init
    s.step()
    s.step()
    st = oracle.nuts_state(n, dtype)
    q, acc, nlf = oracle.nuts_step(ot, x0, st, 0.8, 6, 4, 0, 2, 0, 0, *lay)
    np.testing.assert_array_equal(s.positions(), q)
    np.testing.assert_array_equal(s.accept_counts(), acc)
    np.testing.assert_array_equal(s.leapfrog_counts(), nlf)
    eps, bar = s.step_sizes()
    np.testing.assert_array_equal(eps.astype(dtype), st["eps"])
    np.testing.assert_array_equal(bar.astype(dtype), st["eps_bar"])
    # a run (init_chain_state + warm-up), then steps continuing it
    n_collect, n_discard = 4, 5
    out = s.run(n_collect, n_discard)
    q2, samples, acc2, nlf2 = oracle.nuts_run(ot, q, st, 0.8, 6, 4, 2, n_collect, n_discard, False, *lay)
    np.testing.assert_array_equal(out, samples.transpose(1, 0, 2))
    total = n_collect + n_discard - 1
    for _ in range(3):
        s.step()
    q3, acc3, nlf3 = oracle.nuts_step(ot, q2, st, 0.8, 6, 4, 2 + total + 1, 3, total, n_discard, *lay)
    np.testing.assert_array_equal(s.positions(), q3)
    np.testing.assert_array_equal(s.accept_counts(), acc + acc2 + acc3)
    np.testing.assert_array_equal(s.leapfrog_counts(), nlf + nlf2 + nlf3)
    eps, bar = s.step_sizes()
    np.testing.assert_array_equal(eps.astype(dtype), st["eps"])
    # the run's samples are untouched by the steps
    np.testing.assert_array_equal(s.copy_samples(n_collect), out)
    s.close()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_hmc_and_mh_step(gm, oracle, dtype):
    n, d = 16, 64
    x0 = _x0(gm, n, d, dtype)
    t = gm.RosenbrockND()
    h = gm.HMC(t, x0, 0.01, 9, dtype=dtype).set_seed(8)
    for _ in range(3):
        h.step()
    q, _, acc = oracle.hmc_run(Target.from_product(t, d), x0, 0.01, 9, 8, 0, 3, 3, *h.layout())
    np.testing.assert_array_equal(h.positions(), q)
    np.testing.assert_array_equal(h.accept_counts(), acc)
    h.close()
    prop = gm.IsotropicGaussian(0.2)
    m = gm.MetropolisHastings(t, prop, x0, dtype=dtype).seed(6)
    for _ in range(4):
        m.step()
    q, _, acc = oracle.mh_run(Target.from_product(t, d), x0, 0.2, 6, 0, 4, 4, *m.layout())
    np.testing.assert_array_equal(m.positions(), q)
    np.testing.assert_array_equal(m.accept_counts(), acc)
    m.close()


def test_copy_samples_size_and_stale_device_samples(gm):
    s = gm.HMC(gm.RosenbrockND(), _x0(gm, 8, 4, np.float32), 0.01, 3).set_seed(1)
    ds = s.run_positions(5, 0)
    assert ds.to_host().shape == (8, 5, 4)
    with pytest.raises(gm.GMError):  # a buffer sized for another run is refused
        s.copy_samples(3)
    s.run_positions(9, 0)  # a later run invalidates the earlier handle
    with pytest.raises(RuntimeError):
        ds.to_host()
    with pytest.raises(RuntimeError):
        ds.block(0, 1, 0, 1)
    s.close()


def test_samplers_on_two_devices_one_thread(gm):
    """One thread drives samplers on two devices with gm_set_device calls in
    between: every run must use its own sampler's device (the library asks
    the runtime for the current device instead of caching it)."""
    import ctypes as C
    lib = gm._lib.load()
    n = C.c_int()
    gm._lib.check(lib.gm_device_count(C.byref(n)))
    if n.value < 2:
        pytest.skip("needs two GPUs")
    x0 = gm.init_det(64, 8, np.float32)
    gm._lib.check(lib.gm_set_device(0))
    a = gm.HMC(gm.RosenbrockND(), x0, 0.05, 4).set_seed(1)
    gm._lib.check(lib.gm_set_device(1))
    b = gm.HMC(gm.RosenbrockND(), x0, 0.05, 4).set_seed(1)
    gm._lib.check(lib.gm_set_device(0))
    ra = a.run(5, 1)
    gm._lib.check(lib.gm_set_device(1))
    ra2 = a.run(3, 0)   # a's device is 0 while 1 is current
    gm._lib.check(lib.gm_set_device(0))
    rb = b.run(5, 1)    # b's device is 1 while 0 is current
    np.testing.assert_array_equal(ra, rb)
    assert ra2.shape == (64, 3, 8) and np.all(np.isfinite(ra2))
    a.close()
    b.close()


def test_async_runs_match_synchronous(gm):
    """gm_sampler_set_async: HMC and MH runs return after enqueueing; after a
    synchronize the samples, positions, counters and diagnostics equal a
    synchronous sampler's, and consecutive async runs stay ordered."""
    x0 = gm.init_det(256, 16, np.float32)
    a = gm.HMC(gm.RosenbrockND(), x0, 0.02, 8).set_seed(5)
    b = gm.HMC(gm.RosenbrockND(), x0, 0.02, 8).set_seed(5).set_async(True)
    ra = a.run_positions(7, 3)
    rb = b.run_positions(7, 3)
    rb2 = b.run_positions(4, 0)  # ordered after the first on b's stream
    b.synchronize()
    ra2 = a.run_positions(4, 0)
    np.testing.assert_array_equal(rb2.to_host(), ra2.to_host())
    np.testing.assert_array_equal(b.positions(), a.positions())
    np.testing.assert_array_equal(b.accept_counts(), a.accept_counts())
    ms, n = b.last_run_stats()
    assert ms > 0 and n == 1
    r1, e1 = ra2.split_rhat_ess()
    r2, e2 = rb2.split_rhat_ess()
    np.testing.assert_array_equal(r1, r2)
    with pytest.raises(RuntimeError):
        ra.to_host()  # stale
    del rb
    m = gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(0.5),
                              gm.init_det(64, 8)).seed(3).set_async(True)
    m2 = gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(0.5), gm.init_det(64, 8)).seed(3)
    m.step()
    m.step()
    m2.step()
    m2.step()
    m.synchronize()
    np.testing.assert_array_equal(m.positions(), m2.positions())
