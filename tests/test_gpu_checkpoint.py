"""Checkpoint / resume (gm_state_save / gm_state_load): a sampler restored from
a blob into a fresh sampler continues bit for bit -- the same draws, accept
and leapfrog counts, NUTS step sizes and learned metric -- as the original
continuing in place. The reference keeps this state only inside its objects
(batched_hmc.rs:40; generic_nuts.rs:573-582, 744) and has no checkpointing
(core.rs:177)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _resume_equal(make, first, second):
    a = make()
    first(a)
    blob = a.save_state()
    out_a = second(a)
    b = make()
    b.load_state(blob)
    out_b = second(b)
    np.testing.assert_array_equal(out_a, out_b)
    np.testing.assert_array_equal(a.positions(), b.positions())
    np.testing.assert_array_equal(a.accept_counts(), b.accept_counts())
    np.testing.assert_array_equal(a.leapfrog_counts(), b.leapfrog_counts())
    return a, b


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("dim", [7, 64, 2000])
def test_hmc_resume(gm, dtype, dim):
    x0 = gm.init_with_seed(16, dim, 1, dtype) * dtype(0.5)

    def make():  # the restored sampler starts elsewhere and unseeded
        return gm.HMC(gm.RosenbrockND(), np.zeros_like(x0) if make.n else x0, 0.005, 7, dtype=dtype)
    make.n = 0

    def first(s):
        s.set_seed(5)
        s.run(3, 4)
        make.n = 1
    _resume_equal(make, first, lambda s: s.run(5, 2))


def test_mh_resume(gm):
    x0 = gm.init_with_seed(32, 9, 2)

    def make():
        return gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(0.4), x0)

    def first(s):
        s.seed(8)
        s.run(4, 5)
    _resume_equal(make, first, lambda s: s.run(6, 1))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_nuts_resume(gm, dtype):
    t = gm.DenseGaussian(np.zeros(5), np.diag([0.1, 1.0, 3.0, 0.5, 2.0]))
    x0 = gm.init_with_seed(24, 5, 4, dtype)

    def make():
        return gm.NUTS(t, x0, 0.8, dtype=dtype)

    def first(s):
        s.set_seed(3)
        s.run(4, 12)
    a, b = _resume_equal(make, first, lambda s: s.run(5, 6))
    for u, v in zip(a.step_sizes(), b.step_sizes()):
        np.testing.assert_array_equal(u, v)


@pytest.mark.parametrize("mode", ["diagonal", "dense"])
def test_nuts_mass_resume(gm, mode):
    t = gm.DenseGaussian(np.zeros(4), [[2.0, 0.3, 0, 0], [0.3, 1.0, 0, 0], [0, 0, 0.2, 0], [0, 0, 0, 4.0]])
    x0 = gm.init_with_seed(16, 4, 6)
    cfg = gm.NUTSMassMatrixConfig(mode, start_buffer=5, end_buffer=5, initial_window=10)
    made = []

    def make():  # the original adapts; the restored one gets its metric from the blob
        s = gm.NUTS.new_with_mass_matrix(t, x0, 0.8, cfg) if not made else gm.NUTS(t, x0, 0.8)
        made.append(s)
        return s

    def first(s):
        s.set_seed(2)
        s.run(3, 40)
    a, b = _resume_equal(make, first, lambda s: s.run(4, 40))
    ma, mb = a.mass_matrix(), b.mass_matrix()
    np.testing.assert_array_equal(ma.kind, mb.kind)
    np.testing.assert_array_equal(ma.diag_inv, mb.diag_inv)
    if mode == "dense":
        np.testing.assert_array_equal(ma.dense_inv, mb.dense_inv)


def test_state_mismatch_raises(gm):
    a = gm.HMC(gm.RosenbrockND(), gm.init_det(4, 3, np.float32), 0.01, 3)
    blob = a.save_state()
    with pytest.raises(gm.GMError):
        gm.HMC(gm.RosenbrockND(), gm.init_det(5, 3, np.float32), 0.01, 3).load_state(blob)
    with pytest.raises(gm.GMError):
        gm.HMC(gm.RosenbrockND(), gm.init_det(4, 3), 0.01, 3, dtype=np.float64).load_state(blob)
    with pytest.raises(gm.GMError):
        gm.NUTS(gm.RosenbrockND(), gm.init_det(4, 3, np.float32), 0.8).load_state(blob)
    with pytest.raises(gm.GMError):
        a.load_state(b"not a state blob" * 8)
    with pytest.raises(gm.GMError):
        a.load_state(blob[:40])


def test_state_config_mismatch_raises(gm):
    x0 = gm.init_det(4, 3, np.float32)
    blob = gm.HMC(gm.RosenbrockND(), x0, 0.01, 3).save_state()
    with pytest.raises(gm.GMError):  # another step size
        gm.HMC(gm.RosenbrockND(), x0, 0.02, 3).load_state(blob)
    with pytest.raises(gm.GMError):  # another n_leapfrog
        gm.HMC(gm.RosenbrockND(), x0, 0.01, 4).load_state(blob)
    nb = gm.NUTS(gm.RosenbrockND(), x0, 0.8, max_depth=6).save_state()
    with pytest.raises(gm.GMError):  # another max_depth
        gm.NUTS(gm.RosenbrockND(), x0, 0.8, max_depth=7).load_state(nb)
    with pytest.raises(gm.GMError):  # another target_accept_p
        gm.NUTS(gm.RosenbrockND(), x0, 0.7, max_depth=6).load_state(nb)


def test_truncated_mass_blob_leaves_sampler_unchanged(gm):
    """A truncated or corrupt NUTS blob is rejected before anything is changed
    (the learned metric and the positions stay)."""
    t = gm.DenseGaussian(np.zeros(4), np.diag([2.0, 1.0, 0.2, 4.0]))
    x0 = gm.init_with_seed(8, 4, 6)
    cfg = gm.NUTSMassMatrixConfig("dense", start_buffer=5, end_buffer=5, initial_window=10)
    a = gm.NUTS.new_with_mass_matrix(t, x0, 0.8, cfg).set_seed(2)
    a.run(3, 40)
    blob = a.save_state()
    before = (a.positions(), a.mass_matrix(), a.step_sizes())
    for bad in (blob[:len(blob) // 2], blob[:-8]):
        with pytest.raises(gm.GMError):
            a.load_state(bad)
        after = (a.positions(), a.mass_matrix(), a.step_sizes())
        np.testing.assert_array_equal(before[0], after[0])
        np.testing.assert_array_equal(before[1].kind, after[1].kind)
        np.testing.assert_array_equal(before[1].dense_inv, after[1].dense_inv)
        np.testing.assert_array_equal(before[2][0], after[2][0])
    a.load_state(blob)  # the intact blob still loads
