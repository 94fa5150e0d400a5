"""NUTS with mass-matrix warm-up (GenericNUTS::new_with_mass_matrix,
generic_nuts.rs:33-359, 379-398, 897-921, 948-997) on the GPU, bit-exact
against the oracle's restatement driven by the same Philox streams:
samples, the learned metric, the step sizes; across two runs (metric and
window schedule persist), and with run_progress semantics."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu

SMALL = dict(start_buffer=5, end_buffer=5, initial_window=10)


def _gauss(gm, cov, mean=None):
    cov = np.asarray(cov, dtype=np.float64)
    mean = np.zeros(len(cov)) if mean is None else np.asarray(mean, dtype=np.float64)
    return gm.DenseGaussian(mean, cov)


def _check_run(gm, oracle, t, x0, dtype, mode, runs, progress=False, layout=None, forms=None, mpass=True, **cfg):
    C_, D = x0.shape
    adapt = {1: "diagonal", 2: "dense"}[mode]
    mc = gm.NUTSMassMatrixConfig(adapt, **{**dict(regularize=0.05, jitter=1e-6, dense_max_dim=75), **cfg})
    s = gm.NUTS.new_with_mass_matrix(t, x0, 0.8, mc, dtype=dtype).set_seed(11)
    if layout:
        s.set_layout(*layout)
    if forms:
        s.set_dense_forms(**forms)
    if not mpass:
        s.set_momentum_pass(False)
    lanes, elems = s.layout()
    ot = Target.from_product(t, D)
    st = oracle.nuts_state(C_, dtype)
    om = oracle.nuts_mass(mode, C_, D, dtype, **{k: v for k, v in cfg.items() if k != "dense_max_dim"})
    q = np.array(x0, dtype=dtype)
    init_step = 0
    for nc, nd in runs:
        if progress:
            out, _ = s.run_progress(nc, nd)
        else:
            out = s.run(nc, nd)
        q, smp, _, _ = oracle.nuts_mass_run(ot, q, st, om, 0.8, 10, 11, init_step, nc, nd, progress,
                                            lanes, elems)
        np.testing.assert_array_equal(out, smp.transpose(1, 0, 2))
        total = nc + nd if progress else nc + nd - 1
        init_step += total + 1
        m = s.mass_matrix()
        np.testing.assert_array_equal(m.kind, om.kind)
        np.testing.assert_array_equal(m.diag_inv[om.kind == 1], om.dinv[om.kind == 1])
        np.testing.assert_array_equal(m.diag_sqrt[om.kind == 1], om.dsqrt[om.kind == 1])
        if mode == 2:
            np.testing.assert_array_equal(m.dense_inv[om.kind == 2], om.minv[om.kind == 2])
            np.testing.assert_array_equal(m.dense_chol[om.kind == 2], om.mchol[om.kind == 2])
        eps, bar = s.step_sizes()
        np.testing.assert_array_equal(eps.astype(dtype), st["eps"])
        np.testing.assert_array_equal(bar.astype(dtype), st["eps_bar"])
    return s, om


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_diag_warmup_bitexact(gm, oracle, dtype):
    t = _gauss(gm, np.diag([0.04, 1.0, 4.0, 0.5]))
    x0 = gm.init_with_seed(24, 4, 3, dtype)
    s, om = _check_run(gm, oracle, t, x0, dtype, 1, [(20, 60), (15, 40)], **SMALL)
    assert np.all(om.kind == 1)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_dense_warmup_bitexact(gm, oracle, dtype):
    cov = np.array([[2.0, 0.9, 0.0], [0.9, 1.0, 0.3], [0.0, 0.3, 0.5]])
    t = _gauss(gm, cov, [0.5, -1.0, 0.0])
    x0 = gm.init_with_seed(16, 3, 4, dtype)
    s, om = _check_run(gm, oracle, t, x0, dtype, 2, [(12, 70), (10, 45)], **SMALL)
    assert np.all(om.kind >= 1)


def test_dense_warmup_wide_layout(gm, oracle):
    """D = 40 (two coordinates per lane at the default layout? no: 64 lanes x 1)
    and D = 70 (64 lanes x 2): the lane broadcasts of the dense products."""
    rng = np.random.default_rng(9)
    for D in (40, 70):
        a = rng.standard_normal((D, D))
        cov = a @ a.T / D + 0.5 * np.eye(D)
        t = _gauss(gm, cov)
        x0 = gm.init_with_seed(6, D, 5, np.float64)
        _check_run(gm, oracle, t, x0, np.float64, 2, [(6, 40)], start_buffer=4, end_buffer=4,
                   initial_window=10)


@pytest.mark.parametrize("minv_lds,chol_lds", [("2", "1"), ("1", "1"), ("1", "0"), ("0", "0"), ("-1", "-1")])
@pytest.mark.parametrize("D,chains", [(20, 10), (32, 36)])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_dense_warmup_matrix_core_layout(gm, oracle, minv_lds, chol_lds, D, chains, dtype):
    """f64 and f32 at 16 lanes x 2 (the dense Gaussian's layout; its product
    on the matrix cores for f64) with each form of the dense metric's
    products: M^-1 full in LDS (2), its packed lower triangle with or without
    the packed Cholesky factor (1), and the transposed per-chain matrices in
    global memory (0), and the automatic choice (-1: the packed M^-1 with L
    in global memory, which leaves several subtree-stack levels in LDS)
    (gm_nuts_set_dense_forms, nuts_launch.h); D = 20 pads rows and columns
    to 32, and 10 or 36 chains leave the last wave partly empty (the VALU
    target product there). The launch plan read back shows the form actually
    used."""
    rng = np.random.default_rng(21)
    a = rng.standard_normal((D, D))
    cov = a @ a.T / D + 0.5 * np.eye(D)
    t = _gauss(gm, cov, rng.standard_normal(D))
    x0 = gm.init_with_seed(chains, D, 6, np.float64).astype(dtype)
    forms = dict(minv_lds=int(minv_lds), chol_lds=int(chol_lds))
    s, om = _check_run(gm, oracle, t, x0, dtype, 2, [(8, 45), (6, 20)], start_buffer=4, end_buffer=4,
                       initial_window=10, layout=(16, 2), forms=forms)
    assert s.layout() == (16, 2)
    assert np.any(om.kind == 2)
    plan = s.launch_plan()
    if minv_lds == "-1":
        assert plan["minv_lds"] == 1 and plan["chol_lds"] == 0 and plan["lds_levels"] >= 4, plan
        return
    assert plan["minv_lds"] == int(minv_lds) or (minv_lds == "2" and plan["minv_lds"] == 1)
    assert plan["chol_lds"] <= int(chol_lds) and (plan["chol_lds"] == 0 or plan["minv_lds"] == 1)


@pytest.mark.parametrize("D,chains,dtype,mpass", [(32, 36, np.float64, True), (20, 10, np.float64, True),
                                                  (32, 36, np.float32, True), (32, 36, np.float64, False)])
def test_dense_frozen_sampling_bitexact(gm, oracle, D, chains, dtype, mpass):
    """After the warm-up, a run without windows (run(n, 0), the bench's
    sampling phase) with every chain's metric dense takes the frozen-dense
    kernel (MASS 3: no identity/diagonal branches, no Welford state, two
    waves per SIMD at 16 x 2, its momenta p0 = L z and M^-1 p0 from the
    launch's pre-pass, nuts_dense_momenta_kernel) -- the same bits as the
    oracle, partial wave included; a later warm-up run goes back to the
    adaptive kernel. With the momentum pass off the sampling runs take the
    adaptive kernel, which applies the metric itself: the same bits."""
    rng = np.random.default_rng(31)
    a = rng.standard_normal((D, D))
    cov = a @ a.T / D + 0.5 * np.eye(D)
    t = _gauss(gm, cov, rng.standard_normal(D))
    x0 = gm.init_with_seed(chains, D, 7, np.float64).astype(dtype)
    s, om = _check_run(gm, oracle, t, x0, dtype, 2, [(1, 60), (25, 0), (6, 20), (9, 0)], start_buffer=4,
                       end_buffer=4, initial_window=10, layout=(16, 2), mpass=mpass)
    assert np.all(om.kind == 2)
    assert s.launch_plan()["frozen"] == (1 if mpass else 0)
    s.run(2, 20)
    assert s.launch_plan()["frozen"] == 0


def test_progress_semantics_with_mass(gm, oracle):
    t = _gauss(gm, np.diag([0.25, 2.0, 1.0]))
    x0 = gm.init_with_seed(10, 3, 6, np.float64)
    _check_run(gm, oracle, t, x0, np.float64, 1, [(10, 50)], progress=True, **SMALL)


def test_dense_falls_back_to_diagonal_above_max_dim(gm):
    t = gm.IsotropicGaussian(1.0)
    s = gm.NUTS.new_with_mass_matrix(t, gm.init_det(4, 6), 0.8,
                                     gm.NUTSMassMatrixConfig("dense", dense_max_dim=5, **SMALL))
    s.run(5, 40)
    m = s.mass_matrix()
    assert m.dense_inv is None and np.all(m.kind == 1)


def test_default_schedule_recovers_scales(gm, oracle):
    """The reference defaults (75 / 25 / 50, windows ending at m = 100, 150,
    250, 450, 549 for 600 warm-up steps): chains spot-checked bit-exactly
    against the oracle, and the diagonal metric tracks 0.95 * var + 0.05
    (generic_nuts.rs:962-964) within the noise of a ~100-draw last window."""
    std = np.array([0.3, 1.0, 2.0])
    t = _gauss(gm, np.diag(std ** 2))
    x0 = gm.init_with_seed(256, 3, 8)
    s = gm.NUTS.new_with_mass_matrix(t, x0, 0.8, gm.NUTSMassMatrixConfig()).set_seed(0)
    out = s.run(50, 600)
    m = s.mass_matrix()
    assert np.all(m.kind == 1)
    var = 1.0 / m.diag_inv
    np.testing.assert_allclose(np.median(var, axis=0), 0.95 * std ** 2 + 0.05, rtol=0.5)
    lanes, elems = s.layout()
    for c in (0, 131, 255):
        st = oracle.nuts_state(1, np.float64)
        om = oracle.nuts_mass(1, 1, 3, np.float64)
        _, smp, _, _ = oracle.nuts_mass_run(Target.from_product(t, 3), x0[c:c + 1], st, om, 0.8, 10, 0, 0,
                                            50, 600, False, lanes, elems, chain_offset=c)
        np.testing.assert_array_equal(out[c], smp[:, 0, :])
        np.testing.assert_array_equal(m.diag_inv[c], om.dinv[0])


def test_dense_metric_convention_is_reference_M_equals_cov(gm):
    """The reference's metric convention, pinned on cfg3's target. Its dense
    warm-up sets the MASS matrix to the regularised sample covariance,
    M = C = 0.95 Sigma_hat + 0.05 I (generic_nuts.rs:975-989): dense_from_cov
    keeps inv = C^-1 for the kinetic energy and drift and chol = cholesky(C)
    for the momentum, p = chol z ~ N(0, C) (:209-224, 255-303). Stan's
    convention is the inverse (M^-1 = C): the reference's drift M^-1 p then
    rescales the target's directions by Sigma^-1 instead of Sigma, which is
    why cfg3 with dense adaptation mixes worse than with the identity metric
    (bench cfg3_dense). The engine reproduces the reference:
      * mean over chains of inv(dense_inv) is C to 15 % (Frobenius, relative;
        each chain's last window holds ~200 draws, 512 chains);
      * dense_inv is C^-1 (to 50 %: the mean of inverted estimates is biased
        up by ~n/(n-D-1)), not Stan's C (1.2 away, relative);
      * chol chol^T = inv(dense_inv) per chain (to 1e-9 relative)."""
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((32, 32)))
    cov = q @ np.diag(np.logspace(-1, 1, 32)) @ q.T
    cov = 0.5 * (cov + cov.T)
    t = gm.DenseGaussian(np.zeros(32), cov)
    s = gm.NUTS.new_with_mass_matrix(t, gm.init_det(512, 32), 0.8, gm.NUTSMassMatrixConfig("dense"),
                                     dtype=np.float64).set_seed(5)
    s.run(1, 500)
    m = s.mass_matrix()
    assert np.all(m.kind == 2)
    c_reg = 0.95 * cov + 0.05 * np.eye(32)
    c_hat = np.linalg.inv(m.dense_inv)  # each chain's regularised covariance estimate
    rel = np.linalg.norm(c_hat.mean(axis=0) - c_reg) / np.linalg.norm(c_reg)
    assert rel < 0.15, rel
    minv_mean = m.dense_inv.mean(axis=0)
    inv_c = np.linalg.inv(c_reg)
    assert np.linalg.norm(minv_mean - inv_c) / np.linalg.norm(inv_c) < 0.5
    # Stan's convention would put C itself there: 1.2 away (relative) from C^-1 here
    assert np.linalg.norm(minv_mean - c_reg) / np.linalg.norm(c_reg) > 0.9
    for c in (0, 101, 511):
        L = m.dense_chol[c]
        np.testing.assert_allclose(L @ L.T, c_hat[c], rtol=1e-9, atol=1e-9 * np.abs(c_hat[c]).max())
