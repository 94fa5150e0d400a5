"""NUTS mass-matrix warm-up in the oracle (generic_nuts.rs:33-359, 897-921):
the reference's own MassMatrix unit tests (generic_nuts.rs:1427-1489, SURVEY
KAT 8) and behaviour checks of the warm-up schedule."""
import ctypes as C

import numpy as np

from tests._oracle import Target, _p


def test_diag_kinetic_and_inv_mul_kat(oracle):
    """diagonal_mass_matrix_kinetic_and_inv_mul_are_consistent (:1427-1441)."""
    var = np.array([4.0, 9.0])
    p = np.array([2.0, 3.0])
    ke = C.c_double()
    out = np.zeros(2)
    assert oracle.lib.or_mass_diag_kat(_p(var), 2, 1e-12, _p(p), C.byref(ke), _p(out)) == 0
    assert abs(ke.value - 1.0) < 1e-12
    assert abs(out[0] - 0.5) < 1e-12 and abs(out[1] - 1.0 / 3.0) < 1e-12


def test_dense_inverse_kat(oracle):
    """dense_mass_matrix_inverse_matches_identity_action (:1443-1457)."""
    cov = np.array([2.0, 0.3, 0.3, 1.0])
    p = np.array([0.7, -1.1])
    out = np.zeros(2)
    assert oracle.lib.or_mass_dense_kat(_p(cov), 2, 1e-12, _p(p), _p(out)) == 0
    assert p @ out > 0
    np.testing.assert_allclose(out, np.linalg.solve(cov.reshape(2, 2) + 1e-10 * np.eye(2), p), rtol=1e-9)


def test_warmup_diagonal_update_kat(oracle):
    """warmup_diagonal_update_produces_positive_variances (:1459-1488)."""
    xs = np.array([[-2.0, 1.0], [-1.0, 0.0], [0.0, 1.0], [2.0, -1.0], [1.0, 0.5]])
    inv, sq = np.zeros(2), np.zeros(2)
    assert oracle.lib.or_mass_warmup_diag_kat(_p(xs), 5, 2, 0.05, 1e-6, _p(inv), _p(sq)) == 0
    assert np.all(np.isfinite(inv) & (inv > 0) & np.isfinite(sq) & (sq > 0))
    var = 0.95 * xs.var(axis=0, ddof=1) + 0.05
    np.testing.assert_allclose(inv, 1 / var, rtol=1e-12)
    np.testing.assert_allclose(sq, np.sqrt(var), rtol=1e-12)


def test_identity_mode_matches_plain_nuts(oracle):
    """mode 0 is NUTS::new (identity, no warm-up): bitwise the plain run."""
    x0 = np.random.default_rng(1).standard_normal((6, 3))
    t = Target(2, 3, std=1.5)
    s1, s2 = oracle.nuts_state(6, np.float64), oracle.nuts_state(6, np.float64)
    m = oracle.nuts_mass(0, 6, 3, np.float64)
    a = oracle.nuts_run(t, x0, s1, 0.8, 10, 3, 0, 20, 30, False, 4, 1)
    b = oracle.nuts_mass_run(t, x0, s2, m, 0.8, 10, 3, 0, 20, 30, False, 4, 1)
    np.testing.assert_array_equal(a[1], b[1])


def test_diag_warmup_learns_scales(oracle):
    """Diagonal adaptation on a badly scaled Gaussian: after warm-up the
    metric's variances track the target's, shrunk as the reference does
    (0.95 * sample variance + 0.05, generic_nuts.rs:962-964)."""
    D, C_ = 4, 8
    std = np.array([0.1, 1.0, 3.0, 10.0])
    cov = np.diag(std ** 2)
    t = Target(3, D, mean=np.zeros(D), prec=np.linalg.inv(cov),
               norm_const=-(D * np.log(2 * np.pi) + np.log(np.linalg.det(cov))) / 2)
    x0 = np.random.default_rng(2).standard_normal((C_, D))
    st = oracle.nuts_state(C_, np.float64)
    m = oracle.nuts_mass(1, C_, D, np.float64)
    oracle.nuts_mass_run(t, x0, st, m, 0.8, 10, 5, 0, 10, 1500, False, 4, 1)
    assert np.all(m.kind == 1)
    var = 1.0 / m.dinv
    # the small scale is pinned by the shrinkage: 0.95 * 0.01 + 0.05
    np.testing.assert_allclose(var[:, 0], 0.0595, rtol=0.1)
    med = np.median(var, axis=0)
    assert med[0] < med[1] < med[2], med  # learned ordering of the scales
    assert tuple(m.st.sched) != (100, 25)  # the schedule advanced


def test_dense_warmup_runs(oracle):
    D, C_ = 3, 4
    a = np.array([[2.0, 0.9, 0.0], [0.9, 1.0, 0.3], [0.0, 0.3, 0.5]])
    t = Target(3, D, mean=np.zeros(D), prec=np.linalg.inv(a),
               norm_const=-(D * np.log(2 * np.pi) + np.log(np.linalg.det(a))) / 2)
    x0 = np.random.default_rng(3).standard_normal((C_, D))
    st = oracle.nuts_state(C_, np.float64)
    m = oracle.nuts_mass(2, C_, D, np.float64, start_buffer=10, end_buffer=10, initial_window=20)
    _, smp, _, _ = oracle.nuts_mass_run(t, x0, st, m, 0.8, 10, 7, 0, 50, 200, False, 4, 1)
    assert np.all(m.kind == 2) and np.all(np.isfinite(smp))
    for c in range(C_):
        np.testing.assert_allclose(m.minv[c] @ (m.mchol[c] @ m.mchol[c].T), np.eye(D), atol=1e-8)
