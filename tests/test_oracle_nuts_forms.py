"""The engine's dense-metric NUTS arithmetic tied to the reference's op
structure (CPU, oracle only).

The kernels compute the dense metric's velocity M^-1 p by linearity --
M^-1 (p + g h) = M^-1 p + (M^-1 g) h, so a leapfrog takes one M^-1 product
(of its new gradient) -- with fma-chain products, and the kinetic energy as
0.5 sum p_i v_i from the carried v in the engine's canonical summation order.
The oracle's form 0 is that arithmetic (the GPU tests compare the kernels
with it bit for bit). The oracle's form 1 is the reference as written:
leapfrog_with_mass takes M^-1 of the kicked momentum every leapfrog
(generic_nuts.rs:1409-1417), inv_mul and the kinetic row products are
`acc = acc + inv[i*dim+j] * x[j]` with two roundings, j ascending
(:244-253, :266-273), the kinetic sum runs left to right (:246-253) and the
top-level U-turn takes two fresh products (:1357-1378).

Stated tolerances (engine form vs reference form, measured margins 5-10x):
  one leapfrog   f64: q, p rel 1e-14, M^-1 p rel 1e-13, logp / kinetic rel 1e-14
                 f32: q, p rel 1e-6,  M^-1 p rel 5e-6,  logp / kinetic rel 5e-6
  1024 leapfrogs (a depth-10 trajectory, the default max_depth)
                 f64: q, p, M^-1 p rel 1e-12, |H' - H| 1e-12
                 f32: q, p, M^-1 p rel 5e-4,  |H' - H| 1e-3
(rel = max abs difference / max abs value of the vector.)"""
import numpy as np
import pytest

from tests._oracle import Target

D = 32


def cfg3_target():
    """configs[2]'s target (bench.dense_gauss_32): Sigma = Q diag(logspace(-1,
    1, 32)) Q^T, Q from the QR of a seed-42 N(0, 1) 32x32 matrix."""
    rng = np.random.default_rng(42)
    q, _ = np.linalg.qr(rng.standard_normal((D, D)))
    cov = q @ np.diag(np.logspace(-1, 1, D)) @ q.T
    cov = 0.5 * (cov + cov.T)
    prec = np.linalg.inv(cov)
    prec = 0.5 * (prec + prec.T)
    nc = -(D * np.log(2 * np.pi) + np.linalg.slogdet(cov)[1]) / 2
    return Target(3, D, mean=np.zeros(D), prec=prec, norm_const=nc)


@pytest.fixture(scope="module")
def adapted(oracle):
    """8 chains of cfg3's target after 500 warm-up transitions with dense
    adaptation (the reference's default schedule): their metric, step size and
    position."""
    t = cfg3_target()
    C_ = 8
    x0 = np.random.default_rng(1).standard_normal((C_, D))
    st = oracle.nuts_state(C_, np.float64)
    m = oracle.nuts_mass(2, C_, D, np.float64)
    q, _, _, _ = oracle.nuts_mass_run(t, x0, st, m, 0.8, 10, 7, 0, 1, 500, False, 16, 2)
    assert np.all(m.kind == 2)
    return t, q, st["eps"].copy(), m.minv.copy(), m.mchol.copy()


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


BOUNDS = {  # (dtype, n_leap): (q/p rel, M^-1 p rel, logp/kinetic rel, |dH| abs)
    (np.float64, 1): (1e-14, 1e-13, 1e-14, 1e-12),
    (np.float64, 1024): (1e-12, 1e-12, 1e-12, 1e-12),
    (np.float32, 1): (1e-6, 5e-6, 5e-6, 1e-4),
    (np.float32, 1024): (5e-4, 5e-4, 5e-5, 1e-3),
}


@pytest.mark.parametrize("dtype,n_leap", list(BOUNDS), ids=[f"{d.__name__}-{n}" for d, n in BOUNDS])
def test_dense_trajectory_engine_form_vs_reference_form(oracle, adapted, dtype, n_leap):
    """cfg3_dense's shape (D = 32, the adapted metric, the adapted step size,
    p = L z ~ N(0, M)): one leaf, and a depth-10 trajectory of 1024 leaves from
    the same state, in both forms, agree to the stated bounds."""
    t, q, eps, minv, mchol = adapted
    qp_b, v_b, e_b, h_b = BOUNDS[(dtype, n_leap)]
    worst = np.zeros(4)
    for c in range(len(q)):
        p = (mchol[c] @ np.random.default_rng(100 + c).standard_normal(D)).astype(dtype)
        args = (t, minv[c].astype(dtype), q[c].astype(dtype), p, float(eps[c]), n_leap)
        qa, pa, va, lpa, ka = oracle.dense_traj(*args, 0, 16, 2)
        qb, pb, vb, lpb, kb = oracle.dense_traj(*args, 1, 16, 2)
        assert np.all(np.isfinite(qa)) and np.all(np.isfinite(qb))
        dev = [max(_rel(qa, qb), _rel(pa, pb)), _rel(va, vb),
               max(abs(lpa - lpb) / abs(lpb), abs(ka - kb) / abs(kb)), abs((lpa - ka) - (lpb - kb))]
        worst = np.maximum(worst, dev)
    assert worst[0] <= qp_b and worst[1] <= v_b and worst[2] <= e_b and worst[3] <= h_b, worst


def test_reference_form_is_the_reference_text(oracle):
    """Form 1 restates generic_nuts.rs as written: a pure-Python loop of
    leapfrog_with_mass (:1409-1417, through add_scaled_assign's two roundings)
    with inv_mul (:266-273) and the dense kinetic (:244-253) reproduces it bit
    for bit (D = 5, f64, a dense Gaussian target whose gradient is the
    engine's fma chain, evaluated by the oracle itself)."""
    rng = np.random.default_rng(3)
    d = 5
    a = rng.standard_normal((d, d))
    cov = a @ a.T / d + 0.5 * np.eye(d)
    t = Target(3, d, mean=rng.standard_normal(d), prec=np.linalg.inv(cov), norm_const=-1.5)
    b = rng.standard_normal((d, d))
    m = b @ b.T / d + np.eye(d)
    inv = np.linalg.inv(m)
    q0, p0 = rng.standard_normal(d), rng.standard_normal(d)
    eps, n = 0.17, 7

    def inv_mul(x):
        out = np.zeros(d)
        for i in range(d):
            acc = 0.0
            for j in range(d):
                acc = acc + inv[i, j] * x[j]
            out[i] = acc
        return out

    q, p = q0.copy(), p0.copy()
    _, g = oracle.logp_grad(t, q, d, 1, np.float64)
    g = g[0]
    half = eps * 0.5
    for _ in range(n):
        p = p + g * half
        q = q + inv_mul(p) * eps
        lp, g = oracle.logp_grad(t, q, d, 1, np.float64)
        lp, g = lp[0], g[0]
        p = p + g * half
    ke = 0.0
    for i in range(d):
        row = 0.0
        for j in range(d):
            row = row + inv[i, j] * p[j]
        ke = ke + p[i] * row
    ke = 0.5 * ke
    qb, pb, vb, lpb, kb = oracle.dense_traj(t, inv, q0, p0, eps, n, 1, d, 1)
    np.testing.assert_array_equal(qb, q)
    np.testing.assert_array_equal(pb, p)
    np.testing.assert_array_equal(vb, inv_mul(p))
    assert lpb == lp and kb == ke


def _mc_close(a, b, k=5.0):
    """Per-chain statistics a, b [C] or [C, P] of two runs: the difference of
    their means over chains within k standard errors (chains independent; the
    two runs share seeds and starts, so their difference is smaller still)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    se = np.sqrt(a.var(axis=0, ddof=1) / len(a) + b.var(axis=0, ddof=1) / len(b))
    z = np.abs(a.mean(axis=0) - b.mean(axis=0)) / np.maximum(se, 1e-300)
    return float(np.max(z))


def test_dense_nuts_run_engine_form_vs_reference_form_statistics(oracle):
    """A run with dense adaptation on cfg3's target in both forms, 64 chains,
    run(100, 300): the same chains up to rounding, so per-chain step size,
    tree length, accept count and per-coordinate mean and variance agree
    within 5 standard errors (the GPU test of the kernels against form 1 does
    the same at 512 chains and run(500, 500))."""
    t = cfg3_target()
    C_ = 64
    x0 = np.random.default_rng(2).standard_normal((C_, D))
    res = []
    for form in (0, 1):
        st = oracle.nuts_state(C_, np.float64)
        m = oracle.nuts_mass(2, C_, D, np.float64, form=form)
        _, smp, acc, nlf = oracle.nuts_mass_run(t, x0, st, m, 0.8, 10, 9, 0, 100, 300, False, 16, 2)
        assert np.all(m.kind == 2)
        res.append((st["eps_bar"].copy(), nlf / 399.0, acc, smp.mean(axis=0), smp.var(axis=0)))
    for x, y in zip(*res):
        assert _mc_close(x, y) < 5.0
    # the forms really differ (not one computation twice), yet stay close
    assert not np.array_equal(res[0][3], res[1][3])
