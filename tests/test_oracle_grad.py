"""The Rosenbrock gradient forms of the oracle (and so, by the bit-exact GPU
parity tests, of the kernels) against the mathematics.

The reference differentiates `RosenbrockND::unnorm_logp_batch`
(distributions.rs:544-554) with burn autodiff, so its gradient is the exact
derivative up to rounding; no reference fixture pins its bits (SURVEY.md
§8(c)). This test pins both engine forms -- the 64-lane fused-multiply-add
form (lanes >= 64, wide chains) and the select form (narrower groups) -- to
the closed-form derivative evaluated in float64, and the float64 forms also to
central finite differences of the oracle's own log-density.
"""
import numpy as np
import pytest

from tests._oracle import Target


def rosen_logp(x, a=1.0, b=100.0):
    return -(b * (x[..., 1:] - x[..., :-1] ** 2) ** 2 + (a - x[..., :-1]) ** 2).sum(-1)


def rosen_grad(x, a=1.0, b=100.0):
    g = np.zeros_like(x)
    t = x[..., 1:] - x[..., :-1] ** 2
    g[..., :-1] += 4 * b * x[..., :-1] * t + 2 * (a - x[..., :-1])
    g[..., 1:] -= 2 * b * t
    return g


LAYOUTS = [(64, 1), (64, 2), (32, 2), (16, 4), (128, 4)]  # 64-lane FMA form, select form, wide


@pytest.mark.parametrize("lay", LAYOUTS)
@pytest.mark.parametrize("dtype,rtol", [(np.float64, 1e-13), (np.float32, 2e-5)])
def test_rosenbrock_grad_matches_derivative(oracle, lay, dtype, rtol):
    lanes, elems = lay
    D = min(lanes * elems, 200)
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((16, D)) * 0.8).astype(dtype)
    t = Target(1, D, a=1.0, b=100.0)
    lp, g = oracle.logp_grad(t, x, lanes, elems, dtype)
    x64 = x.astype(np.float64)
    ref_g = rosen_grad(x64)
    scale = np.abs(ref_g).max(axis=1, keepdims=True) + 1.0
    assert np.all(np.abs(g - ref_g) <= rtol * 64 * scale), np.abs(g - ref_g).max()
    np.testing.assert_allclose(lp, rosen_logp(x64), rtol=rtol * 8)


@pytest.mark.parametrize("lay", [(64, 1), (32, 2)])
def test_rosenbrock_grad_central_differences(oracle, lay):
    lanes, elems = lay
    D = lanes * elems
    rng = np.random.default_rng(11)
    x = rng.standard_normal((4, D)) * 0.7
    t = Target(1, D, a=1.0, b=100.0)
    _, g = oracle.logp_grad(t, x, lanes, elems, np.float64)
    h = 1e-6
    fd = np.empty_like(x)
    for i in range(D):
        xp, xm = x.copy(), x.copy()
        xp[:, i] += h
        xm[:, i] -= h
        lp_p, _ = oracle.logp_grad(t, xp, lanes, elems, np.float64)
        lp_m, _ = oracle.logp_grad(t, xm, lanes, elems, np.float64)
        fd[:, i] = (lp_p - lp_m) / (2 * h)
    np.testing.assert_allclose(g, fd, rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("dtype,tol", [(np.float64, 1e-11), (np.float32, 2e-4)])
def test_hmc_leapfrog_forms_agree_to_rounding(oracle, dtype, tol):
    """The oracle's two HMC leapfrog forms: 0, the engine's (kicks and drift
    as fused multiply-adds, the kernels), and 1, the reference's op structure
    (product and sum rounded separately, batched_hmc.rs:166-190 through
    add_scaled_assign, the composed tier-2 ops). The same integrator in exact
    arithmetic: one transition's proposals agree to rounding, and over a run
    the accept rates match."""
    C_, D, L = 32, 64, 20
    x0 = (np.random.default_rng(4).standard_normal((C_, D)) * 0.5).astype(dtype)
    t = Target(1, D, a=1.0, b=100.0)
    _, s0, _ = oracle.hmc_run(t, x0, 0.005, L, 3, 0, 1, 0, 64, 1, form=0)
    _, s1, _ = oracle.hmc_run(t, x0, 0.005, L, 3, 0, 1, 0, 64, 1, form=1)
    assert not np.array_equal(s0, s1)  # the roundings differ ...
    np.testing.assert_allclose(s0, s1, rtol=tol, atol=tol)  # ... and nothing else
    _, _, a0 = oracle.hmc_run(t, x0, 0.005, L, 3, 0, 40, 40, 64, 1, form=0)
    _, _, a1 = oracle.hmc_run(t, x0, 0.005, L, 3, 0, 40, 40, 64, 1, form=1)
    assert abs(a0.mean() - a1.mean()) < 2.0  # of 40 transitions per chain
