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
