"""User targets (CustomTarget: HIP source compiled at run time into the
engine's own sampler kernels). The built-in targets restated as user code in
the oracle's one-chain-per-lane arithmetic must give the oracle's samples bit
for bit -- the runtime-compiled kernels are the ahead-of-time kernels."""
import numpy as np
import pytest

from tests import custom_targets as ct
from tests._oracle import Target

pytestmark = pytest.mark.gpu

DTYPES = [np.float32, np.float64]


def _var(dtype, std):
    return float(dtype(std) * dtype(std))


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("dim", [1, 2, 8, 33])
def test_custom_logp_grad(gm, oracle, dtype, dim):
    x = (gm.init_with_seed(17, dim, 2, np.float64) * 1.2).astype(dtype)
    for src, params, ot in [(ct.ROSENBROCK, [1.0, 100.0], Target(1, dim, a=1.0, b=100.0)),
                            (ct.ISO_GAUSS, [_var(dtype, 1.7)], Target(2, dim, std=1.7))]:
        t = gm.CustomTarget(src, dim, params)
        lp, g = t.unnorm_logp_and_grad_batch(x, dtype)
        olp, og = oracle.logp_grad(ot, x, 1, dim, dtype)
        np.testing.assert_array_equal(lp, olp)
        np.testing.assert_array_equal(g, og)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("dim", [3, 16])
def test_custom_hmc_bitwise(gm, oracle, dtype, dim):
    x0 = (gm.init_with_seed(40, dim, 4, np.float64) * 0.5).astype(dtype)
    t = gm.CustomTarget(ct.ROSENBROCK, dim, [1.0, 100.0])
    s = gm.HMC(t, x0, 0.01, 6, dtype=dtype).set_seed(21)
    assert s.layout() == (1, dim)
    s.set_steps_per_launch(3)
    out = s.run(5, 2)
    q, smp, acc = oracle.hmc_run(Target(1, dim, a=1.0, b=100.0), x0, 0.01, 6, 21, 0, 7, 2, 1, dim)
    np.testing.assert_array_equal(out, smp.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.accept_counts(), acc)


@pytest.mark.parametrize("dtype", DTYPES)
def test_custom_mh_bitwise(gm, oracle, dtype):
    dim = 6
    x0 = gm.init_with_seed(33, dim, 5, np.float64).astype(dtype)
    t = gm.CustomTarget(ct.ISO_GAUSS, dim, [_var(dtype, 1.3)])
    prop = gm.IsotropicGaussian(0.6)
    s = gm.MetropolisHastings(t, prop, x0, dtype=dtype).seed(7)
    out = s.run(6, 3)
    q, smp, acc = oracle.mh_run(Target(2, dim, std=1.3), x0, 0.6, 7, 0, 9, 3, 1, dim)
    np.testing.assert_array_equal(out, smp.transpose(1, 0, 2).astype(np.float64))
    np.testing.assert_array_equal(s.accept_counts(), acc)


@pytest.mark.parametrize("dtype", DTYPES)
def test_custom_nuts_bitwise(gm, oracle, dtype):
    dim = 4
    x0 = (gm.init_with_seed(20, dim, 6, np.float64) * 0.5).astype(dtype)
    t = gm.CustomTarget(ct.ISO_GAUSS, dim, [_var(dtype, 1.1)])
    s = gm.NUTS(t, x0, 0.8, dtype=dtype, max_depth=6).set_seed(13)
    out = s.run(4, 5)
    st = oracle.nuts_state(20, dtype)
    q, smp, acc, nlf = oracle.nuts_run(Target(2, dim, std=1.1), x0, st, 0.8, 6, 13, 0, 4, 5, False, 1, dim)
    np.testing.assert_array_equal(out, smp.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.leapfrog_counts(), nlf)
    eps, bar = s.step_sizes()
    np.testing.assert_array_equal(eps.astype(dtype), st["eps"])


def test_custom_errors(gm):
    x0 = gm.init_det(4, 3)
    with pytest.raises(gm.GMError, match="undeclared identifier"):
        gm.HMC(gm.CustomTarget(ct.BROKEN, 3), x0, 0.1, 2)
    with pytest.raises(gm.GMError):
        gm.HMC(gm.CustomTarget(ct.ISO_GAUSS, 300, [1.0]), gm.init_det(2, 300), 0.1, 2)
    s = gm.HMC(gm.CustomTarget(ct.ISO_GAUSS, 3, [1.0]), x0, 0.1, 2)
    with pytest.raises(gm.GMError):
        s.set_layout(4, 1)
