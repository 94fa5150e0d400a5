"""The dense Gaussian's matrix-core product (gm_device.h, GaussLane::
mfma_product: v_mfma_f64_4x4x4_4b_f64 for f64 chains laid out 16 lanes x 2
coordinates, D <= 32, or 16 lanes x 4 coordinates, D <= 64) against the oracle's j-ascending fma chain, bit for bit,
in every sampler that evaluates the target: HMC, MH and NUTS. Chain counts
that leave the last wave partly empty (the VALU product runs there) and
dimensions below 32 (zero-padded fragments) are included; the sampler results
must not depend on which product ran."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu

LAY = (16, 2)
LAY4 = (16, 4)  # D in (32, 64]: 16 K-steps, 4 independent accumulations per lane


def _gauss(g, dim, seed):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((dim, dim))
    cov = a @ a.T / dim + np.eye(dim)
    return g.DenseGaussian(rng.standard_normal(dim), cov)


def _start(g, n, d, scale=0.5):
    return g.init_with_seed(n, d, 5, np.float64) * scale


@pytest.mark.parametrize("dim,lay", [(17, LAY), (25, LAY), (32, LAY), (33, LAY4), (48, LAY4), (64, LAY4)])
@pytest.mark.parametrize("n_chains", [8, 14])
def test_hmc_dense_gauss_mfma_bitwise(gm, oracle, dim, lay, n_chains):
    t = _gauss(gm, dim, dim)
    x0 = _start(gm, n_chains, dim)
    s = gm.HMC(t, x0, 0.05, 6, dtype=np.float64).set_seed(4)
    s.set_layout(*lay)
    out = s.run(5, 2)
    q, samples, acc = oracle.hmc_run(Target.from_product(t, dim), x0, 0.05, 6, 4, 0, 7, 2, *lay)
    np.testing.assert_array_equal(out, samples.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.positions(), q)
    np.testing.assert_array_equal(s.accept_counts(), acc)
    s.close()


@pytest.mark.parametrize("dim,lay", [(17, LAY), (32, LAY), (33, LAY4), (64, LAY4)])
@pytest.mark.parametrize("n_chains", [8, 13])
def test_mh_dense_gauss_mfma_bitwise(gm, oracle, dim, lay, n_chains):
    t = _gauss(gm, dim, dim + 1)
    x0 = _start(gm, n_chains, dim, 1.0)
    prop = gm.IsotropicGaussian(2.38 / np.sqrt(dim))
    s = gm.MetropolisHastings(t, prop, x0, dtype=np.float64).seed(6)
    s.set_layout(*lay)
    out = s.run(6, 3)
    q, samples, acc = oracle.mh_run(Target.from_product(t, dim), x0, prop.std, 6, 0, 9, 3, *lay)
    np.testing.assert_array_equal(out, samples.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.accept_counts(), acc)
    s.close()


@pytest.mark.parametrize("dim,lay", [(20, LAY), (32, LAY), (33, LAY4), (48, LAY4), (64, LAY4)])
@pytest.mark.parametrize("n_chains", [8, 10])
def test_nuts_dense_gauss_mfma_bitwise(gm, oracle, dim, lay, n_chains):
    t = _gauss(gm, dim, dim + 2)
    x0 = _start(gm, n_chains, dim)
    s = gm.NUTS(t, x0, 0.8, dtype=np.float64, max_depth=7).set_seed(12)
    s.set_layout(*lay)
    s.set_steps_per_launch(4)
    n_collect, n_discard = 6, 5
    out = s.run(n_collect, n_discard)
    st = oracle.nuts_state(n_chains, np.float64)
    q, samples, acc, nlf = oracle.nuts_run(Target.from_product(t, dim), x0, st, 0.8, 7, 12, 0,
                                           n_collect, n_discard, False, *lay)
    np.testing.assert_array_equal(out, samples.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.accept_counts(), acc)
    np.testing.assert_array_equal(s.leapfrog_counts(), nlf)
    eps, bar = s.step_sizes()
    np.testing.assert_array_equal(eps, st["eps"])
    np.testing.assert_array_equal(bar, st["eps_bar"])
    s.close()
