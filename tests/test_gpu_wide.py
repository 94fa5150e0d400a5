"""dim > 1024: one chain per workgroup (hmc_wide_kernel). Samples, positions
and accept counts bit-for-bit against the oracle under the wide layout's
declared summation order (each wave's 64-lane order, wave totals left to
right), including the reference's 10,000-dimensional Rosenbrock benchmark
shape (hmc.rs:757-791: 6 chains, eps 0.01, 50 leapfrogs)."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu


def start(g, n, d, dtype, scale=0.5):
    return (g.init_with_seed(n, d, 5, np.float64) * scale).astype(dtype)


def wide_default(dim, dtype):
    esz = 4 if dtype == np.float32 else 8
    for e in (4, 8, 16, 32):
        if e == 32 and esz == 8:
            continue
        maxt = 1024 if esz * e <= 32 else 512
        w = -(-dim // (64 * e))
        if w * 64 <= maxt:
            return 64 * max(w, 2), e
    raise AssertionError(dim)


@pytest.mark.parametrize("dtype,dim", [(np.float32, 1025), (np.float64, 1025), (np.float32, 3000),
                                       (np.float64, 4096), (np.float32, 6000), (np.float64, 5000),
                                       (np.float32, 12000)])
def test_hmc_wide_bitwise(gm, oracle, dtype, dim):
    n_chains, L, eps = 3, 6, 0.01
    x0 = start(gm, n_chains, dim, dtype)
    for name, t in [("rosenbrock", gm.RosenbrockND()), ("iso", gm.IsotropicGaussian(1.3))]:
        s = gm.HMC(t, x0, eps, L, dtype=dtype).set_seed(7)
        lay = s.layout()
        assert lay == wide_default(dim, dtype), lay
        s.set_steps_per_launch(3)  # state hand-off across launches mid draw block
        out = s.run(4, 3)
        q, samples, acc = oracle.hmc_run(Target.from_product(t, dim), x0, eps, L, 7, 0, 7, 3, *lay)
        np.testing.assert_array_equal(out, samples.transpose(1, 0, 2), err_msg=name)
        np.testing.assert_array_equal(s.positions(), q, err_msg=name)
        np.testing.assert_array_equal(s.accept_counts(), acc, err_msg=name)
        s.close()


@pytest.mark.parametrize("lay", [(128, 16), (256, 8), (512, 4), (640, 4)])
def test_hmc_wide_layouts(gm, oracle, lay):
    dim, dtype = 2000, np.float32
    x0 = start(gm, 2, dim, dtype)
    t = gm.RosenbrockND()
    s = gm.HMC(t, x0, 0.005, 4, dtype=dtype).set_seed(3)
    s.set_layout(*lay)
    out = s.run(3, 1)
    q, samples, acc = oracle.hmc_run(Target.from_product(t, dim), x0, 0.005, 4, 3, 0, 4, 1, *lay)
    np.testing.assert_array_equal(out, samples.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.accept_counts(), acc)


def test_hmc_10000d_reference_benchmark_shape(gm, oracle):
    """test_bench_10000d (hmc.rs:757-791): 6 chains x 10,000-D RosenbrockND,
    eps 0.01, 50 leapfrogs; all chains start at one N(0,1) draw."""
    dim, n = 10000, 6
    x0 = np.repeat(gm.init_with_seed(1, dim, 42, np.float32), n, axis=0)
    s = gm.HMC(gm.RosenbrockND(), x0, 0.01, 50).set_seed(42)
    out = s.run(3, 2)
    assert out.shape == (n, 3, dim)
    q, samples, acc = oracle.hmc_run(Target.from_product(gm.RosenbrockND(), dim), x0, 0.01, 50, 42,
                                     0, 5, 2, *s.layout())
    np.testing.assert_array_equal(out, samples.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.accept_counts(), acc)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_logp_grad_wide_bitwise(gm, oracle, dtype):
    dim = 3001
    x = start(gm, 5, dim, dtype, 1.1)
    for t in (gm.RosenbrockND(), gm.IsotropicGaussian(0.8)):
        lp, g = t.unnorm_logp_and_grad_batch(x, dtype)
        olp, og = oracle.logp_grad(Target.from_product(t, dim), x, *wide_default(dim, dtype), dtype)
        np.testing.assert_array_equal(lp, olp)
        np.testing.assert_array_equal(g, og)


def test_wide_limits_raise(gm):
    x0 = gm.init_det(2, 2000)
    with pytest.raises(Exception):
        gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(0.1), x0)
    with pytest.raises(Exception):
        gm.NUTS(gm.IsotropicGaussian(1.0), x0, 0.8)
    with pytest.raises(Exception):
        gm.HMC(gm.DenseGaussian(np.zeros(2000), np.eye(2000)), x0, 0.1, 2)
    with pytest.raises(Exception):
        gm.HMC(gm.RosenbrockND(), gm.init_det(2, 9000), 0.1, 2, dtype=np.float64)
    s = gm.HMC(gm.RosenbrockND(), gm.init_det(2, 100, np.float32), 0.1, 2)
    with pytest.raises(Exception):
        s.set_layout(128, 4)  # wide layouts need dim > half of their coordinates
    m = gm.MetropolisHastings(gm.IsotropicGaussian(1.0), gm.IsotropicGaussian(0.1), gm.init_det(2, 900))
    with pytest.raises(Exception):
        m.set_layout(128, 8)
