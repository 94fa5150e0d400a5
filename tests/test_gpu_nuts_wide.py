"""NUTS above 256 dimensions on the wide layouts: one chain per workgroup of
lanes/64 waves (nuts_wide.hip; every per-chain sum a block reduction, each
wave's 64-lane total then the waves left to right), bitwise against the
oracle's restatement at the same layout: samples, accept and leapfrog
counts, step sizes; identity and diagonal metric; the dense metric keeps the
one-wave layouts."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu

WIDE = {np.float64: {512: (256, 2), 1024: (512, 2)}, np.float32: {512: (128, 4), 1024: (256, 4)}}


def _targets(gm, name):
    return gm.IsotropicGaussian(1.3) if name == "iso" else gm.RosenbrockND()


def _check(gm, oracle, t, dim, dtype, lay, n_chains=5, max_depth=6, runs=((3, 4),), seed=4, x0=None,
           expect_layout=True):
    if x0 is None:
        x0 = (gm.init_with_seed(n_chains, dim, 2, np.float64) * 0.3).astype(dtype)
    s = gm.NUTS(t, x0, 0.8, dtype=dtype, max_depth=max_depth).set_seed(seed)
    if lay is not None:
        s.set_layout(*lay)
    lanes, elems = s.layout()
    assert lanes > 64 or not expect_layout
    st = oracle.nuts_state(len(x0), dtype)
    q = np.array(x0)
    step = 0
    for nc, nd in runs:
        out = s.run(nc, nd)
        q, smp, acc, nlf = oracle.nuts_run(Target.from_product(t, dim), q, st, 0.8, max_depth, seed, step, nc, nd,
                                           False, lanes, elems)
        np.testing.assert_array_equal(out, smp.transpose(1, 0, 2))
        step += nc + nd
    np.testing.assert_array_equal(s.positions(), q)
    eps, bar = s.step_sizes()
    np.testing.assert_array_equal(eps.astype(dtype), st["eps"])
    np.testing.assert_array_equal(bar.astype(dtype), st["eps_bar"])
    return s


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("dim", [300, 512, 1024])
@pytest.mark.parametrize("target", ["iso", "rosen"])
def test_wide_default_layout_bitwise(gm, oracle, dtype, dim, target):
    """The default NUTS layout above 256 dimensions is a wide one; a partial
    last wave (300 = 4.7 waves of 64 lanes x E) included."""
    t = _targets(gm, target)
    s = _check(gm, oracle, t, dim, dtype, None, max_depth=5 if target == "rosen" else 6)
    want = WIDE[dtype][512 if dim <= 512 else 1024]
    assert s.layout() == want


@pytest.mark.parametrize("lay", [(128, 4), (256, 2), (256, 4), (512, 2)])
def test_wide_layouts_each(gm, oracle, lay):
    dim = lay[0] * lay[1] * 3 // 4  # a partial last wave
    _check(gm, oracle, _targets(gm, "iso"), dim, np.float64, lay, runs=((2, 3), (3, 0)))


def test_wide_diagonal_adaptation_bitwise(gm, oracle):
    """Diagonal metric warm-up on a wide layout (kinetic p^2 inv, drift inv p,
    momentum z sqrt: per-lane products, the sums as every other)."""
    dim, C_ = 300, 6
    t = gm.IsotropicGaussian(1.1)
    x0 = gm.init_with_seed(C_, dim, 8, np.float64)
    cfg = gm.NUTSMassMatrixConfig("diagonal", start_buffer=4, end_buffer=4, initial_window=10)
    s = gm.NUTS.new_with_mass_matrix(t, x0, 0.8, cfg, dtype=np.float64, max_depth=6).set_seed(3)
    lanes, elems = s.layout()
    assert lanes > 64
    out = s.run(6, 40)
    om = oracle.nuts_mass(1, C_, dim, np.float64, start_buffer=4, end_buffer=4, initial_window=10)
    st = oracle.nuts_state(C_, np.float64)
    _, smp, _, _ = oracle.nuts_mass_run(Target.from_product(t, dim), x0, st, om, 0.8, 6, 3, 0, 6, 40, False,
                                        lanes, elems)
    np.testing.assert_array_equal(out, smp.transpose(1, 0, 2))
    m = s.mass_matrix()
    np.testing.assert_array_equal(m.kind, om.kind)
    np.testing.assert_array_equal(m.diag_inv, om.dinv)


def test_wide_dense_request_keeps_one_wave_layout(gm):
    t = gm.IsotropicGaussian(1.0)
    s = gm.NUTS(t, gm.init_det(3, 300), 0.8, dtype=np.float64)
    assert s.layout()[0] > 64
    s.set_mass_adaptation(gm.NUTSMassMatrixConfig("dense", dense_max_dim=400, start_buffer=4, end_buffer=4,
                                                  initial_window=10))
    assert s.layout()[0] <= 64
    with pytest.raises(Exception):
        s.set_layout(256, 2)
