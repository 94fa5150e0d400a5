"""Regression: a subtree truncated inside the right half of a doubling is
still merged into its enclosing subtrees (generic_nuts.rs:1245-1341). The
merged alpha / n_alpha feed dual averaging, so the step sizes expose it even
when the positions agree. Found by the mass-matrix tests: DenseGaussian 4-D,
f64, 24 chains, run(1, 5) diverged on chain 22's step size."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("nd", [5, 10, 40])
@pytest.mark.parametrize("lds_levels", [-1, 0, 1])  # subtree stack in LDS / HBM / split
def test_step_sizes_match_oracle(gm, oracle, dtype, nd, lds_levels):
    t = gm.DenseGaussian(np.zeros(4), np.diag([0.04, 1.0, 4.0, 0.5]))
    x0 = gm.init_with_seed(24, 4, 3, dtype)
    s = gm.NUTS(t, x0, 0.8, dtype=dtype).set_seed(11).set_lds_levels(lds_levels)
    lanes, elems = s.layout()
    out = s.run(3, nd)
    st = oracle.nuts_state(24, dtype)
    q, smp, acc, nlf = oracle.nuts_run(Target.from_product(t, 4), x0, st, 0.8, 10, 11, 0, 3, nd, False,
                                       lanes, elems)
    np.testing.assert_array_equal(out, smp.transpose(1, 0, 2))
    eps, bar = s.step_sizes()
    np.testing.assert_array_equal(eps.astype(dtype), st["eps"])
    np.testing.assert_array_equal(bar.astype(dtype), st["eps_bar"])
    np.testing.assert_array_equal(s.leapfrog_counts(), nlf)
