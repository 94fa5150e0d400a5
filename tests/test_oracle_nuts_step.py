"""The oracle's NUTS::step (nuts.rs:431-433 -> generic_nuts.rs:755-925)
composes with its run: init_chain_state (a run with zero transitions) followed
by k steps is run_progress(k, 0) (generic_nuts.rs:675-716), bit for bit."""
import numpy as np

from tests._oracle import Target


def test_init_then_steps_equals_run_progress(oracle):
    d, n = 6, 5
    rng = np.random.default_rng(1)
    a = rng.standard_normal((d, d))
    prec = np.linalg.inv(a @ a.T / d + np.eye(d))
    t = Target(3, d, mean=rng.standard_normal(d), prec=prec, norm_const=-1.0)
    x0 = rng.standard_normal((n, d)) * 0.5
    lay = (8, 1)
    st1 = oracle.nuts_state(n, np.float64)
    q1, s1, acc1, nlf1 = oracle.nuts_run(t, x0, st1, 0.8, 6, 7, 0, 3, 0, True, *lay)
    st2 = oracle.nuts_state(n, np.float64)
    q0, _, _, _ = oracle.nuts_run(t, x0, st2, 0.8, 6, 7, 0, 1, 0, False, *lay)  # init only
    np.testing.assert_array_equal(q0, x0)
    q2, acc2, nlf2 = oracle.nuts_step(t, q0, st2, 0.8, 6, 7, 0, 3, 0, 0, *lay)
    np.testing.assert_array_equal(q1, q2)
    np.testing.assert_array_equal(acc1, acc2)
    np.testing.assert_array_equal(nlf1, nlf2)
    for k in ("eps", "eps_bar", "h_bar", "mu"):
        np.testing.assert_array_equal(st1[k], st2[k], err_msg=k)
