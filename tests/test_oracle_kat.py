"""Pins the CPU oracle to the reference's own known-answer tests
(tests/golden/reference_kat.json, transcribed from the reference's test
files; each case cites its source). CPU only."""
import json
import math
import os

import numpy as np
import pytest

from tests._oracle import Target

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))


def _gauss2d_target(mean, cov):
    cov = np.asarray(cov, dtype=np.float64)
    # DiffableGaussian2D::new (distributions.rs:229-253)
    det = cov[0, 0] * cov[1, 1] - cov[0, 1] * cov[1, 0]
    inv_det = 1.0 / det
    prec = np.array([[cov[1, 1] * inv_det, -cov[0, 1] * inv_det],
                     [-cov[1, 0] * inv_det, cov[0, 0] * inv_det]])
    two = 2.0
    nc = -(two * math.log(two * math.pi) + math.log(det)) / two
    return Target(3, 2, mean=mean, prec=prec, norm_const=nc)


def test_build_tree_kat(oracle):
    k = KAT["build_tree"]
    t = _gauss2d_target(k["target"]["mean"], k["target"]["cov"])
    i = k["inputs"]
    # RNG-free: n' = 0 makes every merge draw irrelevant; try several streams.
    for seed in (0, 1, 12345):
        out = oracle.build_tree(t, i["q"], i["p"], i["g"], i["logu"], i["v"], i["j"], i["eps"],
                                i["joint0"], seed=seed)
        e, tol = k["expected"], k["tol"]
        for name in ("qm", "pm", "gm", "qp", "pp", "gp", "qprime", "gprime"):
            np.testing.assert_allclose(out[name], e[name], rtol=tol["vec_rel"], atol=tol["vec_abs"],
                                       err_msg=name)
        assert out["n"] == e["n"]
        assert out["s"] == e["s"]
        assert out["n_alpha"] == e["n_alpha"]
        assert abs(out["logp_prime"] - e["logp_prime"]) < tol["logp_abs"]
        assert abs(out["alpha"] - e["alpha"]) < tol["alpha_abs"]


@pytest.mark.parametrize("lanes,elems", [(64, 1), (2, 1), (1, 2)])
def test_find_reasonable_epsilon_kat(oracle, lanes, elems):
    k = KAT["find_reasonable_epsilon"]
    t = Target(2, 2, std=1.0)  # StandardNormal: -sum(0.5 x^2) (nuts.rs:483-496)
    eps = oracle.find_reasonable_epsilon(t, k["inputs"]["q"], k["inputs"]["p"], lanes, elems)
    assert eps == k["expected"]


def test_chain_1_kat(oracle):
    k = KAT["chain_1"]
    t = _gauss2d_target(k["target"]["mean"], k["target"]["cov"])
    st = oracle.nuts_state(1, np.float64)
    q0 = np.array([k["inputs"]["init"]])
    _, samples, _, _ = oracle.nuts_run(t, q0, st, 0.8, 10, 42, 0, 1, 0, False, 64, 1)
    np.testing.assert_allclose(samples[:, 0, :], k["expected"], rtol=k["tol"]["rel"],
                               atol=k["tol"]["abs"])


@pytest.mark.parametrize("case", range(3))
def test_multichain_tracker_rhat_kat(oracle, case):
    k = KAT["mct_rhat"]
    c = k["cases"][case]
    r = oracle.mct_rhat(np.array(c["steps"], dtype=np.float32))
    assert np.max(np.abs(r - np.array(c["expected"], dtype=np.float32))) < k["tol"]


@pytest.mark.parametrize("case", range(2))
@pytest.mark.parametrize("fft", [False, True])
def test_autocov_kat(oracle, case, fft):
    k = KAT["autocov"]
    c = k["cases"][case]
    out = oracle.autocov(np.array(c["x"], dtype=np.float32), fft=fft)
    np.testing.assert_allclose(out, np.array(c["expected"]), atol=k["tol"])


@pytest.mark.parametrize("case", range(3))
def test_iso_gauss_kat(oracle, case):
    c = KAT["iso_gauss"]["cases"][case]
    d = len(c["x"])
    t = Target(2, d, std=c["std"])
    lp, _ = oracle.logp_grad(t, np.array(c["x"]), 64, 1, np.float64)
    lognorm = -(d / 2.0) * (math.log(2.0) + math.log(math.pi) + 2.0 * math.log(c["std"]))
    p = math.exp(lp[0] + lognorm)
    assert abs(p - c["expected_p"]) < c["tol"]


def test_gaussian2d_logp_kat(oracle):
    k = KAT["gaussian2d_logp"]
    cov = np.array(k["cov"])
    det = cov[0, 0] * cov[1, 1] - cov[0, 1] * cov[1, 0]
    prec = np.array([[cov[1, 1], -cov[0, 1]], [-cov[1, 0], cov[0, 0]]]) / det
    # Normalized::logp (distributions.rs:172-190): -ln(2 pi) - 0.5 ln|det| - 0.5 d'P d
    nc = -math.log(2.0 * math.pi) - 0.5 * math.log(abs(det))
    t = Target(3, 2, mean=k["mean"], prec=prec, norm_const=nc)
    lp, _ = oracle.logp_grad(t, np.array(k["x"]), 64, 1, np.float64)
    assert abs(lp[0] - k["expected"]) < k["tol"]


def test_ess_iid_uniform(oracle):
    """ess_1 (stats.rs:841-865) with the engine's uniform stream."""
    k = KAT["ess_iid_uniform"]
    u = np.array([[oracle.lib.or_uniform_co_f(42, c, t, 99, 0) for t in range(1000)]
                  for c in range(4)], dtype=np.float32)[:, :, None]
    r, e = oracle.split_rhat_ess(u)
    assert e.min() > k["expected"]["ess_min_gt"]
    assert r.max() < k["expected"]["rhat_max_lt"]


def test_split_rhat_ess_threads_bitwise(oracle):
    """or_split_rhat_ess_mt (the config-size parity tests' oracle) splits the
    parameters over threads; parameters are independent in stats.rs:456-573,
    so the result is bitwise the single-thread restatement's."""
    rng = np.random.default_rng(11)
    x = (np.cumsum(rng.standard_normal((37, 120, 13)), axis=1) * 0.1
         + rng.standard_normal((37, 120, 13))).astype(np.float32)
    r1, e1 = oracle.split_rhat_ess(x)
    for t in (2, 5, 13, 40):
        rt, et = oracle.split_rhat_ess(x, threads=t)
        np.testing.assert_array_equal(rt, r1)
        np.testing.assert_array_equal(et, e1)
