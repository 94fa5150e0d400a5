"""The identity-metric NUTS and the MH arithmetic tied to the reference's op
structure (CPU, oracle only).

The kernels sum every per-chain quantity in the engine's canonical order
(in-lane, then the lane butterfly) and evaluate exp / ln with their own
restatements of msun; the oracle's form 0 is that arithmetic, bit for bit
(the GPU parity tests). The oracle's form 1 is the reference as written:

* NUTS, identity metric (or_nuts_mass_run with mode 0, form 1): the kinetic
  energy `q = q + v * v` left to right (generic_nuts.rs:230-235), the U-turn
  dots `diff.dot(&vel)` left to right (:1369-1377; a burn tensor sum in the
  reference, euclidean.rs:400-403, whose order the backend picks), and the
  C library's exp / ln / pow where the reference calls f64::exp / ln / powf
  (the leaf's min(1, exp(joint - joint0)) :1197, the dual averaging
  :882-893, init_chain_state's mu :750, find_reasonable_epsilon's ln 0.5 and
  ln 2 :1072-1079).
* MH (or_mh_run form 1): MHMarkovChain::step (metropolis_hastings.rs:306-318)
  with IsotropicGaussian's logp (distributions.rs:378-390) and unnorm_logp
  (:398-406) as written: both sums left to right, log q forward and backward
  computed separately, the current state's log-density recomputed, and the
  accept's ln u and the proposal constant's ln from the C library.

Each form 1 is checked here against a pure-Python loop of the reference text
(bit for bit), and tied to form 0 by stated bounds:

  MH at cfg5's shape (IsotropicGaussian(1) 256-D f64, proposal sd 2.38/16),
  from identical states: |d log alpha| <= 1e-13 |lp'| (measured 3.2e-15) and
  <= 2e-12 absolute (measured 4.5e-13); accept decisions differing <= 0.1 %
  (measured 0 of 10,240).
  NUTS at cfg3's shape (the 32-D dense Gaussian, f64, identity metric): per
  chain final step size, tree length, accept count and per-coordinate mean and
  variance within 5 standard errors.

The GPU tests (tests/test_gpu_forms.py) tie the kernels to form 1 at the
configs' own sizes."""
import ctypes
import math

import numpy as np
import pytest

from tests._oracle import Target
from tests.test_oracle_nuts_forms import _mc_close, cfg3_target

_libm = ctypes.CDLL("libm.so.6")
for _f in ("exp", "log"):
    getattr(_libm, _f).restype = ctypes.c_double
    getattr(_libm, _f).argtypes = [ctypes.c_double]
_libm.pow.restype = ctypes.c_double
_libm.pow.argtypes = [ctypes.c_double, ctypes.c_double]

TAG_MH_PROP, TAG_MH_ACC, TAG_NUTS_MOM, TAG_NUTS_INIT = 4, 5, 6, 11


# --------------------------------------------------------------------- MH
def _ref_mh_run(oracle, std_t, x0, sd, seed, n_steps, collect_from):
    """metropolis_hastings.rs:306-318 with IsotropicGaussian as proposal and
    target, transcribed; the draws are the engine's RNG spec (the proposal
    normals of spec v5, the [0,1) accept uniform)."""
    lib = oracle.lib
    C_, D = x0.shape
    q = x0.copy()
    rows = []
    acc = np.zeros(C_, dtype=np.int64)

    def unnorm_logp(x):                      # distributions.rs:398-406
        s = 0.0
        for v in x:
            s = s + v * v
        return -0.5 * s / (std_t * std_t)

    def prop_logp(frm, to):                  # distributions.rs:378-390
        lp = 0.0
        d = float(len(frm))
        var = sd * sd
        for f, t in zip(frm, to):
            diff = t - f
            lp += -(diff * diff) / (2.0 * var)
        lp += -d * 0.5 * _libm.log(var * math.pi * sd * sd)
        return lp

    for s in range(n_steps):
        row = np.empty((C_, D))
        for c in range(C_):
            cur = [float(v) for v in q[c]]
            prop = [cur[i] + lib.or_tab_normal_d(seed, c, s, TAG_MH_PROP, i) * sd for i in range(D)]
            current_lp = unnorm_logp(cur)
            proposed_lp = unnorm_logp(prop)
            log_q_forward = prop_logp(cur, prop)
            log_q_backward = prop_logp(prop, cur)
            log_accept_ratio = (proposed_lp + log_q_backward) - (current_lp + log_q_forward)
            u = lib.or_uniform_co_d(seed, c, s, TAG_MH_ACC, 0)
            if log_accept_ratio > _libm.log(u):
                q[c] = prop
                acc[c] += 1
            row[c] = q[c]
        if s >= collect_from:
            rows.append(row)
    return q, np.array(rows), acc


def test_mh_reference_form_is_the_reference_text(oracle):
    rng = np.random.default_rng(5)
    C_, D, std_t, sd = 3, 7, 1.3, 0.45
    x0 = rng.standard_normal((C_, D)) * 1.3
    q, smp, acc = oracle.mh_run(Target(2, D, std=std_t), x0, sd, 11, 0, 40, 30, 8, 1, form=1)
    rq, rsmp, racc = _ref_mh_run(oracle, std_t, x0, sd, 11, 40, 30)
    np.testing.assert_array_equal(q, rq)
    np.testing.assert_array_equal(smp, rsmp)
    np.testing.assert_array_equal(acc, racc)
    assert 0 < acc.sum() < 40 * C_
    # and form 0 (the kernels' arithmetic) is a different computation
    la0, _, lnu0 = oracle.mh_terms(Target(2, D, std=std_t), x0, sd, 11, 0, 8, 1, 0)
    la1, _, lnu1 = oracle.mh_terms(Target(2, D, std=std_t), x0, sd, 11, 0, 8, 1, 1)
    assert np.all(np.abs(la0 - la1) <= 1e-13 * np.maximum(np.abs(la1), 1.0))


def test_mh_forms_tied_at_cfg5_shape(oracle):
    """cfg5's target and proposal, 512 chains (the GPU test runs 4096) after
    200 steps from N(0, 1): every 5th of 100 further steps, both forms from the
    same states."""
    C_, D, sd = 512, 256, 2.38 / 16
    t = Target(2, D, std=1.0)
    x0 = np.random.default_rng(0).standard_normal((C_, D))
    _, smp, _ = oracle.mh_run(t, x0, sd, 42, 0, 300, 200, 64, 4, threads=8)
    worst_rel = worst_abs = 0.0
    flips = n = 0
    for k in range(0, 100, 5):
        la0, lp0, lnu0 = oracle.mh_terms(t, smp[k], sd, 42, 300 + k, 64, 4, 0)
        la1, lp1, lnu1 = oracle.mh_terms(t, smp[k], sd, 42, 300 + k, 64, 4, 1)
        d = np.abs(la0 - la1)
        worst_abs = max(worst_abs, float(d.max()))
        worst_rel = max(worst_rel, float((d / np.abs(lp1)).max()))
        flips += int(np.sum((la0 > lnu0) != (la1 > lnu1)))
        n += C_
    assert worst_rel <= 1e-13 and worst_abs <= 2e-12, (worst_rel, worst_abs)
    assert flips <= 1e-3 * n, flips


def test_mh_run_forms_statistics(oracle):
    """run(100, 300) of both forms from the same start: per-coordinate means,
    variances and accept rates within 5 standard errors (64 chains, 32-D)."""
    C_, D, sd = 64, 32, 2.38 / math.sqrt(32)
    t = Target(2, D, std=1.0)
    x0 = np.random.default_rng(8).standard_normal((C_, D))
    res = []
    for form in (0, 1):
        _, smp, acc = oracle.mh_run(t, x0, sd, 3, 0, 400, 100, 32, 1, threads=8, form=form)
        res.append((smp.mean(axis=0), smp.var(axis=0), acc / 400.0))
    for a, b in zip(*res):
        assert _mc_close(a, b) < 5.0


# ------------------------------------------------------------------- NUTS
def _ref_nuts_run(oracle, t, lanes, elems, x0, eps0, n_collect, n_discard, seed, max_depth=10,
                  target_accept=0.8):
    """GenericNUTSChain::run / step / build_tree_with_mass / stop_criterion /
    leapfrog_with_mass / find_reasonable_epsilon (generic_nuts.rs:700-1418)
    under MassMatrix::identity, transcribed. Draws: the engine's RNG spec
    (momenta TAG_NUTS_MOM, the transition's key block for Exp1 and the hashed
    uniforms). The depth cap is the engine's documented deviation (the
    reference has none). Returns per-chain samples, final position, step-size
    state, accept and leapfrog counts."""
    lib = oracle.lib
    C_, D = x0.shape

    def logp_and_grad(q):
        lp, g = oracle.logp_grad(t, np.asarray(q), lanes, elems, np.float64)
        return float(lp[0]), [float(v) for v in g[0]]

    def kinetic(p):                          # :230-235
        q = 0.0
        for v in p:
            q = q + v * v
        return 0.5 * q

    def dot(a, b):
        s = 0.0
        for x, y in zip(a, b):
            s = s + x * y
        return s

    def stop_criterion(qm, qp, pm, pp):      # :1357-1378, identity
        diff = [b - a for a, b in zip(qm, qp)]
        return dot(diff, pm) >= 0.0 and dot(diff, pp) >= 0.0

    counts = {"nlf": 0}

    def leapfrog(q, p, g, eps):              # :1396-1418
        half = 0.5
        p = [pi + gi * (eps * half) for pi, gi in zip(p, g)]
        q = [qi + vi * eps for qi, vi in zip(q, p)]
        lp, g = logp_and_grad(q)
        p = [pi + gi * (eps * half) for pi, gi in zip(p, g)]
        counts["nlf"] += 1
        return q, p, g, lp

    def find_reasonable_epsilon(q0, p0):     # :1025-1102
        eps, half = 1.0, 0.5
        ulogp, g0 = logp_and_grad(q0)
        q, p, g, ulogp1 = leapfrog(q0, p0, g0, eps)
        k = 1.0
        while not (math.isfinite(ulogp1) and all(math.isfinite(v) for v in g)):
            k = k * half
            q, p, g, ulogp1 = leapfrog(q0, p0, g0, eps * k)
        eps = half * k * eps
        la = ulogp1 - ulogp - (kinetic(p) - kinetic(p0))
        a = 1.0 if la > _libm.log(half) else -1.0
        while a * la > -a * _libm.log(2.0):
            eps = eps * _libm.pow(2.0, a)
            q, p, g, ulogp1 = leapfrog(q0, p0, g0, eps)
            la = ulogp1 - ulogp - (kinetic(p) - kinetic(p0))
        return eps

    def build_tree(q, p, g, logu, v, j, eps, joint0, key, ctr):   # :1153-1341
        if j == 0:
            q1, p1, g1, lp1 = leapfrog(q, p, g, float(v) * eps)
            joint = lp1 - kinetic(p1)
            return dict(qm=q1, pm=p1, gm=g1, qp=q1, pp=p1, gp=g1, qprime=q1, gprime=g1, logp_prime=lp1,
                        n=int(logu < joint), s=(logu - 1000.0) < joint,
                        alpha=min(1.0, _libm.exp(joint - joint0)) if joint - joint0 == joint - joint0 else 1.0,
                        n_alpha=1)
        tr = build_tree(q, p, g, logu, v, j - 1, eps, joint0, key, ctr)
        if tr["s"]:
            if v == -1:
                t2 = build_tree(tr["qm"], tr["pm"], tr["gm"], logu, v, j - 1, eps, joint0, key, ctr)
                tr["qm"], tr["pm"], tr["gm"] = t2["qm"], t2["pm"], t2["gm"]
            else:
                t2 = build_tree(tr["qp"], tr["pp"], tr["gp"], logu, v, j - 1, eps, joint0, key, ctr)
                tr["qp"], tr["pp"], tr["gp"] = t2["qp"], t2["pp"], t2["gp"]
            u = lib.or_nuts_u_d(key, 64 + ctr[0])
            ctr[0] += 1
            if u < t2["n"] / max(tr["n"] + t2["n"], 1):
                tr["qprime"], tr["gprime"], tr["logp_prime"] = t2["qprime"], t2["gprime"], t2["logp_prime"]
            tr["n"] += t2["n"]
            tr["s"] = tr["s"] and t2["s"] and stop_criterion(tr["qm"], tr["qp"], tr["pm"], tr["pp"])
            tr["alpha"] = tr["alpha"] + t2["alpha"]
            tr["n_alpha"] += t2["n_alpha"]
        return tr

    gamma, kappa, t0, delta = 0.05, 0.75, 10, target_accept
    total = n_discard + n_collect - 1
    out = []
    for c in range(C_):
        q = [float(v) for v in x0[c]]
        eps, eps_bar, h_bar = float(eps0), 1.0, 0.0
        # init_chain_state (:731-753)
        p_init = [lib.or_normal_d(seed, c, 0, TAG_NUTS_INIT, i) for i in range(D)]
        if abs(eps + 1.0) <= 2.220446049250313e-16:
            eps = find_reasonable_epsilon(q, p_init)
        mu = _libm.log(10.0 * eps)
        counts["nlf"] = 0  # the leapfrog count is the transitions' (the step-size search's are not counted)
        samples = [list(q)] if n_discard == 0 else []
        acc = 0
        for s in range(total):
            m = s + 1
            key, w = oracle.nuts_key(seed, c, s)
            p0 = [lib.or_normal_d(seed, c, s, TAG_NUTS_MOM, i) for i in range(D)]
            logp, g0 = logp_and_grad(q)
            joint = logp - kinetic(p0)
            k = ((w[2] >> 5) << 26) | (w[3] >> 6)
            exp1 = -lib.or_log_d((k + 1) * 1.1102230246251565e-16)
            logu = joint - exp1
            qm, qp, pm, pp, gm, gp = q, q, p0, p0, g0, g0
            j, n, go, alpha, n_alpha = 0, 1, True, 0.0, 0
            ctr = [0]
            while go and j < max_depth:
                v = 1 if lib.or_nuts_u_d(key, 2 * j) < 0.5 else -1
                if v == -1:
                    tr = build_tree(qm, pm, gm, logu, v, j, eps, joint, key, ctr)
                    qm, pm, gm = tr["qm"], tr["pm"], tr["gm"]
                else:
                    tr = build_tree(qp, pp, gp, logu, v, j, eps, joint, key, ctr)
                    qp, pp, gp = tr["qp"], tr["pp"], tr["gp"]
                alpha, n_alpha = tr["alpha"], tr["n_alpha"]
                tmp = min(1.0, tr["n"] / n)
                if tr["s"] and lib.or_nuts_u_d(key, 2 * j + 1) < tmp:
                    q = tr["qprime"]
                    acc += 1
                n += tr["n"]
                go = tr["s"] and stop_criterion(qm, qp, pm, pp)
                j += 1
            eta = 1.0 / (m + t0)
            h_bar = (1.0 - eta) * h_bar + eta * (delta - alpha / n_alpha)
            if m <= n_discard:
                eps = _libm.exp(mu - math.sqrt(m) / gamma * h_bar)
                eta = _libm.pow(float(m), -kappa)
                eps_bar = _libm.exp((1.0 - eta) * _libm.log(eps_bar) + eta * _libm.log(eps))
            else:
                eps = eps_bar
            if 0 <= (s + 1) - n_discard < n_collect:
                samples.append(list(q))
        out.append(dict(samples=np.array(samples), q=np.array(q), eps=eps, eps_bar=eps_bar, h_bar=h_bar, mu=mu,
                        acc=acc, nlf=counts["nlf"]))
    return out


@pytest.mark.parametrize("eps0", [-1.0, 0.3], ids=["find_eps", "given_eps"])
def test_nuts_identity_reference_form_is_the_reference_text(oracle, eps0):
    """6-D dense Gaussian, 3 chains, run(5, 4) (8 transitions: 4 of them
    adapting the step size), f64: the oracle's form 1 equals the transcription
    bit for bit -- samples, final positions, step-size state, accept and
    leapfrog counts."""
    rng = np.random.default_rng(21)
    d = 6
    a = rng.standard_normal((d, d))
    cov = a @ a.T / d + 0.3 * np.eye(d)
    t = Target(3, d, mean=rng.standard_normal(d) * 0.5, prec=np.linalg.inv(cov), norm_const=-2.0)
    C_ = 3
    x0 = rng.standard_normal((C_, d))
    st = oracle.nuts_state(C_, np.float64)
    st["eps"][:] = eps0
    q, smp, acc, nlf = oracle.nuts_run(t, x0, st, 0.8, 10, 17, 0, 5, 4, False, 8, 1, form=1)
    ref = _ref_nuts_run(oracle, t, 8, 1, x0, eps0, 5, 4, 17)
    for c in range(C_):
        np.testing.assert_array_equal(smp[:, c, :], ref[c]["samples"])
        np.testing.assert_array_equal(q[c], ref[c]["q"])
        assert st["eps"][c] == ref[c]["eps"] and st["eps_bar"][c] == ref[c]["eps_bar"]
        assert st["h_bar"][c] == ref[c]["h_bar"] and st["mu"][c] == ref[c]["mu"]
        assert acc[c] == ref[c]["acc"] and nlf[c] == ref[c]["nlf"]
    assert acc.sum() > 0 and nlf.min() >= 8
    # form 0 (the kernels' arithmetic) differs from it, slightly
    st0 = oracle.nuts_state(C_, np.float64)
    st0["eps"][:] = eps0
    q0, _, _, _ = oracle.nuts_run(t, x0, st0, 0.8, 10, 17, 0, 5, 4, False, 8, 1)
    assert not (np.array_equal(q0, q) and np.array_equal(st0["eps_bar"], st["eps_bar"]))


def test_nuts_identity_forms_statistics_cfg3_target(oracle):
    """cfg3's 32-D dense Gaussian under the identity metric, 64 chains,
    run(100, 300) of both forms from the same start (the GPU test runs the
    kernels against form 1 at 512 chains, run(500, 500)): per-chain final step
    size, tree length, accept count and per-coordinate mean and variance
    within 5 standard errors."""
    t = cfg3_target()
    C_, D = 64, 32
    x0 = np.random.default_rng(4).standard_normal((C_, D))
    res = []
    for form in (0, 1):
        st = oracle.nuts_state(C_, np.float64)
        _, smp, acc, nlf = oracle.nuts_run(t, x0, st, 0.8, 10, 9, 0, 100, 300, False, 16, 2, threads=8, form=form)
        res.append((st["eps_bar"].copy(), nlf / 399.0, acc, smp.mean(axis=0), smp.var(axis=0)))
    for x, y in zip(*res):
        assert _mc_close(x, y) < 5.0
    assert not np.array_equal(res[0][3], res[1][3])
