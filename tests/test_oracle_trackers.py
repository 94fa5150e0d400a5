"""The oracle's restatement of the run_progress trackers (stats.rs:24-339)
against an independent float32 NumPy loop written from the reference text
(every operation rounded to f32 in the reference's order)."""
import numpy as np

f = np.float32
ALPHA = f(0.01)


def np_chain_trackers(x0, states):
    C, P = x0.shape
    p = np.full(C, f(-1.0), dtype=np.float32)
    last = x0.astype(np.float32).copy()
    mean = np.zeros((C, P), dtype=np.float32)
    msq = np.zeros((C, P), dtype=np.float32)
    for k, xs in enumerate(states.astype(np.float32)):
        n = f(k + 1)
        for c in range(C):
            for j in range(P):
                mean[c, j] = f(f(f(mean[c, j] * f(n - f(1.0))) + xs[c, j]) / n)
                x2 = f(xs[c, j] * xs[c, j])
                msq[c, j] = x2 if k == 0 else f(f(f(msq[c, j] * f(n - f(1.0))) + x2) / n)
            p0 = p[c] if p[c] >= 0 else f(float(xs[c, 0] != last[c, 0]))
            acc = f(float(np.any(xs[c] != last[c])))
            p[c] = f(f(f(f(1.0) - ALPHA) * p0) + f(ALPHA * acc))
            last[c] = xs[c]
    return p, mean, msq


def np_collect_rhat(n, mean, msq):
    C, P = mean.shape
    nf = f(n)
    nsum = f(0.0)
    for _ in range(C):
        nsum = f(nsum + nf)
    navg = f(nsum / f(C))
    out = np.empty(P, dtype=np.float32)
    for j in range(P):
        w = f(0.0)
        for c in range(C):
            w = f(w + f(f(f(msq[c, j] - f(mean[c, j] * mean[c, j])) * nf) / f(nf - f(1.0))))
        w = f(w / f(C))
        g = f(0.0)
        for c in range(C):
            g = f(g + mean[c, j])
        g = f(g / f(C))
        b = f(0.0)
        for c in range(C):
            d = f(mean[c, j] - g)
            b = f(b + f(d * d))
        b = f(b / f(C * P - 1))
        v = f(b + f(w * f(f(navg - f(1.0)) / navg)))
        out[j] = f(np.sqrt(f(v / w)))
    return out


def np_mct_p_accept(steps):
    p = f(0.0)
    prev = np.zeros(steps.shape[1:], dtype=np.float32)
    for xs in steps:
        for c in range(xs.shape[0]):
            acc = f(float(np.any(xs[c] != prev[c])))
            p = f(f(f(f(1.0) - ALPHA) * p) + f(ALPHA * acc))
        prev = xs
    return p


def test_chain_trackers_and_collect_rhat(oracle):
    rng = np.random.default_rng(4)
    C, P, n = 5, 3, 7
    x0 = rng.standard_normal((C, P)).astype(np.float32)
    states = rng.standard_normal((n, C, P)).astype(np.float32)
    states[2, 1] = states[1, 1]      # a rejected step
    states[4, 3, 0] = states[3, 3, 0]  # first coordinate equal, others not
    p, m, q = oracle.chain_trackers(x0, states)
    ep, em, eq = np_chain_trackers(x0, states)
    np.testing.assert_array_equal(p, ep)
    np.testing.assert_array_equal(m, em)
    np.testing.assert_array_equal(q, eq)
    np.testing.assert_array_equal(oracle.collect_rhat(n, m, q), np_collect_rhat(n, em, eq))


def test_mct_p_accept(oracle):
    rng = np.random.default_rng(6)
    steps = rng.standard_normal((6, 4, 3)).astype(np.float32)
    steps[3, 2] = steps[2, 2]
    assert oracle.mct_p_accept(steps) == np_mct_p_accept(steps)
