"""The NUTS kernel decides `u < RN(a / b)` (the merge's n''/max(n'+n'', 1)
and the top level's min(1, n'/n), generic_nuts.rs:1305-1306, 860-861)
without the IEEE division on its common path (nuts_device.h
draw_below_ratio): d = RN(RN(u b) - a); d < -a 2^-(P-4) -> true,
d > a 2^-(P-4) -> false, otherwise the quotient decides. This checks the
bounded-error argument behind the fast path in IEEE f64 and f32 arithmetic
(numpy scalars, the same operations and roundings as the kernel) against the
exact decision, on draws placed at and around RN(a/b) where a wrong fast
path would show, and on random draws. The GPU parity tests check the kernel
itself bit for bit against the oracle's division."""
import numpy as np


def fast(u, a, b, dt):
    rel = dt(2.0 ** -49) if dt == np.float64 else dt(2.0 ** -20)
    d = dt(dt(u * b) - a)
    m = dt(a * rel)
    if d < -m:
        return True
    if d > m:
        return False
    return None  # the kernel's division branch


def exact(u, a, b):
    return u < (a / b)  # numpy: the IEEE quotient RN(a/b) in the operands' type


def _check(dt, P, n_pairs, seed):
    rng = np.random.default_rng(seed)
    band = 0
    total = 0
    for _ in range(n_pairs):
        b = int(rng.integers(1, 1 << 20))
        a = int(rng.integers(0, b + 1))
        A, B = dt(a), dt(b)
        q = A / B
        cands = [q]
        x = q
        for _k in range(3):
            x = np.nextafter(x, dt(0))
            cands.append(x)
        x = q
        for _k in range(3):
            x = np.nextafter(x, dt(1))
            cands.append(x)
        cands += [dt(rng.integers(0, 1 << P)) * dt(2.0 ** -P) for _ in range(4)]
        for u in cands:
            # the draws are k 2^-P with k < 2^P: keep candidates on that grid
            if not (0 <= u < 1) or dt(u * dt(2.0 ** P)) != np.floor(u * dt(2.0 ** P)):
                continue
            total += 1
            f = fast(u, A, B, dt)
            if f is None:
                band += 1
                continue
            assert f == exact(u, A, B), (u, a, b)
    return band, total


def test_draw_below_ratio_f64():
    band, total = _check(np.float64, 53, 4000, 1)
    assert total > 20000 and band < total  # the band holds only draws at RN(a/b) and its neighbours


def test_draw_below_ratio_f32():
    band, total = _check(np.float32, 24, 4000, 2)
    assert total > 20000 and band < total


def test_draw_below_ratio_edges():
    for dt in (np.float64, np.float32):
        one = dt(1.0) - (dt(2.0 ** -53) if dt == np.float64 else dt(2.0 ** -24))
        assert fast(dt(0), dt(0), dt(7), dt) is None and not exact(dt(0), dt(0), dt(7))
        assert fast(dt(0.5), dt(0), dt(7), dt) is False
        assert fast(one, dt(5), dt(5), dt) in (True, None) and exact(one, dt(5), dt(5))
        assert fast(dt(0), dt(3), dt(5), dt) is True
