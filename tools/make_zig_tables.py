"""Ziggurat tables for the standard normal (Marsaglia & Tsang 2000, 256 layers)
of the round-3 experiment that drew the f64 MH proposal normals by the
ziggurat (measured slower than Box-Muller on the GPU and not kept:
profiles/r03/ab/summary.json).

f(x) = exp(-x^2/2) on x >= 0 is covered by 256 layers of equal area v: layer
0 is the base strip [0, r) x [0, f(r)) plus the tail beyond r (its "width"
X[0] = v / f(r)), layer i >= 1 spans [0, X[i]) x [F[i], F[i+1]) with
X[1] = r, X[i+1] = sqrt(-2 ln(v / X[i] + F[i])), X[256] = 0, F[i] = f(X[i]),
F[256] = 1. r is solved (bisection, f64) so that the top layer's area
X[255] (1 - F[255]) equals v. The experiment compiled the hex literals this
script prints into both the kernel and the oracle.

    python tools/make_zig_tables.py   # prints the C initializers
"""
import math
import sys

N = 256


def layers(r):
    v = r * math.exp(-0.5 * r * r) + math.sqrt(math.pi / 2) * math.erfc(r / math.sqrt(2))
    x = [0.0] * (N + 1)
    x[0] = v / math.exp(-0.5 * r * r)
    x[1] = r
    for i in range(1, N - 1):
        a = v / x[i] + math.exp(-0.5 * x[i] * x[i])
        if a >= 1.0:
            return v, x, -1.0  # r too small: the layers reach the top early
        x[i + 1] = math.sqrt(-2.0 * math.log(a))
    top = x[N - 1] * (1.0 - math.exp(-0.5 * x[N - 1] ** 2))
    return v, x, top - v


def solve():
    lo, hi = 3.0, 4.0  # residual: < 0 at lo (runs out), > 0 at hi
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        _, _, res = layers(mid)
        if res < 0:
            lo = mid
        else:
            hi = mid
    r = hi
    v, x, res = layers(r)
    x[N] = 0.0
    f = [math.exp(-0.5 * t * t) for t in x]
    f[N] = 1.0
    return r, v, x, f


def main():
    r, v, x, f = solve()
    out = sys.stdout
    print(f"/* ziggurat (normal, 256 layers): r = {r!r}, v = {v!r} (tools/make_zig_tables.py) */", file=out)
    for name, t in (("X", x), ("F", f)):
        print(f"#define GM_ZIG_{name}_INIT \\", file=out)
        for k in range(0, N + 1, 4):
            chunk = ", ".join(float(z).hex() for z in t[k:k + 4])
            print(f"  {chunk}{',' if k + 4 <= N else ''} \\", file=out)
        print("", file=out)
    print(f"#define GM_ZIG_R {float(r).hex()}", file=out)


if __name__ == "__main__":
    main()
