"""The f64 MH proposal normals (spec v5, gm_rng.h normals_tab) build their
two uniforms without integer-to-double conversions: u1 = fma(D1, 2^-52, c)
with D1 = 2^52 + (k1 >> 1) assembled from bits and c = -1 + (1 + (k1 & 1))
2^-53, and the angle th = fma(D2, 2 pi 2^-53, -pi) with D2 = 2^52 + (k2 mod
2^45). This restates those formulas in Python with an exactly rounded fma
(Fraction arithmetic, one rounding) and checks them against the spec's
conversions (Unif<double>::oc / ::co, j = floor(256 u2), th = (u2 - j/256)
2 pi) on random and edge words. CPU only; the kernel's bits are pinned
against the oracle by the GPU MH parity tests."""
import random
import struct
from fractions import Fraction

TWO_PI = float.fromhex("0x1.921fb54442d18p+2")
M32 = 2 ** 32 - 1


def _u2d(u):
    return struct.unpack("<d", struct.pack("<Q", u & (2 ** 64 - 1)))[0]


def _fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))  # one correct rounding


def _spec(x, y, z, w):
    k1 = ((x >> 5) << 26) | (y >> 6)
    u1 = float(k1 + 1) * 1.1102230246251565e-16
    k2 = ((z >> 5) << 26) | (w >> 6)
    u2 = float(k2) * 1.1102230246251565e-16
    j = int(u2 * 256.0)
    return u1, j, (u2 - float(j) * 0.00390625) * TWO_PI


def _assembled(x, y, z, w):
    d1 = _u2d(((0x43300000 | (x >> 12)) << 32) | (((x << 20) & 0xFE000000) | (y >> 7)))
    u1 = _fma(d1, 2.0 ** -52, _u2d(0xBFEFFFFFFFFFFFFE if (y & 64) else 0xBFEFFFFFFFFFFFFF))
    d2 = _u2d(((0x43300000 | ((z >> 11) & 0x1FFF)) << 32) | (((z << 21) & 0xFC000000) | (w >> 6)))
    th = _fma(d2, float.fromhex("0x1.921fb54442d18p-51"), -float.fromhex("0x1.921fb54442d18p+1"))
    return u1, z >> 24, th


def test_assembled_uniforms_equal_spec_conversions():
    rng = random.Random(5)
    edge = [(0, 0, 0, 0), (M32, M32, M32, M32), (M32, M32 - 64, 0, M32), (31, 63, 2 ** 24 - 1, 63),
            (2 ** 31, 2 ** 31, 2 ** 31, 2 ** 31), (0, 64, 2 ** 24, 0), (M32, 63, M32, 0)]
    words = edge + [tuple(rng.getrandbits(32) for _ in range(4)) for _ in range(20000)]
    for wd in words:
        assert _assembled(*wd) == _spec(*wd), wd
