"""Tables of the table-driven Box-Muller (RNG spec v5: the f64 MH proposal
normals and the f32 HMC momenta): 128 (1/c_j, ln c_j) pairs,
c_j = 1 + (j + 1/2)/128, for ln m = ln c_j + ln(1 + (m/c_j - 1)) on m in
[1, 2); 256 (sin, cos)(2 pi j/256) pairs for the angle-addition sin/cos. The
f32 tables hold 1/c_j rounded to f32 and ln of the reciprocal of THAT value
(so m * (1/c_j) - 1 stays the exact residual of the f32 factor), and sin/cos
rounded to f32. Also the 64 values 2^(j/64) of the NUTS leaf's table-driven
exp (gm_rng.h leaf_alpha_tab), each the double nearest the exact power
(50-digit decimal arithmetic, then one correctly rounded conversion).
Written as C initializers (hex literals): the kernel (gm_bm_tables.h) and
the oracle hold the same data.

    python tools/make_bm_tables.py > general-mcmc_amd/csrc/gm_bm_tables.h
"""
import decimal
import math

import numpy as np


def main():
    print("// gm_bm_tables.h -- tables of the table-driven Box-Muller (RNG spec v5),")
    print("// written by tools/make_bm_tables.py; oracle/gm_bm_tables.h is the same file.")
    print("#pragma once")
    lg = []
    for j in range(128):
        c = 1.0 + (j + 0.5) / 128.0
        lg += [1.0 / c, math.log(c)]
    print("#define GM_BM_LOG_INIT \\")
    for k in range(0, len(lg), 4):
        print("  " + ", ".join(v.hex() for v in lg[k:k + 4]) + (", \\" if k + 4 < len(lg) else " \\"))
    print("")
    sc = []
    for j in range(256):
        a = 2.0 * math.pi * j / 256.0
        sc += [math.sin(a), math.cos(a)]
    # exact values where they are exact
    for j in range(256):
        if j % 64 == 0:
            q = j // 64
            sc[2 * j], sc[2 * j + 1] = [(0.0, 1.0), (1.0, 0.0), (0.0, -1.0), (-1.0, 0.0)][q]
    print("#define GM_BM_SINCOS_INIT \\")
    for k in range(0, len(sc), 4):
        print("  " + ", ".join(float(v).hex() for v in sc[k:k + 4]) + (", \\" if k + 4 < len(sc) else " \\"))
    print("")
    lg32 = []
    for j in range(128):
        ic = np.float32(1.0 / (1.0 + (j + 0.5) / 128.0))
        lg32 += [ic, np.float32(-math.log(float(ic)))]
    sc32 = [np.float32(v) for v in sc]
    for name, vals in (("GM_BM32_LOG_INIT", lg32), ("GM_BM32_SINCOS_INIT", sc32)):
        print(f"#define {name} \\")
        for k in range(0, len(vals), 4):
            print("  " + ", ".join(float(v).hex() + "f" for v in vals[k:k + 4]) +
                  (", \\" if k + 4 < len(vals) else " \\"))
        print("")
    decimal.getcontext().prec = 50
    ln2 = decimal.Decimal(2).ln()
    e64 = [float((ln2 * j / 64).exp()) for j in range(64)]
    assert e64[0] == 1.0 and all(abs(v - 2.0 ** (j / 64)) <= 2.3e-16 for j, v in enumerate(e64))
    print("#define GM_EXP64_INIT \\")
    for k in range(0, 64, 4):
        print("  " + ", ".join(v.hex() for v in e64[k:k + 4]) + (", \\" if k + 4 < 64 else " \\"))
    print("")


if __name__ == "__main__":
    main()
