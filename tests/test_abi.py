"""The C-ABI boundary: libgmcmc.so loads, exports every function that
include/gmcmc.h declares, the Python binding covers exactly that set, and the
host-only entry points behave. No GPU compute here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gmcmc.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gm_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    import general_mcmc_amd as g
    lib = g._lib.load()
    names = header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), f"{n} declared in gmcmc.h but not exported"
    assert sorted(g._lib.SIGNATURES) == names, "ctypes signatures out of sync with gmcmc.h"


def test_gauss_from_cov_matches_reference_formula():
    import general_mcmc_amd as g
    lib = g._lib.load()
    cov = np.array([[4.0, 2.0], [2.0, 3.0]])
    prec = np.empty((2, 2))
    nc = C.c_double()
    g._lib.check(lib.gm_gauss_from_cov(2, g._lib.ptr(cov), g._lib.ptr(prec), C.byref(nc)))
    det = 4 * 3 - 2 * 2
    np.testing.assert_array_equal(prec, np.array([[3.0, -2.0], [-2.0, 4.0]]) * (1.0 / det))
    assert nc.value == -(2.0 * np.log(2.0 * np.pi) + np.log(det)) / 2.0
    rng = np.random.default_rng(1)
    a = rng.standard_normal((32, 32))
    cov = a @ a.T + 32 * np.eye(32)
    prec = np.empty_like(cov)
    g._lib.check(lib.gm_gauss_from_cov(32, g._lib.ptr(cov), g._lib.ptr(prec), C.byref(nc)))
    np.testing.assert_allclose(prec, np.linalg.inv(cov), rtol=1e-10, atol=1e-12)
    sign, logdet = np.linalg.slogdet(cov)
    assert abs(nc.value - (-(32 * np.log(2 * np.pi) + logdet) / 2)) < 1e-9


def test_gauss_from_cov_rejects_indefinite():
    import general_mcmc_amd as g
    lib = g._lib.load()
    cov = np.array([[1.0, 2.0], [2.0, 1.0]])
    prec = np.empty((2, 2))
    nc = C.c_double()
    assert lib.gm_gauss_from_cov(2, g._lib.ptr(cov), g._lib.ptr(prec), C.byref(nc)) == g._lib.GM_EINVAL
    assert b"positive definite" in lib.gm_last_error()


def test_init_positions_match_oracle_stream(oracle):
    """init_det (core.rs:444-449) analogue: N(0,1) from the INIT stream, seed 42."""
    import general_mcmc_amd as g
    x = g.init_det(5, 7)
    ref = np.array([[oracle.lib.or_normal_d(42, c, 0, 1, d) for d in range(7)] for c in range(5)])
    np.testing.assert_array_equal(x, ref)
    assert g.init_det(3, 4, np.float32).dtype == np.float32


def test_init_positions_rows_are_a_slice_of_the_global_start():
    """A shard's rows (gm_init_positions_rows) equal the same rows of the
    whole start, including the multi-threaded path (>= 2^20 draws)."""
    import general_mcmc_amd as g
    full = g.init_with_seed(4200, 256, 42)
    np.testing.assert_array_equal(g.init_with_seed(1000, 256, 42, row0=3000)[:1000], full[3000:4000])
    np.testing.assert_array_equal(g.init_with_seed(7, 256, 42, row0=13), full[13:20])


def test_no_silent_cpu_fallback_without_gpu():
    """Without a visible GPU the samplers must raise, never compute elsewhere."""
    import general_mcmc_amd as g
    lib = g._lib.load()
    n = C.c_int(0)
    if lib.gm_device_count(C.byref(n)) == 0 and n.value > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(g.GMError):
        g.HMC(g.RosenbrockND(), np.zeros((2, 3)), 0.01, 5)


def test_missing_library_fails_loudly(tmp_path):
    import general_mcmc_amd as g
    with pytest.raises(g.GMError):
        g._lib.load(str(tmp_path / "nope.so"))
