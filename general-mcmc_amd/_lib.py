"""ctypes binding of libgmcmc.so (include/gmcmc.h).

The product path has no CPU fallback: if the HIP library is missing, or no
GPU is visible, every sampler raises instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GMCMC_LIB", os.path.join(_HERE, "lib", "libgmcmc.so"))

GM_OK, GM_EINVAL, GM_EHIP, GM_ENOMEM, GM_ERCCL, GM_ESTATE = range(6)
GM_F32, GM_F64 = 0, 1
GM_TARGET_ROSENBROCK, GM_TARGET_ISO_GAUSS, GM_TARGET_GAUSS, GM_TARGET_CUSTOM = 1, 2, 3, 4
UNIQUE_ID_BYTES = 128


class GMError(RuntimeError):
    """A non-zero status from libgmcmc (message from gm_last_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[gmcmc status {code}] {msg}")
        self.code = code


class gm_target(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("reserved", C.c_int32),
        ("dim", C.c_int64),
        ("a", C.c_double),
        ("b", C.c_double),
        ("std", C.c_double),
        ("mean", C.POINTER(C.c_double)),
        ("prec", C.POINTER(C.c_double)),
        ("norm_const", C.c_double),
        ("source", C.c_char_p),
        ("params", C.POINTER(C.c_double)),
        ("n_params", C.c_int64),
    ]


class gm_progress(C.Structure):
    _fields_ = [("done", C.c_int64), ("total", C.c_int64), ("p_accept", C.c_float),
                ("max_rhat", C.c_float)]


PROGRESS_FN = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(gm_progress))

_vp = C.c_void_p
_i64 = C.c_int64
_i32 = C.c_int32
_u64 = C.c_uint64
_dbl = C.c_double
_ip = C.c_int

# name -> (restype, argtypes). Mirrors include/gmcmc.h one-to-one; the test
# suite checks that every symbol the header declares is listed and exported.
SIGNATURES = {
    "gm_last_error": (C.c_char_p, []),
    "gm_device_count": (_ip, [C.POINTER(C.c_int)]),
    "gm_set_device": (_ip, [C.c_int]),
    "gm_device_synchronize": (_ip, []),
    "gm_gauss_from_cov": (_ip, [_i64, _vp, _vp, _vp]),
    "gm_init_positions": (_ip, [_u64, _i64, _i64, _ip, _vp]),
    "gm_init_positions_rows": (_ip, [_u64, _i64, _i64, _i64, _ip, _vp]),
    "gm_target_logp_grad": (_ip, [C.POINTER(gm_target), _ip, _i64, _vp, _vp, _vp]),
    "gm_custom_target_check": (_ip, [C.c_char_p, _ip, _i64, _i32]),
    "gm_hmc_create": (_ip, [C.POINTER(gm_target), _ip, _i64, _i64, _vp, _dbl, _i64, _i64, C.POINTER(_vp)]),
    "gm_mh_create": (_ip, [C.POINTER(gm_target), _ip, _i64, _i64, _vp, _dbl, _i64, C.POINTER(_vp)]),
    "gm_nuts_create": (_ip, [C.POINTER(gm_target), _ip, _i64, _i64, _vp, _dbl, _i32, _i64, C.POINTER(_vp)]),
    "gm_set_seed": (_ip, [_vp, _u64]),
    "gm_step": (_ip, [_vp]),
    "gm_run": (_ip, [_vp, _i64, _i64, _vp]),
    "gm_run_device": (_ip, [_vp, _i64, _i64, C.POINTER(_vp)]),
    "gm_run_device_progress": (_ip, [_vp, _i64, _i64, C.POINTER(_vp)]),
    "gm_run_progress": (_ip, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "gm_copy_samples": (_ip, [_vp, _i64, _vp]),
    "gm_copy_sample_block": (_ip, [_vp, _i64, _i64, _i64, _i64, _vp]),
    "gm_get_positions": (_ip, [_vp, _vp]),
    "gm_set_positions": (_ip, [_vp, _vp]),
    "gm_get_accept_counts": (_ip, [_vp, _vp]),
    "gm_get_leapfrog_counts": (_ip, [_vp, _vp]),
    "gm_nuts_get_step_size": (_ip, [_vp, _vp, _vp]),
    "gm_nuts_set_mass_adaptation": (_ip, [_vp, _i32, _i64, _i64, _i64, _dbl, _dbl, _i64]),
    "gm_nuts_set_lds_levels": (_ip, [_vp, _i32]),
    "gm_nuts_set_dense_forms": (_ip, [_vp, _i32, _i32]),
    "gm_nuts_get_plan": (_ip, [_vp, _vp, _i32]),
    "gm_nuts_set_momentum_pass": (_ip, [_vp, _i32]),
    "gm_build_info": (C.c_char_p, []),
    "gm_nuts_get_mass": (_ip, [_vp, C.POINTER(_i32), _vp, _vp, _vp, _vp, _vp]),
    "gm_sampler_layout": (_ip, [_vp, C.POINTER(_i32), C.POINTER(_i32)]),
    "gm_sampler_set_layout": (_ip, [_vp, _i32, _i32]),
    "gm_sampler_last_run_stats": (_ip, [_vp, C.POINTER(_dbl), C.POINTER(_i64)]),
    "gm_sampler_set_steps_per_launch": (_ip, [_vp, _i64]),
    "gm_sampler_set_unroll": (_ip, [_vp, _i32]),
    "gm_sampler_set_async": (_ip, [_vp, _i32]),
    "gm_sampler_synchronize": (_ip, [_vp]),
    "gm_sampler_reserve": (_ip, [_vp, _i64]),
    "gm_state_size": (_ip, [_vp, C.POINTER(_u64)]),
    "gm_state_save": (_ip, [_vp, _vp, _u64]),
    "gm_state_load": (_ip, [_vp, _vp, _u64]),
    "gm_destroy": (_ip, [_vp]),
    "gm_split_rhat_ess": (_ip, [_vp, _ip, _i64, _i64, _i64, _vp, _vp]),
    "gm_split_rhat_ess_device": (_ip, [_vp, _ip, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp]),
    "gm_comm_get_unique_id": (_ip, [_vp]),
    "gm_comm_init": (_ip, [_vp, _i32, _i32, C.POINTER(_vp)]),
    "gm_comm_destroy": (_ip, [_vp]),
    "gm_comm_info": (_ip, [_vp, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "gm_split_rhat_ess_dist": (_ip, [_vp, _vp, _ip, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp]),
    "gm_split_rhat_ess_shards": (_ip, [_vp, _ip, _ip, _i64, _i64, _i64, _i64, _i64, _i64, _vp, _vp]),
    # run_progress statistics
    "gm_run_progress_cb": (_ip, [_vp, _i64, _i64, _vp, _vp, _vp, PROGRESS_FN, _vp, _dbl]),
    "gm_sampler_chain_stats": (_ip, [_vp, C.POINTER(_u64), _vp, _vp, _vp]),
    "gm_mct_create": (_ip, [_i64, _i64, C.POINTER(_vp)]),
    "gm_mct_step": (_ip, [_vp, _vp, _ip]),
    "gm_mct_stats": (_ip, [_vp, _vp, _vp, _vp]),
    "gm_mct_destroy": (_ip, [_vp]),
    # granular BatchVector ops (tier 2)
    "gm_malloc": (_ip, [C.POINTER(_vp), C.c_size_t]),
    "gm_free": (_ip, [_vp]),
    "gm_memcpy_htod": (_ip, [_vp, _vp, C.c_size_t]),
    "gm_memcpy_dtoh": (_ip, [_vp, _vp, C.c_size_t]),
    "gm_memcpy_dtod": (_ip, [_vp, _vp, C.c_size_t]),
    "gm_bv_kinetic_energy": (_ip, [_ip, _i64, _i64, _vp, _vp]),
    "gm_bv_masked_assign": (_ip, [_ip, _i64, _i64, _vp, _vp, _vp]),
    "gm_bv_add_scaled_assign": (_ip, [_ip, _i64, _vp, _vp, _dbl]),
    "gm_bv_fill_random_normal": (_ip, [_ip, _i64, _i64, _vp, _u64, C.c_uint32, _u64]),
    "gm_bv_sample_uniform": (_ip, [_ip, _i64, _vp, _u64, C.c_uint32, _u64]),
    "gm_bv_energy_sub": (_ip, [_ip, _i64, _vp, _vp, _vp]),
    "gm_bv_energy_add": (_ip, [_ip, _i64, _vp, _vp, _vp]),
    "gm_bv_energy_neg": (_ip, [_ip, _i64, _vp, _vp]),
    "gm_bv_energy_ln": (_ip, [_ip, _i64, _vp, _vp]),
    "gm_bv_accept_mask": (_ip, [_ip, _i64, _vp, _vp, _vp]),
    "gm_bv_scale_assign": (_ip, [_ip, _i64, _vp, _dbl]),
    "gm_bv_fill": (_ip, [_ip, _i64, _vp, _dbl]),
    "gm_bv_dot": (_ip, [_ip, _i64, _vp, _vp, C.POINTER(_dbl)]),
    "gm_bv_target_create": (_ip, [C.POINTER(gm_target), _ip, C.POINTER(_vp)]),
    "gm_bv_logp_and_grad": (_ip, [_vp, _i64, _vp, _vp, _vp]),
    "gm_bv_target_destroy": (_ip, [_vp]),
    "gm_bv_leapfrog": (_ip, [_vp, _i64, _vp, _vp, _vp, _vp, C.c_double]),
}

_lib = None


def load(path: str | None = None) -> C.CDLL:
    """Load libgmcmc.so (raises if it is not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise GMError(GM_ESTATE, f"{p} not found: build it with `make -C general-mcmc_amd` "
                                 "(no CPU fallback exists)")
    lib = C.CDLL(p)
    if path is None and "GMCMC_LIB" not in os.environ:
        _check_build(lib, p)
    for name, (res, args) in SIGNATURES.items():
        if "GMCMC_LIB" in os.environ and not hasattr(lib, name):
            continue  # an A/B build of an earlier tree may predate an entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def build_info(lib=None) -> dict:
    """The loaded library's source digest (gm_build_info, embedded at build
    time) and the digest of the sources in this tree."""
    lib = lib or load()
    fn = getattr(lib, "gm_build_info", None)
    built = None
    if fn is not None:
        fn.restype = C.c_char_p
        built = fn().decode()
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_gm_source_digest", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                                          "source_digest.py"))
    tree = None
    if spec is not None and os.path.exists(spec.origin):
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        tree = "src:" + mod.digest()
    return {"library": built, "tree": tree, "match": built is not None and built == tree}


def _check_build(lib, p) -> None:
    info = build_info(lib)
    if info["tree"] is not None and not info["match"]:
        raise GMError(GM_ESTATE, f"{p} was built from other sources ({info['library']}) than this tree's "
                                 f"({info['tree']}): rebuild with `make -C general-mcmc_amd`")


def check(rc: int) -> None:
    if rc != GM_OK:
        msg = load().gm_last_error()
        raise GMError(rc, msg.decode() if msg else "")


_gpu_checked = False


def require_gpu() -> C.CDLL:
    """The library, after checking that a HIP device is visible."""
    global _gpu_checked
    lib = load()
    if not _gpu_checked:
        n = C.c_int(0)
        rc = lib.gm_device_count(C.byref(n))
        if rc != GM_OK or n.value < 1:
            raise GMError(GM_EHIP, "no HIP device visible: libgmcmc runs on MI355X (gfx950) only")
        _gpu_checked = True
    return lib


def dtype_code(dtype) -> int:
    dt = np.dtype(dtype)
    if dt == np.float32:
        return GM_F32
    if dt == np.float64:
        return GM_F64
    raise ValueError(f"unsupported dtype {dt} (f32 or f64)")


def np_dtype(code: int):
    return np.float32 if code == GM_F32 else np.float64


def ptr(a: np.ndarray) -> C.c_void_p:
    return a.ctypes.data_as(C.c_void_p)
