"""Convergence diagnostics (stats.rs), computed on the GPU.

split_rhat_mean_ess  stats.rs:439-450 (R-hat = sqrt(W/V), the reference's
                     orientation, stats.rs:452-454; ESS via Geyer's initial
                     monotone sequence, stats.rs:523-573)
basic_stats          stats.rs:342-368
RunStats             stats.rs:371-394
MultiChainTracker    stats.rs:199-339 (device); ChainTracker stats.rs:24-131 runs
                     fused in the MH / NUTS kernels during run_progress
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import NamedTuple

import numpy as np

from . import _lib


def split_rhat_mean_ess(sample) -> tuple[np.ndarray, np.ndarray]:
    """sample: [chains, draws, params] (host array). Returns (rhat, ess), f32."""
    x = np.asarray(sample)
    if x.dtype not in (np.float32, np.float64):
        x = x.astype(np.float64)
    x = np.ascontiguousarray(x)
    if x.ndim != 3:
        raise ValueError("sample must be [chains, draws, params]")
    c, n, p = x.shape
    rhat = np.empty(p, dtype=np.float32)
    ess = np.empty(p, dtype=np.float32)
    lib = _lib.require_gpu()
    _lib.check(lib.gm_split_rhat_ess(_lib.ptr(x), _lib.dtype_code(x.dtype), c, n, p,
                                     _lib.ptr(rhat), _lib.ptr(ess)))
    return rhat, ess


def split_rhat_mean_ess_device(dev_ptr: int, dtype, n_chains: int, n_draws: int, n_params: int,
                               strides: tuple[int, int, int]):
    """Same, on device memory (element strides: chain, draw, param)."""
    rhat = np.empty(n_params, dtype=np.float32)
    ess = np.empty(n_params, dtype=np.float32)
    lib = _lib.require_gpu()
    _lib.check(lib.gm_split_rhat_ess_device(C.c_void_p(dev_ptr), _lib.dtype_code(dtype), n_chains,
                                            n_draws, n_params, strides[0], strides[1], strides[2],
                                            _lib.ptr(rhat), _lib.ptr(ess)))
    return rhat, ess


@dataclass
class BasicStats:
    name: str
    min: float
    median: float
    max: float
    mean: float
    std: float

    def __str__(self) -> str:
        return (f"{self.name} in [{self.min:.2f}, {self.max:.2f}], median: {self.median:.2f}, "
                f"mean: {self.mean:.2f} ± {self.std:.2f}")


def basic_stats(name: str, data) -> BasicStats:
    """stats.rs:342-368: sort descending; min = last, max = first, median =
    element len/2 of the descending order; std with ddof = 1."""
    d = np.sort(np.asarray(data, dtype=np.float32))[::-1]
    std = float(np.std(d, ddof=1)) if len(d) > 1 else float("nan")
    return BasicStats(name, float(d[-1]), float(d[len(d) // 2]), float(d[0]),
                      float(np.mean(d, dtype=np.float32)), std)


@dataclass
class RunStats:
    ess: BasicStats
    rhat: BasicStats

    @classmethod
    def from_sample(cls, sample) -> "RunStats":
        rhat, ess = split_rhat_mean_ess(sample)
        return cls.from_arrays(rhat, ess)

    @classmethod
    def from_arrays(cls, rhat, ess) -> "RunStats":
        return cls(basic_stats("ESS", ess), basic_stats("Split R-hat", rhat))

    def __str__(self) -> str:
        return f"{self.ess}\n{self.rhat}"


# ---- live run_progress statistics (stats.rs:24-339) ----------------------

class Progress(NamedTuple):
    """One progress report of run_progress: transitions done of total, the
    tracker acceptance estimate and max R-hat (NaN skipped)."""
    done: int
    total: int
    p_accept: float
    max_rhat: float


@dataclass
class ChainStats:
    """ChainTracker::stats (stats.rs:35-46, 122-131) for every chain."""
    n: int
    p_accept: np.ndarray  # [C]
    mean: np.ndarray      # [C, dim]
    sm2: np.ndarray       # [C, dim]


def _print_progress(prefix: str):
    """A one-line progress bar on stderr in the reference's format
    ("{prefix:8} {bar:40} {pos}/{len} | p(accept)≈.. max(rhat)≈..")."""
    import sys

    def show(p: Progress):
        frac = p.done / p.total if p.total else 1.0
        fill = int(round(40 * frac))
        bar = "=" * max(fill - 1, 0) + (">" if 0 < fill < 40 else "=" if fill else "") + "-" * (40 - fill)
        msg = f"p(accept)≈{p.p_accept:.2f} max(rhat)≈{p.max_rhat:.2f}"
        end = "\n" if p.done >= p.total else "\r"
        sys.stderr.write(f"{prefix:8} {bar} {p.done}/{p.total} | {msg}{end}")
        sys.stderr.flush()
    return show


class MultiChainTracker:
    """MultiChainTracker (stats.rs:199-339) on the device: step() with the
    [n_chains, n_params] positions (host array, or a device pointer with
    its dtype), then p_accept / rhat() / max_rhat()."""

    def __init__(self, n_chains: int, n_params: int):
        self.lib = _lib.require_gpu()
        self.n_chains, self.n_params = int(n_chains), int(n_params)
        h = C.c_void_p()
        _lib.check(self.lib.gm_mct_create(self.n_chains, self.n_params, C.byref(h)))
        self.h = h
        self._dev = None

    def step(self, x=None, *, dev_ptr: int | None = None, dtype=np.float32) -> None:
        if dev_ptr is None:
            a = np.ascontiguousarray(x)
            if a.shape != (self.n_chains, self.n_params):
                raise ValueError("positions must be [n_chains, n_params]")
            if a.dtype not in (np.float32, np.float64):
                a = a.astype(np.float64)
            if self._dev is None or self._dev.dtype != a.dtype:
                from .batch_vector import DeviceMatrix
                self._dev = DeviceMatrix(a.shape, a.dtype)
            _lib.check(self.lib.gm_memcpy_htod(C.c_void_p(self._dev.ptr), _lib.ptr(a), a.nbytes))
            dev_ptr, dtype = self._dev.ptr, a.dtype
        _lib.check(self.lib.gm_mct_step(self.h, C.c_void_p(dev_ptr), _lib.dtype_code(dtype)))

    @property
    def p_accept(self) -> float:
        p = C.c_float()
        _lib.check(self.lib.gm_mct_stats(self.h, C.byref(p), None, None))
        return p.value

    def rhat(self) -> np.ndarray:
        r = np.empty(self.n_params, dtype=np.float32)
        _lib.check(self.lib.gm_mct_stats(self.h, None, _lib.ptr(r), None))
        return r

    def max_rhat(self) -> float:
        m = C.c_float()
        _lib.check(self.lib.gm_mct_stats(self.h, None, None, C.byref(m)))
        return m.value

    def close(self):
        if getattr(self, "h", None) is not None:
            self.lib.gm_mct_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
