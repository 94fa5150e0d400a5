"""Convergence diagnostics (stats.rs), computed on the GPU.

split_rhat_mean_ess  stats.rs:439-450 (R-hat = sqrt(W/V), the reference's
                     orientation, stats.rs:452-454; ESS via Geyer's initial
                     monotone sequence, stats.rs:523-573)
basic_stats          stats.rs:342-368
RunStats             stats.rs:371-394
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

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
