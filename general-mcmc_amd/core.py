"""Initial positions and the multi-chain runner helpers (core.rs).

`init`, `init_det`, `init_with_seed` (core.rs:434-475) return n x d iid
standard-normal starting points. The reference draws them from
SmallRng + rand_distr (not reproducible outside its crates); here they come
from the engine's Philox stream (tag INIT), computed by libgmcmc on the host.
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib


def init_with_seed(n: int, d: int, seed: int, dtype=np.float64, row0: int = 0) -> np.ndarray:
    """Rows [row0, row0 + n) of the seeded start (row0 > 0: a shard of a
    larger global start, identical to slicing it)."""
    out = np.empty((n, d), dtype=dtype)
    lib = _lib.load()
    _lib.check(lib.gm_init_positions_rows(seed, row0, n, d, _lib.dtype_code(dtype), _lib.ptr(out)))
    return out


def init_det(n: int, d: int, dtype=np.float64) -> np.ndarray:
    """Deterministic start (seed 42, core.rs:444-449)."""
    return init_with_seed(n, d, 42, dtype)


def init(n: int, d: int, dtype=np.float64) -> np.ndarray:
    """Random start (core.rs:434-440)."""
    return init_with_seed(n, d, int.from_bytes(os.urandom(8), "little"), dtype)
