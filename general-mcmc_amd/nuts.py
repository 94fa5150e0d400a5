"""No-U-Turn sampler (nuts.rs:89-438 over generic_nuts.rs).

NUTS(target, initial_positions, target_accept_p).set_seed(s).run(n_collect, n_discard)
keeps the reference's step-count conventions:
run performs n_collect + n_discard - 1 transitions (row 0 is the start when
n_discard == 0); run_progress performs n_collect + n_discard.
Every chain runs its own trajectory tree on the GPU (identity mass matrix,
dual-averaging step size, as NUTS::new configures GenericNUTS).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._sampler import Sampler


class NUTS(Sampler):
    _progress_prefix = "Global"
    _progress_interval = 1.0  # seconds between progress reports

    def __init__(self, target, initial_positions, target_accept_p: float, dtype=None,
                 max_depth: int = 0, chain_offset: int = 0):
        self.target_accept_p = float(target_accept_p)
        super().__init__(lambda lib: lib.gm_nuts_create, target, initial_positions, dtype,
                         chain_offset, self.target_accept_p, int(max_depth))

    def set_seed(self, seed: int) -> "NUTS":
        """nuts.rs:299-304 / generic_nuts.rs:550-556."""
        return self._seed(seed)

    def step_sizes(self) -> tuple[np.ndarray, np.ndarray]:
        """Per-chain (epsilon, epsilon_bar)."""
        eps = np.empty(self.n_chains, dtype=np.float64)
        bar = np.empty(self.n_chains, dtype=np.float64)
        _lib.check(self._lib.gm_nuts_get_step_size(self._h, _lib.ptr(eps), _lib.ptr(bar)))
        return eps, bar


class NUTSChain:
    """Single-chain facade (nuts.rs:311-438): run returns [n_collect, dim]."""

    def __init__(self, target, initial_position, target_accept_p: float, dtype=None,
                 max_depth: int = 0):
        x = np.asarray(initial_position)
        self._inner = NUTS(target, x[None, :], target_accept_p, dtype=dtype, max_depth=max_depth)

    def set_seed(self, seed: int) -> "NUTSChain":
        self._inner.set_seed(seed)
        return self

    def run(self, n_collect: int, n_discard: int) -> np.ndarray:
        return self._inner.run(n_collect, n_discard)[0]

    def position(self) -> np.ndarray:
        return self._inner.positions()[0]
