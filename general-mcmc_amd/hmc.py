"""Data-parallel HMC (hmc.rs:75-339 over batched_hmc.rs:29-216).

    sampler = HMC(RosenbrockND(), init_det(4096, 64, np.float32), 0.01, 50).set_seed(42)
    sample = sampler.run(100, 100)            # [chains, n_collect, dim]
    sample, stats = sampler.run_progress(100, 100)

One transition of every chain is one pass of the fused gfx950 kernel
(momentum draw, kinetic energy, L leapfrogs with the analytic gradient,
Metropolis accept); positions stay on the device between calls.
"""
from __future__ import annotations

import numpy as np

from ._sampler import Sampler


class HMC(Sampler):
    _progress_prefix = "HMC"
    _progress_interval = 0.5  # seconds between progress reports

    def __init__(self, target, initial_positions, step_size: float, n_leapfrog: int,
                 dtype=None, chain_offset: int = 0):
        self._step_size = float(step_size)
        self._n_leapfrog = int(n_leapfrog)
        super().__init__(lambda lib: lib.gm_hmc_create, target, initial_positions, dtype,
                         chain_offset, self._step_size, self._n_leapfrog)

    def set_seed(self, seed: int) -> "HMC":
        """hmc.rs:143-148 (engine streams are per sampler, not backend-global)."""
        return self._seed(seed)

    def step_size(self) -> float:
        return self._step_size

    def n_leapfrog(self) -> int:
        return self._n_leapfrog
