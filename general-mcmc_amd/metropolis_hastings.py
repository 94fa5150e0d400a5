"""Random-walk Metropolis-Hastings (metropolis_hastings.rs:90-324) driven like
ChainRunner::run (core.rs:219-229): n_discard + n_collect transitions per
chain, output [chains, n_collect, dim] as float64 (the reference's Trace
conversion, core.rs:39-72, 100-110)."""
from __future__ import annotations

import numpy as np

from ._sampler import Sampler
from .distributions import IsotropicGaussian


class MetropolisHastings(Sampler):
    _progress_prefix = "Global"
    _progress_interval = 1.0  # seconds between progress reports

    def __init__(self, target, proposal: IsotropicGaussian, initial_states, dtype=None,
                 chain_offset: int = 0):
        if not isinstance(proposal, IsotropicGaussian):
            raise TypeError("the device MH kernel implements the IsotropicGaussian proposal")
        self.proposal = proposal
        super().__init__(lambda lib: lib.gm_mh_create, target, initial_states,
                         dtype if dtype is not None else np.float64, chain_offset, proposal.std)

    def seed(self, seed: int) -> "MetropolisHastings":
        """metropolis_hastings.rs:189-197."""
        return self._seed(seed)

    set_seed = seed

    def run(self, n_collect: int, n_discard: int) -> np.ndarray:
        return super().run(n_collect, n_discard).astype(np.float64, copy=False)

    def run_progress(self, n_collect: int, n_discard: int, progress=None, interval=None):
        """ChainRunner::run_progress (core.rs:251-403): f64 samples + RunStats,
        with every chain's ChainTracker stepped on the device each transition."""
        out, stats = super().run_progress(n_collect, n_discard, progress, interval)
        return out.astype(np.float64, copy=False), stats
