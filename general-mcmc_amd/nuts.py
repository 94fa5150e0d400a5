"""No-U-Turn sampler (nuts.rs:89-438 over generic_nuts.rs).

NUTS(target, initial_positions, target_accept_p).set_seed(s).run(n_collect, n_discard)
keeps the reference's step-count conventions:
run performs n_collect + n_discard - 1 transitions (row 0 is the start when
n_discard == 0); run_progress performs n_collect + n_discard.
Every chain runs its own trajectory tree on the GPU (identity mass matrix,
dual-averaging step size, as NUTS::new configures GenericNUTS).
NUTS.new_with_mass_matrix adds the warm-up metric adaptation of
GenericNUTS::new_with_mass_matrix (generic_nuts.rs:33-359, 379-398).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._sampler import Sampler


@dataclass
class NUTSMassMatrixConfig:
    """NUTSMassMatrixConfig (generic_nuts.rs:43-79): adaptation is "none",
    "diagonal" or "dense"; the defaults are the reference's Default impl."""
    adaptation: str = "diagonal"
    start_buffer: int = 75
    end_buffer: int = 50
    initial_window: int = 25
    regularize: float = 0.05
    jitter: float = 1e-6
    dense_max_dim: int = 75

    @classmethod
    def disabled(cls) -> "NUTSMassMatrixConfig":
        return cls("none", 0, 0, 0, 0.0, 0.0, 0)

    @property
    def mode(self) -> int:
        return {"none": 0, "diagonal": 1, "dense": 2}[self.adaptation.lower()]


@dataclass
class MassMatrix:
    """The per-chain metric: kind [C] (0 identity, 1 diagonal, 2 dense), the
    diagonal inverse / sqrt [C, dim], the dense inverse / Cholesky factor
    [C, dim, dim] (None unless dense adaptation is on)."""
    kind: np.ndarray
    diag_inv: np.ndarray
    diag_sqrt: np.ndarray
    dense_inv: np.ndarray | None
    dense_chol: np.ndarray | None


class NUTS(Sampler):
    _progress_prefix = "Global"
    _progress_interval = 1.0  # seconds between progress reports

    def __init__(self, target, initial_positions, target_accept_p: float, dtype=None,
                 max_depth: int = 0, chain_offset: int = 0):
        self.target_accept_p = float(target_accept_p)
        super().__init__(lambda lib: lib.gm_nuts_create, target, initial_positions, dtype,
                         chain_offset, self.target_accept_p, int(max_depth))

    @classmethod
    def new_with_mass_matrix(cls, target, initial_positions, target_accept_p: float,
                             mass_config: NUTSMassMatrixConfig, **kw) -> "NUTS":
        """GenericNUTS::new_with_mass_matrix (generic_nuts.rs:379-398)."""
        s = cls(target, initial_positions, target_accept_p, **kw)
        s.set_mass_adaptation(mass_config)
        return s

    def set_mass_adaptation(self, cfg: NUTSMassMatrixConfig) -> "NUTS":
        _lib.check(self._lib.gm_nuts_set_mass_adaptation(
            self._h, cfg.mode, cfg.start_buffer, cfg.end_buffer, cfg.initial_window, cfg.regularize,
            cfg.jitter, cfg.dense_max_dim))
        return self

    def mass_matrix(self) -> MassMatrix:
        mode = C.c_int32()
        kind = np.zeros(self.n_chains, dtype=np.int32)
        _lib.check(self._lib.gm_nuts_get_mass(self._h, C.byref(mode), _lib.ptr(kind), None, None, None, None))
        d = (self.n_chains, self.dim)
        dinv, dsq = np.zeros(d, dtype=self.dtype), np.zeros(d, dtype=self.dtype)
        minv = mchol = None
        if mode.value == 2:
            minv = np.zeros(d + (self.dim,), dtype=self.dtype)
            mchol = np.zeros(d + (self.dim,), dtype=self.dtype)
        if mode.value:
            _lib.check(self._lib.gm_nuts_get_mass(self._h, None, None, _lib.ptr(dinv), _lib.ptr(dsq),
                                                  None if minv is None else _lib.ptr(minv),
                                                  None if mchol is None else _lib.ptr(mchol)))
        return MassMatrix(kind, dinv, dsq, minv, mchol)

    def set_seed(self, seed: int) -> "NUTS":
        """nuts.rs:299-304 / generic_nuts.rs:550-556."""
        return self._seed(seed)

    def set_lds_levels(self, levels: int):
        """Subtree-stack levels kept in LDS (-1: as many as fit); the rest in
        HBM. Identical results either way."""
        _lib.check(self._lib.gm_nuts_set_lds_levels(self._h, int(levels)))
        return self

    def set_dense_forms(self, minv_lds: int = -1, chol_lds: int = -1):
        """Placement of the dense metric's matrices (gm_nuts_set_dense_forms):
        minv_lds -1 automatic (= 1), 1 the packed triangle in LDS, 2 the full
        matrix when it fits (else packed), 0 global memory; chol_lds -1
        automatic (= 0), 1 the packed Cholesky factor in LDS too. Identical
        results."""
        _lib.check(self._lib.gm_nuts_set_dense_forms(self._h, int(minv_lds), int(chol_lds)))
        return self

    def set_momentum_pass(self, on: bool = True):
        """Draw the transition momenta in one parallel pass per launch (the
        default) or inside the tree kernel; identical results."""
        _lib.check(self._lib.gm_nuts_set_momentum_pass(self._h, 1 if on else 0))
        return self

    def launch_plan(self) -> dict:
        """The last launch's on-chip plan (gm_nuts_get_plan)."""
        p = np.zeros(6, dtype=np.int32)
        _lib.check(self._lib.gm_nuts_get_plan(self._h, _lib.ptr(p), len(p)))
        return {"lds_levels": int(p[0]), "minv_lds": int(p[1]), "minv_off": int(p[2]), "chol_lds": int(p[3]),
                "chol_off": int(p[4]), "frozen": int(p[5])}

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
