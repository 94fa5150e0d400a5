"""Granular BatchVector operations on device matrices (tier 2 of the boundary).

The reference makes its batched HMC generic over the `BatchVector` trait
(euclidean.rs:145-195), implemented for `Tensor<B, 2>` of shape
[n_chains, dim] (euclidean.rs:358-534), and over
`BatchedHamiltonianTarget::logp_and_grad` (batched_hmc.rs:18-22). This module
exposes the same operations on device buffers held by libgmcmc
(`gm_bv_*` in include/gmcmc.h), and `BatchedGenericHMC` drives them in the
reference's step order (batched_hmc.rs:129-190).

The fused sampler (`HMC`) is the performance path. This op-by-op path is
for callers that plug their own step logic into the seam. A step composed here
reads the same Philox streams and reduces in the same order as the fused
kernel; its kicks and drift are the reference's `add_scaled_assign` (product
and sum rounded separately, euclidean.rs:392-394), where the fused kernel uses
fused multiply-adds, so the two agree to rounding and each matches its own
form of the oracle bit for bit. With `fused_leapfrog=True` the leapfrog is
one `gm_bv_leapfrog` kernel in the fused kernel's form (its bits).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


class DeviceMatrix:
    """A device buffer of shape (n_chains, dim), or (n_chains,) for energies
    and masks. Owned: freed on close() / garbage collection."""

    def __init__(self, shape, dtype):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self.lib = _lib.require_gpu()
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = C.c_void_p()
        _lib.check(self.lib.gm_malloc(C.byref(p), self.nbytes))
        self.ptr = p.value or 0

    @classmethod
    def from_host(cls, arr) -> "DeviceMatrix":
        a = np.ascontiguousarray(arr)
        m = cls(a.shape, a.dtype)
        _lib.check(m.lib.gm_memcpy_htod(C.c_void_p(m.ptr), _lib.ptr(a), m.nbytes))
        return m

    @classmethod
    def like(cls, other: "DeviceMatrix", dtype=None) -> "DeviceMatrix":
        return cls(other.shape, dtype or other.dtype)

    def to_host(self) -> np.ndarray:
        out = np.empty(self.shape, dtype=self.dtype)
        _lib.check(self.lib.gm_memcpy_dtoh(_lib.ptr(out), C.c_void_p(self.ptr), self.nbytes))
        return out

    def assign(self, other: "DeviceMatrix") -> None:
        """assign (euclidean.rs:380-382)."""
        _same(self, other)
        _lib.check(self.lib.gm_memcpy_dtod(C.c_void_p(self.ptr), C.c_void_p(other.ptr), self.nbytes))

    @property
    def n_chains(self) -> int:
        return self.shape[0]

    @property
    def dim(self) -> int:
        return self.shape[1] if len(self.shape) > 1 else 1

    @property
    def code(self) -> int:
        return _lib.dtype_code(self.dtype)

    def close(self) -> None:
        if getattr(self, "ptr", 0):
            self.lib.gm_free(C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _same(a: DeviceMatrix, b: DeviceMatrix) -> None:
    if a.shape != b.shape or a.dtype != b.dtype:
        raise ValueError(f"shape/dtype mismatch: {a.shape} {a.dtype} vs {b.shape} {b.dtype}")


def _vp(m: DeviceMatrix | None):
    return C.c_void_p(m.ptr if m is not None else 0)


# ---- BatchVector ops (euclidean.rs:447-534) --------------------------------

def kinetic_energy(p: DeviceMatrix, out: DeviceMatrix | None = None) -> DeviceMatrix:
    """0.5 * sum_j p[c, j]^2 per chain -> [n_chains] (euclidean.rs:464-472)."""
    out = out or DeviceMatrix((p.n_chains,), p.dtype)
    _lib.check(p.lib.gm_bv_kinetic_energy(p.code, p.n_chains, p.dim, _vp(p), _vp(out)))
    return out


def masked_assign(x: DeviceMatrix, other: DeviceMatrix, mask: DeviceMatrix) -> None:
    """x[c, :] = other[c, :] where mask[c] (euclidean.rs:474-482)."""
    _same(x, other)
    if mask.dtype != np.uint8 or mask.shape != (x.n_chains,):
        raise ValueError("mask must be uint8 [n_chains]")
    _lib.check(x.lib.gm_bv_masked_assign(x.code, x.n_chains, x.dim, _vp(x), _vp(other), _vp(mask)))


def add_scaled_assign(x: DeviceMatrix, other: DeviceMatrix, alpha: float) -> None:
    """x = x + other * alpha (euclidean.rs:392-394)."""
    _same(x, other)
    n = int(np.prod(x.shape))
    _lib.check(x.lib.gm_bv_add_scaled_assign(x.code, n, _vp(x), _vp(other), float(alpha)))


def scale_assign(x: DeviceMatrix, alpha: float) -> None:
    """x = x * alpha (EuclideanVector::scale_assign, euclidean.rs:396-398)."""
    _lib.check(x.lib.gm_bv_scale_assign(x.code, int(np.prod(x.shape)), _vp(x), float(alpha)))


def fill(x: DeviceMatrix, value: float = 0.0) -> None:
    """Every element = value (fill_zero / zeros_like, euclidean.rs:22-26)."""
    _lib.check(x.lib.gm_bv_fill(x.code, int(np.prod(x.shape)), _vp(x), float(value)))


def dot(a: DeviceMatrix, b: DeviceMatrix) -> float:
    """Sum of a*b over every element (EuclideanVector::dot, euclidean.rs:400-403)."""
    _same(a, b)
    out = C.c_double()
    _lib.check(a.lib.gm_bv_dot(a.code, int(np.prod(a.shape)), _vp(a), _vp(b), C.byref(out)))
    return out.value


def fill_random_normal(x: DeviceMatrix, seed: int, step: int, chain_offset: int = 0) -> None:
    """N(0, 1) momentum draws of transition `step` (euclidean.rs:484-496)."""
    _lib.check(x.lib.gm_bv_fill_random_normal(x.code, x.n_chains, x.dim, _vp(x), seed, chain_offset, step))


def sample_uniform(n_chains: int, dtype, seed: int, step: int, chain_offset: int = 0) -> DeviceMatrix:
    """[n_chains] accept uniforms in [0, 1) (euclidean.rs:498-509)."""
    out = DeviceMatrix((n_chains,), dtype)
    _lib.check(out.lib.gm_bv_sample_uniform(out.code, n_chains, _vp(out), seed, chain_offset, step))
    return out


def _energy2(fn: str, a: DeviceMatrix, b: DeviceMatrix) -> DeviceMatrix:
    _same(a, b)
    out = DeviceMatrix.like(a)
    _lib.check(getattr(a.lib, fn)(a.code, a.shape[0], _vp(a), _vp(b), _vp(out)))
    return out


def _energy1(fn: str, a: DeviceMatrix) -> DeviceMatrix:
    out = DeviceMatrix.like(a)
    _lib.check(getattr(a.lib, fn)(a.code, a.shape[0], _vp(a), _vp(out)))
    return out


def energy_sub(a, b):
    return _energy2("gm_bv_energy_sub", a, b)


def energy_add(a, b):
    return _energy2("gm_bv_energy_add", a, b)


def energy_neg(a):
    return _energy1("gm_bv_energy_neg", a)


def energy_ln(a):
    return _energy1("gm_bv_energy_ln", a)


def accept_mask(log_accept: DeviceMatrix, ln_u: DeviceMatrix) -> DeviceMatrix:
    """uint8 [n_chains]: log_accept >= ln_u, NaN -> 0 (euclidean.rs:527-533)."""
    _same(log_accept, ln_u)
    out = DeviceMatrix((log_accept.shape[0],), np.uint8)
    _lib.check(log_accept.lib.gm_bv_accept_mask(log_accept.code, log_accept.shape[0], _vp(log_accept),
                                                 _vp(ln_u), _vp(out)))
    return out


class BatchTarget:
    """A built-in target on the device: logp_and_grad over [n_chains, dim]
    (BatchedHamiltonianTarget, batched_hmc.rs:18-22; hmc.rs:42-61)."""

    def __init__(self, target, dim: int, dtype=np.float32):
        self.lib = _lib.require_gpu()
        self.dtype = np.dtype(dtype)
        self._struct, self._keep = target.to_struct(dim)
        h = C.c_void_p()
        _lib.check(self.lib.gm_bv_target_create(C.byref(self._struct), _lib.dtype_code(self.dtype), C.byref(h)))
        self.h = h

    def logp_and_grad(self, x: DeviceMatrix, grad: DeviceMatrix, logp: DeviceMatrix | None = None) -> DeviceMatrix:
        _same(x, grad)
        logp = logp or DeviceMatrix((x.n_chains,), x.dtype)
        _lib.check(self.lib.gm_bv_logp_and_grad(self.h, x.n_chains, _vp(x), _vp(grad), _vp(logp)))
        return logp

    def leapfrog(self, q: DeviceMatrix, p: DeviceMatrix, grad: DeviceMatrix, logp: DeviceMatrix | None,
                 step_size) -> None:
        """One leapfrog in place, state in device memory (gm_bv_leapfrog: the
        loop body of batched_hmc.rs:166-190 as one kernel)."""
        _same(q, p)
        _same(q, grad)
        _lib.check(self.lib.gm_bv_leapfrog(self.h, q.n_chains, _vp(q), _vp(p), _vp(grad),
                                           _vp(logp), float(step_size)))

    def close(self):
        if getattr(self, "h", None) is not None:
            self.lib.gm_bv_target_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BatchedGenericHMC:
    """BatchedGenericHMC (batched_hmc.rs:25-190) driven through the
    granular ops: one transition = the nine stages of `step`
    (batched_hmc.rs:129-163) with the leapfrog of 166-190."""

    def __init__(self, target, initial_positions, step_size: float, n_leapfrog: int, seed: int = 0,
                 chain_offset: int = 0, fused_leapfrog: bool = False):
        x0 = np.ascontiguousarray(initial_positions)
        self.dtype = x0.dtype
        self.n_chains, self.dim = x0.shape
        self.target = BatchTarget(target, self.dim, self.dtype)
        self.position = DeviceMatrix.from_host(x0)
        self.momentum = DeviceMatrix.like(self.position)
        self.grad = DeviceMatrix.like(self.position)
        self.proposal_pos = DeviceMatrix.like(self.position)
        self.proposal_mom = DeviceMatrix.like(self.position)
        self.step_size = self.dtype.type(step_size)
        self.n_leapfrog = int(n_leapfrog)
        self.seed = int(seed)
        self.chain_offset = int(chain_offset)
        self.t = 0  # transition index (keys the random streams)
        # one gm_bv_leapfrog kernel per leapfrog instead of four ops (the fused
        # kernel's fused multiply-add kicks and drift: its bits)
        self.fused_leapfrog = bool(fused_leapfrog)

    def set_seed(self, seed: int) -> "BatchedGenericHMC":
        self.seed, self.t = int(seed), 0
        return self

    def _leapfrog(self) -> DeviceMatrix:
        half = self.dtype.type(0.5) * self.step_size
        logp = self.target.logp_and_grad(self.proposal_pos, self.grad)
        if self.fused_leapfrog:
            for _ in range(self.n_leapfrog):
                self.target.leapfrog(self.proposal_pos, self.proposal_mom, self.grad, logp, self.step_size)
            return logp
        for _ in range(self.n_leapfrog):
            add_scaled_assign(self.proposal_mom, self.grad, half)
            add_scaled_assign(self.proposal_pos, self.proposal_mom, self.step_size)
            logp = self.target.logp_and_grad(self.proposal_pos, self.grad, logp)
            add_scaled_assign(self.proposal_mom, self.grad, half)
        return logp

    def step(self) -> None:
        fill_random_normal(self.momentum, self.seed, self.t, self.chain_offset)      # 1
        ke_current = kinetic_energy(self.momentum)                                   # 2
        logp_current = self.target.logp_and_grad(self.position, self.grad)           # 3
        self.proposal_pos.assign(self.position)                                      # 4
        self.proposal_mom.assign(self.momentum)
        logp_proposed = self._leapfrog()                                             # 5
        ke_proposed = kinetic_energy(self.proposal_mom)                              # 6
        log_accept = energy_add(energy_sub(logp_proposed, logp_current),             # 7
                                energy_sub(ke_current, ke_proposed))
        u = sample_uniform(self.n_chains, self.dtype, self.seed, self.t, self.chain_offset)  # 8
        mask = accept_mask(log_accept, energy_ln(u))                                 # 9
        masked_assign(self.position, self.proposal_pos, mask)
        self.t += 1

    def run(self, n_collect: int, n_discard: int) -> np.ndarray:
        """[n_chains, n_collect, dim] (hmc.rs:164-181)."""
        for _ in range(n_discard):
            self.step()
        out = np.empty((self.n_chains, n_collect, self.dim), dtype=self.dtype)
        for k in range(n_collect):
            self.step()
            out[:, k, :] = self.position.to_host()
        return out

    def positions(self) -> np.ndarray:
        return self.position.to_host()
