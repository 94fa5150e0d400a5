"""Built-in targets and the isotropic-Gaussian proposal.

Mirrors the reference's distributions module (distributions.rs): the same
names and parameters, but each target is a descriptor of a device-side
log-density with an analytic gradient (no autodiff graph, hmc.rs:42-61).

    RosenbrockND          distributions.rs:535-555   (a=1, b=100, any dim)
    Rosenbrock2D(a, b)    distributions.rs:495-530
    IsotropicGaussian(s)  distributions.rs:349-406   (target and MH proposal)
    DiffableGaussian2D    distributions.rs:215-320
    DenseGaussian         DiffableGaussian2D generalised to dim D
    Gaussian2D            distributions.rs:161-208   (Target, no norm const)
    CustomTarget          a user target (the Target / GradientTarget traits,
                          distributions.rs:67-110) as HIP source, compiled at
                          run time into the sampler kernels
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib


class _TargetBase:
    """A device-evaluated target. `dim` is None when the target adapts to the
    sampler's dimension (RosenbrockND, IsotropicGaussian)."""

    dim: int | None = None

    def _fill(self, t: _lib.gm_target, dim: int) -> list:
        raise NotImplementedError

    def to_struct(self, dim: int):
        if self.dim is not None and self.dim != dim:
            # the reference panics here (distributions.rs:267, 302)
            raise ValueError(f"{type(self).__name__}: expected dimension={self.dim}, got {dim}")
        t = _lib.gm_target()
        t.dim = dim
        keep = self._fill(t, dim)
        return t, keep

    # BatchedGradientTarget::unnorm_logp_batch (distributions.rs:67-78), plus the
    # gradient the reference gets from autodiff (hmc.rs:42-61).
    def unnorm_logp_and_grad_batch(self, positions, dtype=None):
        x = np.asarray(positions)
        if dtype is None:
            dtype = x.dtype if x.dtype in (np.float32, np.float64) else np.float64
        x = np.ascontiguousarray(x, dtype=dtype)
        if x.ndim == 1:
            x = x[None, :]
        n, dim = x.shape
        t, keep = self.to_struct(dim)
        lp = np.empty(n, dtype=dtype)
        g = np.empty((n, dim), dtype=dtype)
        lib = _lib.require_gpu()
        _lib.check(lib.gm_target_logp_grad(C.byref(t), _lib.dtype_code(dtype), n, _lib.ptr(x),
                                           _lib.ptr(lp), _lib.ptr(g)))
        del keep
        return lp, g

    def unnorm_logp_batch(self, positions, dtype=None):
        return self.unnorm_logp_and_grad_batch(positions, dtype)[0]

    # GradientTarget::unnorm_logp / unnorm_logp_and_grad (distributions.rs:80-90)
    def unnorm_logp_and_grad(self, position, dtype=None):
        lp, g = self.unnorm_logp_and_grad_batch(np.asarray(position)[None, :], dtype)
        return lp[0], g[0]

    # Target::unnorm_logp (distributions.rs:107-110)
    def unnorm_logp(self, position, dtype=None):
        return self.unnorm_logp_and_grad(position, dtype)[0]


class RosenbrockND(_TargetBase):
    """-sum_{i<D-1} [100 (x_{i+1} - x_i^2)^2 + (1 - x_i)^2]."""

    a = 1.0
    b = 100.0

    def _fill(self, t, dim):
        t.kind = _lib.GM_TARGET_ROSENBROCK
        t.a, t.b = 1.0, 100.0
        return []


class Rosenbrock2D(_TargetBase):
    def __init__(self, a: float = 1.0, b: float = 100.0):
        self.a = float(a)
        self.b = float(b)
        self.dim = 2

    def _fill(self, t, dim):
        t.kind = _lib.GM_TARGET_ROSENBROCK
        t.a, t.b = self.a, self.b
        return []


class IsotropicGaussian(_TargetBase):
    """Zero-mean isotropic Gaussian N(0, std^2 I): a target (any dim) and the
    random-walk proposal of Metropolis-Hastings (x' = x + std * N(0, I))."""

    def __init__(self, std: float = 1.0):
        self.std = float(std)

    def _fill(self, t, dim):
        t.kind = _lib.GM_TARGET_ISO_GAUSS
        t.std = self.std
        return []

    # Proposal::logp (distributions.rs:378-390), including the reference's
    # constant -d/2 ln(var * pi * std^2); host-side helper for tests/diagnostics.
    def proposal_logp(self, frm, to) -> float:
        frm = np.asarray(frm, dtype=np.float64)
        to = np.asarray(to, dtype=np.float64)
        var = self.std * self.std
        lp = float(np.sum(-((to - frm) ** 2) / (2 * var)))
        return lp + -len(frm) * 0.5 * math.log(var * math.pi * self.std * self.std)


class _GaussBase(_TargetBase):
    def __init__(self, mean, cov, norm_const: float | None):
        self.mean = np.ascontiguousarray(np.asarray(mean, dtype=np.float64))
        self.cov = np.ascontiguousarray(np.asarray(cov, dtype=np.float64))
        d = self.mean.shape[0]
        if self.cov.shape != (d, d):
            raise ValueError("cov must be [dim, dim]")
        self.dim = d
        self.inv_cov = np.empty((d, d), dtype=np.float64)
        nc = C.c_double(0.0)
        lib = _lib.load()
        _lib.check(lib.gm_gauss_from_cov(d, _lib.ptr(self.cov), _lib.ptr(self.inv_cov), C.byref(nc)))
        self.log_norm_const = nc.value
        self.norm_const = nc.value if norm_const is None else norm_const

    def _fill(self, t, dim):
        t.kind = _lib.GM_TARGET_GAUSS
        t.mean = self.mean.ctypes.data_as(C.POINTER(C.c_double))
        t.prec = self.inv_cov.ctypes.data_as(C.POINTER(C.c_double))
        t.norm_const = self.norm_const
        return [self.mean, self.inv_cov]


class DiffableGaussian2D(_GaussBase):
    """distributions.rs:215-320: logp includes -(2 ln 2pi + ln|Sigma|)/2."""

    def __init__(self, mean, cov):
        super().__init__(mean, cov, None)
        if self.dim != 2:
            raise ValueError("Gaussian2D: expected dimension=2.")


class DenseGaussian(_GaussBase):
    """Full-covariance Gaussian in D dims (config 3's target)."""

    def __init__(self, mean, cov):
        super().__init__(mean, cov, None)


class Gaussian2D(_GaussBase):
    """distributions.rs:161-208. As a Target: -0.5 d^T Sigma^-1 d (no constant);
    `logp` (Normalized) adds -ln(2 pi) - 0.5 ln|det Sigma|."""

    def __init__(self, mean, cov):
        super().__init__(mean, cov, 0.0)
        if self.dim != 2:
            raise ValueError("Gaussian2D: expected dimension=2.")

    def logp(self, position) -> float:
        c = self.cov
        det = c[0, 0] * c[1, 1] - c[0, 1] * c[1, 0]
        return float(self.unnorm_logp(np.asarray(position, dtype=np.float64))) + (
            -math.log(2.0 * math.pi) - 0.5 * math.log(abs(det)))


class CustomTarget(_TargetBase):
    """A user-defined target, the counterpart of implementing the reference's
    GradientTarget / BatchedGradientTarget traits (distributions.rs:67-110).

    `source` is HIP C++ defining, for T = float and double,

        template <class T>
        __device__ T gm_logp_grad(const T* x, T* g, const T* params);

    which receives one chain's position x[GM_DIM] (GM_DIM is a macro equal to
    `dim`), writes the gradient of the unnormalised log-density to g[GM_DIM]
    and returns the log-density. `params` are copied to the device in the
    sampler's dtype. The source is compiled at run time (hiprtc) together
    with the engine's own HMC / MH / NUTS kernels, one chain per lane
    (layout 1 x dim, dim <= 256); a compile error raises at sampler creation
    with the compiler log. The gradient is the user's: there is no autodiff
    on the device."""

    def __init__(self, source: str, dim: int, params=()):
        self.source = str(source)
        self.dim = int(dim)
        self.params = np.ascontiguousarray(np.asarray(params, dtype=np.float64).reshape(-1))

    def _fill(self, t, dim):
        t.kind = _lib.GM_TARGET_CUSTOM
        src = self.source.encode()
        t.source = src
        t.params = self.params.ctypes.data_as(C.POINTER(C.c_double))
        t.n_params = self.params.size
        return [src, self.params]

    _KINDS = {"logp": 0, "hmc": 1, "mh": 2, "nuts": 3}

    def check(self, sampler: str = "hmc", dtype=np.float64) -> None:
        """Compile the source into `sampler`'s kernel ("hmc", "mh", "nuts" or
        "logp") without running it; raises GMError with the compiler log."""
        lib = _lib.load()
        _lib.check(lib.gm_custom_target_check(self.source.encode(), _lib.dtype_code(dtype), self.dim,
                                              self._KINDS[sampler]))
