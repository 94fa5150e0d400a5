"""ctypes wrapper of the CPU oracle (oracle/liboracle.so) -- test
infrastructure only: the checker the GPU results are compared with."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")

_vp, _i64, _i32, _u64, _u32, _dbl, _flt, _int = (C.c_void_p, C.c_int64, C.c_int32, C.c_uint64,
                                                   C.c_uint32, C.c_double, C.c_float, C.c_int)


class or_target(C.Structure):
    _fields_ = [("kind", C.c_int32), ("dim", C.c_int32), ("a", C.c_double), ("b", C.c_double),
                ("std", C.c_double), ("mean", C.POINTER(C.c_double)),
                ("prec", C.POINTER(C.c_double)), ("norm_const", C.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def load():
    global _lib
    if _lib is not None:
        return Oracle(_lib)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
            os.path.getmtime(os.path.join(ORACLE_DIR, f))
            for f in ("gm_oracle.c", "gm_oracle_t.inc", "gm_oracle.h")):
        build()
    lib = C.CDLL(LIB)
    tp = C.POINTER(or_target)
    for sfx, rt in (("d", _dbl), ("f", _flt)):
        getattr(lib, f"or_log_{sfx}").restype = rt
        getattr(lib, f"or_log_{sfx}").argtypes = [rt]
        getattr(lib, f"or_exp_{sfx}").restype = rt
        getattr(lib, f"or_exp_{sfx}").argtypes = [rt]
        getattr(lib, f"or_cos2pi_{sfx}").restype = rt
        getattr(lib, f"or_cos2pi_{sfx}").argtypes = [rt]
        getattr(lib, f"or_normal_{sfx}").restype = rt
        getattr(lib, f"or_normal_{sfx}").argtypes = [_u64, _u32, _u64, _u32, _u32]
        getattr(lib, f"or_mom_normal_{sfx}").restype = rt
        getattr(lib, f"or_mom_normal_{sfx}").argtypes = [_u64, _u32, _u64, _u32, _u32]
        if sfx == "d":
            lib.or_leaf_alpha_d.restype = rt
            lib.or_leaf_alpha_d.argtypes = [rt]
            lib.or_tab_normal_d.restype = rt
            lib.or_tab_normal_d.argtypes = [_u64, _u32, _u64, _u32, _u32]
            lib.or_tab_normal_pair.restype = None
            lib.or_tab_normal_pair.argtypes = [_vp, _vp]
        else:
            lib.or_tab_normal_pair_f.restype = None
            lib.or_tab_normal_pair_f.argtypes = [_u32, _u32, _vp]
        getattr(lib, f"or_uniform_co_{sfx}").restype = rt
        getattr(lib, f"or_uniform_co_{sfx}").argtypes = [_u64, _u32, _u64, _u32, _u32]
        getattr(lib, f"or_logp_grad_{sfx}").restype = rt
        getattr(lib, f"or_logp_grad_{sfx}").argtypes = [tp, _int, _int, _vp, _vp]
        getattr(lib, f"or_hmc_run_{sfx}").argtypes = [tp, _int, _int, _i64, _int, _vp, _dbl, _int,
                                                      _u64, _u64, _u32, _i64, _i64, _vp, _vp, _int, _int]
        getattr(lib, f"or_mh_run_{sfx}").argtypes = [tp, _int, _int, _i64, _int, _vp, _dbl, _u64,
                                                     _u64, _u32, _i64, _i64, _vp, _vp, _int, _int]
        getattr(lib, f"or_mh_terms_{sfx}").argtypes = [tp, _int, _int, _i64, _int, _vp, _dbl, _u64, _u64,
                                                       _u32, _int, _vp, _vp, _vp, _int]
        getattr(lib, f"or_nuts_run_{sfx}").argtypes = [tp, _int, _int, _i64, _int, _vp, _vp, _vp,
                                                       _vp, _vp, _dbl, _int, _u64, _u64, _u32,
                                                       _i64, _i64, _int, _vp, _vp, _vp, _int]
        getattr(lib, f"or_nuts_step_{sfx}").argtypes = [tp, _int, _int, _i64, _int, _vp, _vp, _vp,
                                                        _vp, _vp, _dbl, _int, _u64, _u64, _u32,
                                                        _i64, _i64, _i64, _vp, _vp, _int]
    for sfx in ("d", "f"):
        getattr(lib, f"or_nuts_mass_run_{sfx}").argtypes = [
            tp, _int, _int, _i64, _int, _vp, _vp, _vp, _vp, _vp, _dbl, _int, _u64, _u64, _u32, _i64,
            _i64, _int, _vp, _vp, _vp, C.POINTER(or_mass_cfg), C.POINTER(or_mass_state), _int]
    for sfx in ("d", "f"):
        getattr(lib, f"or_dense_traj_{sfx}").argtypes = [tp, _int, _int, _int, _vp, _vp, _vp, _dbl, _int,
                                                         _int, _vp, _vp]
    lib.or_mass_state_init.argtypes = [C.POINTER(or_mass_cfg), _i64, _int, _int, C.POINTER(or_mass_state)]
    lib.or_mass_diag_kat.argtypes = [_vp, _int, _dbl, _vp, _vp, _vp]
    lib.or_mass_dense_kat.argtypes = [_vp, _int, _dbl, _vp, _vp]
    lib.or_mass_warmup_diag_kat.argtypes = [_vp, _int, _int, _dbl, _dbl, _vp, _vp]
    lib.or_philox.argtypes = [C.POINTER(C.c_uint32)] * 3
    lib.or_nuts_key.restype = _u64
    lib.or_nuts_key.argtypes = [_u64, _u32, _u64, C.POINTER(C.c_uint32)]
    lib.or_nuts_u_d.restype = _dbl
    lib.or_nuts_u_d.argtypes = [_u64, _u32]
    lib.or_find_reasonable_epsilon_d.restype = _dbl
    lib.or_find_reasonable_epsilon_d.argtypes = [tp, _int, _int, _vp, _vp]
    lib.or_build_tree_d.argtypes = [tp, _int, _int, _vp, _vp, _vp, _dbl, _int, _int, _dbl, _dbl,
                                    _u64, _u32, _u64, _vp, _vp]
    lib.or_split_rhat_ess.argtypes = [_vp, _i64, _i64, _i64, _vp, _vp]
    lib.or_split_rhat_ess_mt.argtypes = [_vp, _i64, _i64, _i64, _vp, _vp, C.c_int]
    lib.or_autocov_bf.argtypes = [_vp, _i64, _i64, _vp]
    lib.or_autocov_fft.argtypes = [_vp, _i64, _i64, _vp]
    lib.or_mct_rhat.argtypes = [_vp, _i64, _i64, _i64, _vp]
    lib.or_mct_p_accept.restype = _flt
    lib.or_mct_p_accept.argtypes = [_vp, _i64, _i64, _i64]
    lib.or_ct_init.argtypes = [_i64, _i64, _vp, _vp, _vp, _vp, _vp]
    lib.or_ct_step.argtypes = [_i64, _i64, _u64, _vp, _vp, _vp, _vp, _vp]
    lib.or_collect_rhat.argtypes = [_i64, _i64, _u64, _vp, _vp, _vp]
    _lib = lib
    return Oracle(lib)


class CpuHmc:
    """oracle/libcpu_hmc.so: bench.py's CPU baseline (the reference's batched
    HMC op structure at -O3; not bit-matching -- see cpu_hmc.c)."""

    def __init__(self, lib):
        self.lib = lib
        lib.cpu_hmc_rosenbrock_f32.argtypes = [_vp, _i64, _int, _dbl, _int, _i64, _u64, _int, _vp]

    def run(self, q, eps, L, n_steps, seed, threads, accepts=None):
        assert q.dtype == np.float32 and q.flags["C_CONTIGUOUS"]
        rc = self.lib.cpu_hmc_rosenbrock_f32(_p(q), q.shape[0], q.shape[1], eps, L, n_steps, seed, threads,
                                             _p(accepts))
        assert rc == 0


def cpu_hmc():
    """The CPU-baseline library, or None if it is not built."""
    path = os.path.join(ORACLE_DIR, "libcpu_hmc.so")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(os.path.join(ORACLE_DIR, "cpu_hmc.c")):
        try:
            build()
        except Exception:
            return None
    if not os.path.exists(path):
        return None
    return CpuHmc(C.CDLL(path))


class or_mass_cfg(C.Structure):
    _fields_ = [("mode", C.c_int), ("start_buffer", C.c_int64), ("end_buffer", C.c_int64),
                ("initial_window", C.c_int64), ("regularize", C.c_double), ("jitter", C.c_double),
                ("form", C.c_int)]


class or_mass_state(C.Structure):
    _fields_ = [("kind", C.c_void_p), ("dinv", C.c_void_p), ("dsqrt", C.c_void_p),
                ("minv", C.c_void_p), ("mchol", C.c_void_p), ("sched", C.c_int64 * 2)]


class NutsMass:
    """Host arrays of the oracle's per-chain mass state (or_mass_state)."""

    def __init__(self, lib, mode, C_, D, dtype, start_buffer=75, end_buffer=50, initial_window=25,
                 regularize=0.05, jitter=1e-6, form=0):
        # form 0: the engine's arithmetic (the kernels' bits); 1: the
        # reference's op structure (fresh M^-1 products, two roundings)
        self.cfg = or_mass_cfg(mode, start_buffer, end_buffer, initial_window, regularize, jitter, form)
        self.kind = np.zeros(C_, dtype=np.int32)
        self.dinv = np.zeros((C_, D), dtype=dtype)
        self.dsqrt = np.zeros((C_, D), dtype=dtype)
        nd = D if mode == 2 else 0
        self.minv = np.zeros((C_, nd, nd), dtype=dtype)
        self.mchol = np.zeros((C_, nd, nd), dtype=dtype)
        self.st = or_mass_state(_p(self.kind).value, _p(self.dinv).value, _p(self.dsqrt).value,
                                _p(self.minv).value if nd else None, _p(self.mchol).value if nd else None)
        lib.or_mass_state_init(C.byref(self.cfg), C_, D, int(np.dtype(dtype) == np.float64),
                               C.byref(self.st))


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _sfx(dtype):
    return "d" if np.dtype(dtype) == np.float64 else "f"


class Target:
    """Oracle-side description of a built-in target (mirrors gm_target)."""

    def __init__(self, kind, dim, a=1.0, b=100.0, std=1.0, mean=None, prec=None, norm_const=0.0):
        self.kind, self.dim, self.a, self.b, self.std = kind, dim, a, b, std
        self.mean = None if mean is None else np.ascontiguousarray(mean, dtype=np.float64)
        self.prec = None if prec is None else np.ascontiguousarray(prec, dtype=np.float64)
        self.norm_const = norm_const

    @classmethod
    def from_product(cls, t, dim):
        """Same parameters as a general_mcmc_amd target."""
        st, _ = t.to_struct(dim)
        mean = prec = None
        if st.kind == 3:
            mean = np.asarray(t.mean, dtype=np.float64)
            prec = np.asarray(t.inv_cov, dtype=np.float64)
        return cls(st.kind, dim, st.a, st.b, st.std, mean, prec, st.norm_const)

    def struct(self):
        t = or_target()
        t.kind, t.dim, t.a, t.b, t.std, t.norm_const = (self.kind, self.dim, self.a, self.b,
                                                         self.std, self.norm_const)
        if self.mean is not None:
            t.mean = self.mean.ctypes.data_as(C.POINTER(C.c_double))
            t.prec = self.prec.ctypes.data_as(C.POINTER(C.c_double))
        return t


class Oracle:
    def __init__(self, lib):
        self.lib = lib

    def philox(self, ctr, key):
        a = (C.c_uint32 * 4)(*ctr)
        k = (C.c_uint32 * 2)(*key)
        o = (C.c_uint32 * 4)()
        self.lib.or_philox(a, k, o)
        return list(o)

    def nuts_key(self, seed, chain, st):
        """The NUTS transition's stream key and its Philox words (spec v3)."""
        w = (C.c_uint32 * 4)()
        k = self.lib.or_nuts_key(seed, chain, st, w)
        return k, list(w)

    def logp_grad(self, target: Target, x, lanes, elems, dtype):
        x = np.ascontiguousarray(np.atleast_2d(x), dtype=dtype)
        n, d = x.shape
        lp = np.empty(n, dtype=dtype)
        g = np.zeros((n, lanes * elems), dtype=dtype)
        t = target.struct()
        fn = getattr(self.lib, f"or_logp_grad_{_sfx(dtype)}")
        for i in range(n):
            lp[i] = fn(C.byref(t), lanes, elems, _p(x[i]), g[i].ctypes.data_as(C.c_void_p))
        return lp, np.ascontiguousarray(g[:, :d])

    def hmc_run(self, target: Target, q, eps, L, seed, step0, n_steps, collect_from, lanes, elems,
                chain_offset=0, threads=8, form=0):
        """form 0: the engine's leapfrog (fused multiply-add kicks and drift,
        the kernels); 1: the reference's op structure (the composed tier-2
        ops)."""
        q = np.array(q, copy=True, order="C")
        C_, D = q.shape
        rows = max(0, n_steps - collect_from)
        samples = np.zeros((rows, C_, D), dtype=q.dtype)
        acc = np.zeros(C_, dtype=np.int64)
        t = target.struct()
        rc = getattr(self.lib, f"or_hmc_run_{_sfx(q.dtype)}")(
            C.byref(t), lanes, elems, C_, D, _p(q), eps, L, seed, step0, chain_offset, n_steps,
            collect_from, _p(samples), _p(acc), threads, form)
        assert rc == 0
        return q, samples, acc

    def mh_run(self, target: Target, q, prop_std, seed, step0, n_steps, collect_from, lanes, elems,
               chain_offset=0, threads=8, form=0):
        """form 0: the kernels' arithmetic; 1: the reference's op structure
        (left-to-right proposal and IsotropicGaussian sums, log q forward and
        backward separately, metropolis_hastings.rs:306-318)."""
        q = np.array(q, copy=True, order="C")
        C_, D = q.shape
        rows = max(0, n_steps - collect_from)
        samples = np.zeros((rows, C_, D), dtype=q.dtype)
        acc = np.zeros(C_, dtype=np.int64)
        t = target.struct()
        rc = getattr(self.lib, f"or_mh_run_{_sfx(q.dtype)}")(
            C.byref(t), lanes, elems, C_, D, _p(q), prop_std, seed, step0, chain_offset, n_steps,
            collect_from, _p(samples), _p(acc), threads, form)
        assert rc == 0
        return q, samples, acc

    def mh_terms(self, target: Target, x, prop_std, seed, st, lanes, elems, form, chain_offset=0, threads=8):
        """One MH step's (log alpha, proposal log-density, ln u) per chain from
        the states x [C, D] at counter step st, in the given form."""
        x = np.ascontiguousarray(x)
        C_, D = x.shape
        la, lp1, lnu = (np.empty(C_, dtype=x.dtype) for _ in range(3))
        t = target.struct()
        rc = getattr(self.lib, f"or_mh_terms_{_sfx(x.dtype)}")(
            C.byref(t), lanes, elems, C_, D, _p(x), prop_std, seed, st, chain_offset, form, _p(la), _p(lp1),
            _p(lnu), threads)
        assert rc == 0
        return la, lp1, lnu

    def nuts_state(self, n, dtype):
        return {"eps": np.full(n, -1.0, dtype=dtype), "eps_bar": np.ones(n, dtype=dtype),
                "h_bar": np.zeros(n, dtype=dtype),
                "mu": np.full(n, np.log(10.0), dtype=dtype)}

    def nuts_run(self, target: Target, q, state, target_accept, max_depth, seed, init_step,
                 n_collect, n_discard, progress, lanes, elems, chain_offset=0, threads=8, form=0):
        """form 0: the kernels' arithmetic; 1: the reference's op structure
        under the identity metric (left-to-right kinetic sum and U-turn dots,
        generic_nuts.rs:230-235, 1369-1377): or_nuts_mass_run with mode 0."""
        if form:
            m = self.nuts_mass(0, np.asarray(q).shape[0], np.asarray(q).shape[1], np.asarray(q).dtype, form=form)
            return self.nuts_mass_run(target, q, state, m, target_accept, max_depth, seed, init_step, n_collect,
                                      n_discard, progress, lanes, elems, chain_offset, threads)
        q = np.array(q, copy=True, order="C")
        C_, D = q.shape
        samples = np.zeros((n_collect, C_, D), dtype=q.dtype)
        acc = np.zeros(C_, dtype=np.int64)
        nlf = np.zeros(C_, dtype=np.int64)
        t = target.struct()
        rc = getattr(self.lib, f"or_nuts_run_{_sfx(q.dtype)}")(
            C.byref(t), lanes, elems, C_, D, _p(q), _p(state["eps"]), _p(state["eps_bar"]),
            _p(state["h_bar"]), _p(state["mu"]), target_accept, max_depth, seed, init_step,
            chain_offset, n_collect, n_discard, int(progress), _p(samples), _p(acc), _p(nlf),
            threads)
        assert rc == 0
        return q, samples, acc, nlf

    def nuts_step(self, target: Target, q, state, target_accept, max_depth, seed, step0, n_steps,
                  m0, n_discard, lanes, elems, chain_offset=0, threads=8):
        """NUTS::step n_steps times (no init_chain_state, nothing collected)."""
        q = np.array(q, copy=True, order="C")
        C_, D = q.shape
        acc = np.zeros(C_, dtype=np.int64)
        nlf = np.zeros(C_, dtype=np.int64)
        t = target.struct()
        rc = getattr(self.lib, f"or_nuts_step_{_sfx(q.dtype)}")(
            C.byref(t), lanes, elems, C_, D, _p(q), _p(state["eps"]), _p(state["eps_bar"]),
            _p(state["h_bar"]), _p(state["mu"]), target_accept, max_depth, seed, step0,
            chain_offset, n_steps, m0, n_discard, _p(acc), _p(nlf), threads)
        assert rc == 0
        return q, acc, nlf

    def split_rhat_ess(self, x, threads: int = 1):
        """split_rhat_mean_ess (stats.rs:439-450) of a [C, N, P] sample (cast
        to f32 first, stats.rs:443); threads > 1 splits the parameters over
        threads (bitwise the same result)."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        c, n, p = x.shape
        r = np.empty(p, dtype=np.float32)
        e = np.empty(p, dtype=np.float32)
        if threads > 1:
            self.lib.or_split_rhat_ess_mt(_p(x), c, n, p, _p(r), _p(e), int(threads))
        else:
            self.lib.or_split_rhat_ess(_p(x), c, n, p, _p(r), _p(e))
        return r, e

    def autocov(self, x, fft=False):
        x = np.ascontiguousarray(x, dtype=np.float32)
        n, d = x.shape
        out = np.empty((n, d), dtype=np.float32)
        (self.lib.or_autocov_fft if fft else self.lib.or_autocov_bf)(_p(x), n, d, _p(out))
        return out

    def mct_rhat(self, steps):
        s = np.ascontiguousarray(steps, dtype=np.float32)
        ns, c, p = s.shape
        r = np.empty(p, dtype=np.float32)
        self.lib.or_mct_rhat(_p(s), ns, c, p, _p(r))
        return r

    def nuts_mass(self, mode, C_, D, dtype, **cfg):
        return NutsMass(self.lib, mode, C_, D, dtype, **cfg)

    def nuts_mass_run(self, target: Target, q, state, mass: NutsMass, target_accept, max_depth, seed,
                      init_step, n_collect, n_discard, progress, lanes, elems, chain_offset=0,
                      threads=8):
        """or_nuts_run with mass-matrix warm-up (GenericNUTS::new_with_mass_matrix)."""
        q = np.array(q, copy=True, order="C")
        C_, D = q.shape
        samples = np.zeros((n_collect, C_, D), dtype=q.dtype)
        acc = np.zeros(C_, dtype=np.int64)
        nlf = np.zeros(C_, dtype=np.int64)
        t = target.struct()
        rc = getattr(self.lib, f"or_nuts_mass_run_{_sfx(q.dtype)}")(
            C.byref(t), lanes, elems, C_, D, _p(q), _p(state["eps"]), _p(state["eps_bar"]),
            _p(state["h_bar"]), _p(state["mu"]), target_accept, max_depth, seed, init_step,
            chain_offset, n_collect, n_discard, int(progress), _p(samples), _p(acc), _p(nlf),
            C.byref(mass.cfg), C.byref(mass.st), threads)
        assert rc == 0
        return q, samples, acc, nlf

    def dense_traj(self, target: Target, inv, q, p, eps, n_leap, form, lanes, elems):
        """n_leap leapfrogs under the dense metric M^-1 = inv from (q, p) in
        the engine's form (0) or the reference's (1): (q, p, M^-1 p, logp,
        kinetic)."""
        dt = np.asarray(q).dtype
        q = np.array(q, dtype=dt, copy=True)
        p = np.array(p, dtype=dt, copy=True)
        inv = np.ascontiguousarray(inv, dtype=dt)
        vel = np.zeros_like(q)
        out = np.zeros(2, dtype=dt)
        t = target.struct()
        rc = getattr(self.lib, f"or_dense_traj_{_sfx(dt)}")(C.byref(t), lanes, elems, q.shape[0], _p(inv), _p(q),
                                                             _p(p), eps, n_leap, form, _p(vel), _p(out))
        assert rc == 0
        return q, p, vel, out[0], out[1]

    def mct_p_accept(self, steps):
        """MultiChainTracker acceptance EMA after stepping [nsteps, C, P]."""
        x = np.ascontiguousarray(steps, dtype=np.float32)
        return self.lib.or_mct_p_accept(_p(x), *x.shape)

    def chain_trackers(self, x0, states):
        """A batch of ChainTrackers: new(x0 [C, P]) then step() with each of
        states [n, C, P]; returns (p_accept [C], mean, msq [C, P])."""
        x0 = np.ascontiguousarray(x0, dtype=np.float32)
        C_, P = x0.shape
        p = np.empty(C_, dtype=np.float32)
        last, mean, msq = (np.empty((C_, P), dtype=np.float32) for _ in range(3))
        self.lib.or_ct_init(C_, P, _p(x0), _p(p), _p(last), _p(mean), _p(msq))
        for k, xs in enumerate(np.ascontiguousarray(states, dtype=np.float32)):
            self.lib.or_ct_step(C_, P, k + 1, _p(np.ascontiguousarray(xs)), _p(p), _p(last), _p(mean),
                                _p(msq))
        return p, mean, msq

    def collect_rhat(self, n, mean, msq):
        mean = np.ascontiguousarray(mean, dtype=np.float32)
        msq = np.ascontiguousarray(msq, dtype=np.float32)
        r = np.empty(mean.shape[1], dtype=np.float32)
        self.lib.or_collect_rhat(mean.shape[0], mean.shape[1], n, _p(mean), _p(msq), _p(r))
        return r

    def find_reasonable_epsilon(self, target: Target, q, p, lanes=64, elems=1):
        t = target.struct()
        q = np.ascontiguousarray(q, dtype=np.float64)
        p = np.ascontiguousarray(p, dtype=np.float64)
        return self.lib.or_find_reasonable_epsilon_d(C.byref(t), lanes, elems, _p(q), _p(p))

    def build_tree(self, target: Target, q, p, g, logu, v, j, eps, joint0, seed=0, chain=0, step=0,
                   lanes=64, elems=1):
        t = target.struct()
        d = target.dim
        vecs = np.zeros((8, d), dtype=np.float64)
        sc = np.zeros(5, dtype=np.float64)
        q, p, g = (np.ascontiguousarray(a, dtype=np.float64) for a in (q, p, g))
        self.lib.or_build_tree_d(C.byref(t), lanes, elems, _p(q), _p(p), _p(g), logu, v, j, eps,
                                 joint0, seed, chain, step, _p(vecs), _p(sc))
        names = ["qm", "pm", "gm", "qp", "pp", "gp", "qprime", "gprime"]
        out = {k: vecs[i] for i, k in enumerate(names)}
        out.update(logp_prime=sc[0], n=int(sc[1]), s=bool(sc[2]), alpha=sc[3], n_alpha=int(sc[4]))
        return out
