"""Common plumbing for the sampler facades: a libgmcmc sampler handle."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .stats import ChainStats, Progress, RunStats, _print_progress, split_rhat_mean_ess_device


@dataclass
class DeviceSamples:
    """Samples left on the GPU by run_positions: [n_collect, n_chains, dim]
    (batched_hmc.rs:115-123). Valid until the sampler's next run or close."""

    ptr: int
    n_collect: int
    n_chains: int
    dim: int
    dtype: type
    owner: "Sampler"
    generation: int = -1

    def _check_live(self):
        # the device buffer belongs to the sampler's LAST run: a later run may
        # have resized (freed) it or overwritten it
        if self.owner._h is None or self.generation != self.owner._gen:
            raise RuntimeError("DeviceSamples are stale: the sampler has run again (or was closed) "
                               "since they were produced")

    def to_host(self) -> np.ndarray:
        self._check_live()
        return self.owner.copy_samples(self.n_collect)

    def block(self, row0: int, n_rows: int, chain0: int, n_chains: int) -> np.ndarray:
        """Rows [row0, row0+n_rows) x chains [chain0, chain0+n_chains) on the
        host, [n_rows, n_chains, dim] (one strided device-to-host copy)."""
        self._check_live()
        out = np.empty((n_rows, n_chains, self.dim), dtype=self.dtype)
        _lib.check(self.owner._lib.gm_copy_sample_block(self.owner._h, row0, n_rows, chain0, n_chains,
                                                        _lib.ptr(out)))
        return out

    def split_rhat_ess(self):
        self._check_live()
        self.owner.synchronize()  # an asynchronous run may still be writing them
        return split_rhat_mean_ess_device(self.ptr, self.dtype, self.n_chains, self.n_collect,
                                          self.dim, (self.dim, self.n_chains * self.dim, 1))


class Sampler:
    _kind = ""

    def __init__(self, create_fn, target, initial_positions, dtype, chain_offset, *extra):
        x = np.asarray(initial_positions)
        if x.ndim != 2:
            raise ValueError("initial_positions must be [n_chains][dim]")
        if dtype is None:
            dtype = np.float64 if x.dtype == np.float64 else np.float32
        self.dtype = np.dtype(dtype).type
        x = np.ascontiguousarray(x, dtype=self.dtype)
        self.n_chains, self.dim = x.shape
        self._target = target
        t, keep = target.to_struct(self.dim)
        lib = _lib.require_gpu()
        h = C.c_void_p()
        _lib.check(create_fn(lib)(C.byref(t), _lib.dtype_code(self.dtype), self.n_chains, self.dim,
                                  _lib.ptr(x), *extra, chain_offset, C.byref(h)))
        del keep
        self._h = h
        self._lib = lib
        self._gen = 0  # incremented by every run: DeviceSamples of older runs are stale

    # -- lifetime ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.gm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- common API -------------------------------------------------------
    def _seed(self, seed: int):
        _lib.check(self._lib.gm_set_seed(self._h, int(seed) & 0xFFFFFFFFFFFFFFFF))
        return self

    def step(self):
        _lib.check(self._lib.gm_step(self._h))

    def run(self, n_collect: int, n_discard: int) -> np.ndarray:
        """[n_chains, n_collect, dim] on the host."""
        out = np.empty((self.n_chains, n_collect, self.dim), dtype=self.dtype)
        self._gen += 1
        _lib.check(self._lib.gm_run(self._h, n_collect, n_discard, _lib.ptr(out)))
        return out

    def run_positions(self, n_collect: int, n_discard: int) -> DeviceSamples:
        p = C.c_void_p()
        self._gen += 1
        _lib.check(self._lib.gm_run_device(self._h, n_collect, n_discard, C.byref(p)))
        return DeviceSamples(p.value or 0, n_collect, self.n_chains, self.dim, self.dtype, self, self._gen)

    _progress_prefix = "Sampler"
    _progress_interval = 1.0

    def run_progress(self, n_collect: int, n_discard: int, progress=None, interval: float | None = None):
        """(sample [n_chains, n_collect, dim], RunStats | None): the statistics
        are the device-side split-R-hat/ESS of the collected draws.

        `progress`: None (silent), True (a progress line on stderr, as the
        reference's progress bars, hmc.rs:255-288 / core.rs:272-345), or a
        callable receiving a `Progress` (done, total, p_accept, max_rhat)
        from the device-side trackers at most every `interval` seconds and
        after the last transition."""
        out = np.empty((self.n_chains, n_collect, self.dim), dtype=self.dtype)
        cb = _lib.PROGRESS_FN()
        if progress is not None and progress is not False:
            fn = _print_progress(self._progress_prefix) if progress is True else progress

            def _cb(_user, info):
                i = info.contents
                fn(Progress(int(i.done), int(i.total), float(i.p_accept), float(i.max_rhat)))
            cb = _lib.PROGRESS_FN(_cb)
        iv = self._progress_interval if interval is None else float(interval)
        stats = None
        self._gen += 1
        if n_collect >= 2:
            rhat = np.empty(self.dim, dtype=np.float32)
            ess = np.empty(self.dim, dtype=np.float32)
            _lib.check(self._lib.gm_run_progress_cb(self._h, n_collect, n_discard, _lib.ptr(out),
                                                    _lib.ptr(rhat), _lib.ptr(ess), cb, None, iv))
            stats = RunStats.from_arrays(rhat, ess)
        else:
            _lib.check(self._lib.gm_run_progress_cb(self._h, n_collect, n_discard, _lib.ptr(out), None,
                                                    None, cb, None, iv))
        return out, stats

    def chain_stats(self) -> "ChainStats":
        """ChainTracker::stats of every chain after an MH / NUTS run_progress
        (stats.rs:122-131): n, p_accept [C], mean [C, dim], sm2 [C, dim]."""
        n = C.c_uint64()
        p = np.empty(self.n_chains, dtype=np.float32)
        m = np.empty((self.n_chains, self.dim), dtype=np.float32)
        v = np.empty((self.n_chains, self.dim), dtype=np.float32)
        _lib.check(self._lib.gm_sampler_chain_stats(self._h, C.byref(n), _lib.ptr(p), _lib.ptr(m),
                                                    _lib.ptr(v)))
        return ChainStats(int(n.value), p, m, v)

    def copy_samples(self, n_collect: int) -> np.ndarray:
        """Samples of the last run, [n_chains, n_collect, dim] on the host
        (n_collect must be that run's: the library rejects a mismatch)."""
        out = np.empty((self.n_chains, n_collect, self.dim), dtype=self.dtype)
        _lib.check(self._lib.gm_copy_samples(self._h, n_collect, _lib.ptr(out)))
        return out

    def positions(self) -> np.ndarray:
        out = np.empty((self.n_chains, self.dim), dtype=self.dtype)
        _lib.check(self._lib.gm_get_positions(self._h, _lib.ptr(out)))
        return out

    def set_positions(self, x) -> None:
        x = np.ascontiguousarray(np.asarray(x, dtype=self.dtype))
        if x.shape != (self.n_chains, self.dim):
            raise ValueError("positions must be [n_chains][dim]")
        _lib.check(self._lib.gm_set_positions(self._h, _lib.ptr(x)))

    def accept_counts(self) -> np.ndarray:
        out = np.empty(self.n_chains, dtype=np.int64)
        _lib.check(self._lib.gm_get_accept_counts(self._h, _lib.ptr(out)))
        return out

    def leapfrog_counts(self) -> np.ndarray:
        out = np.empty(self.n_chains, dtype=np.int64)
        _lib.check(self._lib.gm_get_leapfrog_counts(self._h, _lib.ptr(out)))
        return out

    def layout(self) -> tuple[int, int]:
        a, b = C.c_int32(), C.c_int32()
        _lib.check(self._lib.gm_sampler_layout(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def set_layout(self, lanes: int, elems: int):
        _lib.check(self._lib.gm_sampler_set_layout(self._h, lanes, elems))
        return self

    def reserve(self, n_collect: int):
        """Pre-size the device sample buffer for runs of up to n_collect
        collected transitions (no allocation inside those runs)."""
        # growing the buffer frees the one earlier DeviceSamples point into
        self._gen += 1
        _lib.check(self._lib.gm_sampler_reserve(self._h, n_collect))
        return self

    def set_async(self, on: bool = True):
        """HMC / MH: run_positions and step return once the kernels are
        enqueued; call synchronize() (or gm_device_synchronize) before using
        the samples elsewhere (gm_sampler_set_async)."""
        _lib.check(self._lib.gm_sampler_set_async(self._h, 1 if on else 0))
        return self

    def synchronize(self):
        _lib.check(self._lib.gm_sampler_synchronize(self._h))

    def set_steps_per_launch(self, n: int):
        _lib.check(self._lib.gm_sampler_set_steps_per_launch(self._h, n))
        return self

    def set_unroll(self, n: int):
        """HMC leapfrog-loop unroll: 0 automatic, or 1, 2, 4 (same results)."""
        _lib.check(self._lib.gm_sampler_set_unroll(self._h, int(n)))
        return self

    def save_state(self) -> bytes:
        """Checkpoint (gm_state_save): positions, counters, seed and stream
        position, NUTS adaptation and metric. The reference has none
        (core.rs:177 TODO); a sampler restored with load_state continues the
        same draws bit for bit."""
        n = C.c_uint64()
        _lib.check(self._lib.gm_state_size(self._h, C.byref(n)))
        buf = (C.c_char * n.value)()
        _lib.check(self._lib.gm_state_save(self._h, buf, n.value))
        return bytes(buf)

    def load_state(self, blob: bytes):
        """Resume from save_state's bytes (same sampler kind, dtype, shape and
        chain offset)."""
        buf = (C.c_char * len(blob)).from_buffer_copy(blob)
        _lib.check(self._lib.gm_state_load(self._h, buf, len(blob)))
        return self

    def last_run_stats(self) -> tuple[float, int]:
        ms, n = C.c_double(), C.c_int64()
        _lib.check(self._lib.gm_sampler_last_run_stats(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def target(self):
        return self._target
