"""Multi-GPU execution: one process per GPU, chains sharded in contiguous
blocks, no communication while sampling; the split-R-hat/ESS diagnostic is
the single exchange (an RCCL all-gather inside libgmcmc over xGMI).

The control plane (rank discovery, barrier, the RCCL unique-id broadcast,
max-over-ranks timing) uses torch.distributed with the gloo backend, so the
process never initialises torch's own HIP runtime.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib


def shard(n_global: int, world: int, rank: int) -> tuple[int, int]:
    """(offset, count) of rank's contiguous block; equal shards required by the
    diagnostic all-gather, so n_global must divide evenly."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    if n_global % world:
        raise ValueError(f"{n_global} chains do not split evenly over {world} ranks")
    c = n_global // world
    return rank * c, c


class ControlPlane:
    """torch.distributed (gloo) from the torchrun environment; a no-op when
    WORLD_SIZE is 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def broadcast_bytes(self, payload: bytes | None, src: int = 0) -> bytes:
        if self.dist is None:
            return payload
        obj = [payload]
        self.dist.broadcast_object_list(obj, src=src)
        return obj[0]

    def gather(self, obj) -> list:
        """Every rank's obj, on every rank (rank order)."""
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def max(self, values) -> np.ndarray:
        v = np.asarray(values, dtype=np.float64)
        if self.dist is None:
            return v
        import torch
        t = torch.tensor(v)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return t.numpy()

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


class Comm:
    """RCCL communicator owned by libgmcmc (gm_comm_init)."""

    def __init__(self, cp: ControlPlane, lib=None):
        self.lib = lib or _lib.load()
        self.cp = cp
        uid = None
        if cp.rank == 0:
            buf = (C.c_char * _lib.UNIQUE_ID_BYTES)()
            _lib.check(self.lib.gm_comm_get_unique_id(buf))
            uid = bytes(buf)
        uid = cp.broadcast_bytes(uid)
        buf = (C.c_char * _lib.UNIQUE_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        _lib.check(self.lib.gm_comm_init(buf, cp.world, cp.rank, C.byref(h)))
        self.h = h

    def info(self) -> dict:
        """What RCCL reports for this communicator (ncclCommCount /
        ncclCommUserRank / ncclCommCuDevice)."""
        n, r, d = C.c_int32(), C.c_int32(), C.c_int32()
        _lib.check(self.lib.gm_comm_info(self.h, C.byref(n), C.byref(r), C.byref(d)))
        return {"nranks": n.value, "rank": r.value, "device": d.value}

    def split_rhat_ess(self, ds) -> tuple[np.ndarray, np.ndarray]:
        """Diagnostics of the union of all ranks' chains from each rank's
        DeviceSamples ([n_collect][C_local][dim] on its GPU)."""
        ds._check_live()
        ds.owner.synchronize()  # an asynchronous run may still be writing them
        rhat = np.empty(ds.dim, dtype=np.float32)
        ess = np.empty(ds.dim, dtype=np.float32)
        _lib.check(self.lib.gm_split_rhat_ess_dist(
            self.h, C.c_void_p(ds.ptr), _lib.dtype_code(ds.dtype), ds.n_chains, ds.n_collect, ds.dim,
            ds.dim, ds.n_chains * ds.dim, 1, _lib.ptr(rhat), _lib.ptr(ess)))
        return rhat, ess

    def close(self):
        if getattr(self, "h", None) is not None:
            self.lib.gm_comm_destroy(self.h)
            self.h = None


def split_rhat_ess_shards(shards) -> tuple[np.ndarray, np.ndarray]:
    """Diagnostics of the union of several DeviceSamples shards on this GPU
    (equal chain counts, same n_collect and dim), assembled exactly as the
    RCCL all-gather of Comm.split_rhat_ess assembles the ranks' blocks
    (gm_split_rhat_ess_shards)."""
    lib = _lib.require_gpu()
    d0 = shards[0]
    for d in shards:
        d._check_live()
        d.owner.synchronize()
        if (d.n_chains, d.n_collect, d.dim, np.dtype(d.dtype)) != (d0.n_chains, d0.n_collect, d0.dim,
                                                                   np.dtype(d0.dtype)):
            raise ValueError("shards must have equal chain counts, draws, dims and dtypes")
    ptrs = (C.c_void_p * len(shards))(*[d.ptr for d in shards])
    rhat = np.empty(d0.dim, dtype=np.float32)
    ess = np.empty(d0.dim, dtype=np.float32)
    _lib.check(lib.gm_split_rhat_ess_shards(
        ptrs, len(shards), _lib.dtype_code(d0.dtype), d0.n_chains, d0.n_collect, d0.dim,
        d0.dim, d0.n_chains * d0.dim, 1, _lib.ptr(rhat), _lib.ptr(ess)))
    return rhat, ess
