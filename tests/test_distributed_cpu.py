"""The N > 1 control plane on the CPU with gloo, world_size 2: contiguous
shards keyed by global chain id (the oracle replays each rank's shard and
the union equals the unsharded run), the byte broadcast that carries the
RCCL unique id, and the max-over-ranks timing reduction. The RCCL data
exchange itself needs GPUs (tests/test_gpu_distributed.py, and the driver's
8-GPU bench)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    from general_mcmc_amd.distributed import ControlPlane, shard
    from tests import _oracle
    import general_mcmc_amd as gm

    cp = ControlPlane()
    assert (cp.world, cp.rank) == (world, rank)
    off, c = shard(12, world, rank)
    x_all = gm.init_with_seed(12, 5, 42, np.float32)
    ora = _oracle.load()
    q, smp, acc = ora.hmc_run(_oracle.Target(1, 5), x_all[off:off + c], 0.05, 4, 7, 0, 6, 2, 8, 1,
                              chain_offset=off, threads=1)
    np.save(os.path.join(outdir, f"shard{rank}.npy"), smp)
    payload = bytes(range(128)) if rank == 0 else None
    got = cp.broadcast_bytes(payload)
    assert got == bytes(range(128))
    m = cp.max([float(rank), 10.0 - rank])
    assert list(m) == [world - 1.0, 10.0]
    cp.barrier()
    cp.close()


def test_gloo_world2_control_plane_and_sharding(tmp_path, oracle):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    import general_mcmc_amd as gm
    from tests._oracle import Target
    x_all = gm.init_with_seed(12, 5, 42, np.float32)
    _, full, _ = oracle.hmc_run(Target(1, 5), x_all, 0.05, 4, 7, 0, 6, 2, 8, 1)
    parts = [np.load(tmp_path / f"shard{r}.npy") for r in range(world)]
    np.testing.assert_array_equal(np.concatenate(parts, axis=1), full)


def test_shard_bounds():
    from general_mcmc_amd.distributed import shard
    assert [shard(65536, 8, r) for r in (0, 7)] == [(0, 8192), (57344, 8192)]
    with pytest.raises(ValueError):
        shard(10, 3, 0)
