"""Sample egress and on-disk formats (the reference's `io` module:
io/csv.rs, io/arrow.rs, io/parquet.rs).

Every writer takes either a host array or the `DeviceSamples` handle that
`run_positions` returns. A DeviceSamples is streamed from the GPU in blocks
(gm_copy_sample_block, one strided copy each), so a sample larger than host
memory never exists on the host whole.

Layouts, as in the reference:
  save_csv / save_arrow / save_parquet   data[chain][observation][dim], rows
                                         ordered chain-major (csv.rs:47-71,
                                         arrow.rs:53-117, parquet.rs:49-110)
  save_csv_tensor                        same, values converted to f32 first
                                         (csv.rs:113-147)
  save_parquet_tensor                    tensor[observation][chain][dim], rows
                                         ordered observation-major, columns
                                         observation, chain, dim_* (parquet.rs:
                                         112-221). This is the device layout of
                                         run_positions, and the reverse of the
                                         [chain, obs, dim] that HMC::run returns
                                         (a reference inconsistency, kept).
Schema: chain / observation UInt32 (non-null), dim_i Float64 (non-null).
CSV values use Rust's Display for the element type (shortest round-trip
digits, never an exponent; NaN, inf).
"""
from __future__ import annotations

import numpy as np

from ._sampler import DeviceSamples

_CHAIN_BLOCK_BYTES = 64 << 20  # host staging per streamed block


# ---- sources: host arrays or device samples, in [chain, obs, dim] ----------

def _chain_major_blocks(data):
    """Yields (chain0, block[c, n, d]) over the sample in chain order."""
    if isinstance(data, DeviceSamples):
        C, N, D = data.n_chains, data.n_collect, data.dim
        per_chain = max(1, N * D * np.dtype(data.dtype).itemsize)
        cb = max(1, min(C, _CHAIN_BLOCK_BYTES // per_chain))
        for c0 in range(0, C, cb):
            n = min(cb, C - c0)
            yield c0, data.block(0, N, c0, n).transpose(1, 0, 2)  # [N][n][D] -> [n][N][D]
        return
    a = np.asarray(data)
    if a.ndim != 3:
        raise ValueError("data must be [chain][observation][dim]")
    yield 0, a


def _shape(data):
    if isinstance(data, DeviceSamples):
        return data.n_chains, data.n_collect, data.dim
    a = np.asarray(data)
    if a.ndim != 3:
        raise ValueError("expected a 3-D array")
    return a.shape


# ---- CSV --------------------------------------------------------------------

def _display(v) -> str:
    """Rust `Display` of a number (what `to_string()` writes, csv.rs:66)."""
    if isinstance(v, (np.integer, int)):
        return str(int(v))
    if np.isnan(v):
        return "NaN"
    if np.isinf(v):
        return "inf" if v > 0 else "-inf"
    return np.format_float_positional(v, unique=True, trim="-")


def _write_csv(blocks, n_dims, filename):
    with open(filename, "w", newline="") as f:
        f.write(",".join(["chain", "observation"] + [f"dim_{i}" for i in range(n_dims)]) + "\n")
        for c0, blk in blocks:
            for ci, chain in enumerate(blk):
                for oi, obs in enumerate(chain):
                    f.write(",".join([str(c0 + ci), str(oi)] + [_display(v) for v in obs]) + "\n")


def save_csv(data, filename: str) -> None:
    """save_csv (csv.rs:47-71): header chain, observation, dim_0..; one row
    per (chain, observation)."""
    _, _, D = _shape(data)
    _write_csv(_chain_major_blocks(data), D, filename)


def save_csv_tensor(tensor, filename: str) -> None:
    """save_csv_tensor (csv.rs:113-147): as save_csv, with the values
    converted to f32 first (`to_vec::<f32>`, csv.rs:123-125)."""
    _, _, D = _shape(tensor)
    blocks = ((c0, b.astype(np.float32)) for c0, b in _chain_major_blocks(tensor))
    _write_csv(blocks, D, filename)


# ---- Arrow / Parquet ---------------------------------------------------------

def _schema(n_dims, obs_first=False):
    import pyarrow as pa
    idx = [pa.field("chain", pa.uint32(), nullable=False),
           pa.field("observation", pa.uint32(), nullable=False)]
    if obs_first:
        idx = idx[::-1]
    return pa.schema(idx + [pa.field(f"dim_{i}", pa.float64(), nullable=False) for i in range(n_dims)])


def _chain_major_batch(schema, c0, blk):
    import pyarrow as pa
    n, N, D = blk.shape
    chain = np.repeat(np.arange(c0, c0 + n, dtype=np.uint32), N)
    obs = np.tile(np.arange(N, dtype=np.uint32), n)
    vals = blk.reshape(n * N, D).astype(np.float64)  # Into<f64>
    cols = [pa.array(chain, pa.uint32()), pa.array(obs, pa.uint32())]
    cols += [pa.array(np.ascontiguousarray(vals[:, i]), pa.float64()) for i in range(D)]
    return pa.record_batch(cols, schema=schema)


def _empty_batch(schema):
    import pyarrow as pa
    return pa.record_batch([pa.array([], f.type) for f in schema], schema=schema)


def save_arrow(data, filename: str) -> None:
    """save_arrow (arrow.rs:53-117): an Arrow IPC file. A host array is one
    record batch, as the reference writes; streamed device samples are one
    batch per chain block (the same rows in the same order)."""
    import pyarrow as pa
    C, N, D = _shape(data)
    schema = _schema(D)
    with pa.OSFile(filename, "wb") as sink, pa.ipc.new_file(sink, schema) as w:
        if C * N == 0:
            w.write_batch(_empty_batch(schema))  # zero-row batch (arrow.rs:76-77, 104-111)
            return
        for c0, blk in _chain_major_blocks(data):
            w.write_batch(_chain_major_batch(schema, c0, blk))


def save_parquet(data, filename: str) -> None:
    """save_parquet (parquet.rs:49-110): same schema as save_arrow,
    uncompressed (the parquet crate's default WriterProperties)."""
    import pyarrow.parquet as pq
    C, N, D = _shape(data)
    schema = _schema(D)
    with pq.ParquetWriter(filename, schema, compression="NONE") as w:
        for c0, blk in _chain_major_blocks(data):
            if blk.size:
                w.write_batch(_chain_major_batch(schema, c0, blk))


def save_parquet_tensor(tensor, filename: str) -> None:
    """save_parquet_tensor (parquet.rs:152-221): tensor[observation][chain][dim],
    columns observation, chain, dim_*; rows observation-major. A
    DeviceSamples is already laid out this way on the GPU and streams by row
    blocks."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    if isinstance(tensor, DeviceSamples):
        N, C, D = tensor.n_collect, tensor.n_chains, tensor.dim
        per_row = max(1, C * D * np.dtype(tensor.dtype).itemsize)
        rb = max(1, min(N, _CHAIN_BLOCK_BYTES // per_row))
        blocks = ((r0, tensor.block(r0, min(rb, N - r0), 0, C)) for r0 in range(0, N, rb))
    else:
        a = np.asarray(tensor)
        if a.ndim != 3:
            raise ValueError("tensor must be [observation][chain][dim]")
        N, C, D = a.shape
        blocks = iter([(0, a)])
    schema = _schema(D, obs_first=True)
    with pq.ParquetWriter(filename, schema, compression="NONE") as w:
        for r0, blk in blocks:
            n = blk.shape[0]
            if n * C == 0:
                continue
            obs = np.repeat(np.arange(r0, r0 + n, dtype=np.uint32), C)
            chain = np.tile(np.arange(C, dtype=np.uint32), n)
            vals = blk.reshape(n * C, D).astype(np.float64)
            cols = [pa.array(obs, pa.uint32()), pa.array(chain, pa.uint32())]
            cols += [pa.array(np.ascontiguousarray(vals[:, i]), pa.float64()) for i in range(D)]
            w.write_batch(pa.record_batch(cols, schema=schema))
