"""Sample writers (io/csv.rs, io/arrow.rs, io/parquet.rs): the reference's
own io tests, restated on the host-array path."""
import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest


@pytest.fixture(scope="module")
def io():
    import general_mcmc_amd.io as m
    return m


def test_csv_empty(io, tmp_path):  # csv.rs:162-180
    f = tmp_path / "e.csv"
    io.save_csv(np.zeros((0, 0, 0), dtype=np.float32), str(f))
    assert f.read_text().strip() == "chain,observation"


def test_csv_single(io, tmp_path):  # csv.rs:182-199
    f = tmp_path / "s.csv"
    io.save_csv(np.array([[[42.0]]]), str(f))
    assert f.read_text().strip() == "chain,observation,dim_0\n0,0,42"


def test_csv_multi_chain_ints(io, tmp_path):  # csv.rs:201-222
    f = tmp_path / "m.csv"
    io.save_csv(np.array([[[1, 2], [3, 4]], [[10, 20], [30, 40]]]), str(f))
    assert f.read_text().strip() == (
        "chain,observation,dim_0,dim_1\n0,0,1,2\n0,1,3,4\n1,0,10,20\n1,1,30,40")


def test_csv_tensor_f32_display(io, tmp_path):  # csv.rs:224-268
    f = tmp_path / "t.csv"
    io.save_csv_tensor(np.array([[[1.0, 2.0], [3.0, 4.0]], [[1.1, 2.1], [3.1, 4.1]]]), str(f))
    rows = [r.split(",") for r in f.read_text().strip().split("\n")]
    assert rows[0] == ["chain", "observation", "dim_0", "dim_1"]
    assert rows[1:] == [["0", "0", "1", "2"], ["0", "1", "3", "4"], ["1", "0", "1.1", "2.1"],
                        ["1", "1", "3.1", "4.1"]]  # f32 shortest digits


def test_rust_display_format(io):
    d = io._display
    assert d(np.float64(1e-7)) == "0.0000001" and d(np.float64(1e21)) == "1000000000000000000000"
    assert d(np.float64(-0.0)) == "-0" and d(np.float64(np.nan)) == "NaN"
    assert d(np.float64(-np.inf)) == "-inf" and d(np.float32(0.1)) == "0.1"
    assert d(np.float64(np.float32(0.1))) == "0.10000000149011612"


def test_arrow_empty(io, tmp_path):  # arrow.rs:131-161
    f = tmp_path / "e.arrow"
    io.save_arrow(np.zeros((0, 0, 0), dtype=np.float32), str(f))
    r = pa.ipc.open_file(str(f))
    assert r.num_record_batches == 1
    b = r.get_batch(0)
    assert b.num_rows == 0 and b.num_columns == 2


def test_arrow_multi_chain_f32(io, tmp_path):  # arrow.rs:205-290
    f = tmp_path / "m.arrow"
    io.save_arrow(np.array([[[1, 2.5], [3, 4.5]], [[10, 20.5], [30, 40.5]]], dtype=np.float32), str(f))
    r = pa.ipc.open_file(str(f))
    assert r.num_record_batches == 1
    t = r.read_all()
    assert t.schema.names == ["chain", "observation", "dim_0", "dim_1"]
    assert t.schema.field("chain").type == pa.uint32() and not t.schema.field("chain").nullable
    assert t.schema.field("dim_0").type == pa.float64()
    assert t.column("chain").to_pylist() == [0, 0, 1, 1]
    assert t.column("observation").to_pylist() == [0, 1, 0, 1]
    assert t.column("dim_0").to_pylist() == [1.0, 3.0, 10.0, 30.0]
    assert t.column("dim_1").to_pylist() == [2.5, 4.5, 20.5, 40.5]


def test_parquet_empty(io, tmp_path):  # parquet.rs:236-258
    f = tmp_path / "e.parquet"
    io.save_parquet(np.zeros((0, 0, 0), dtype=np.float32), str(f))
    assert f.stat().st_size > 0
    assert list(pq.ParquetFile(str(f)).iter_batches()) == []


def test_parquet_single_and_multi(io, tmp_path):  # parquet.rs:262-380
    f = tmp_path / "s.parquet"
    io.save_parquet(np.array([[[42.0]]]), str(f))
    t = pq.read_table(str(f))
    assert t.num_rows == 1 and t.num_columns == 3 and t.column("dim_0").to_pylist() == [42.0]
    f = tmp_path / "m.parquet"
    io.save_parquet(np.array([[[1.0, 2.0], [3.0, 4.0]], [[10.0, 20.0], [30.0, 40.0]]]), str(f))
    t = pq.read_table(str(f))
    assert t.column("chain").to_pylist() == [0, 0, 1, 1]
    assert t.column("observation").to_pylist() == [0, 1, 0, 1]
    assert t.column("dim_1").to_pylist() == [2.0, 4.0, 20.0, 40.0]
    assert pq.ParquetFile(str(f)).metadata.row_group(0).column(2).compression == "UNCOMPRESSED"


def test_parquet_tensor_obs_major(io, tmp_path):  # parquet.rs:382-446
    f = tmp_path / "t.parquet"
    x = np.array([[[1.0, 2.0], [3.0, 4.0]], [[1.1, 2.1], [3.1, 4.1]]], dtype=np.float32)
    io.save_parquet_tensor(x, str(f))
    t = pq.read_table(str(f))
    assert t.schema.names == ["observation", "chain", "dim_0", "dim_1"]
    assert t.column("observation").to_pylist() == [0, 0, 1, 1]
    assert t.column("chain").to_pylist() == [0, 1, 0, 1]
    np.testing.assert_allclose(t.column("dim_0").to_pylist(), [1.0, 3.0, 1.1, 3.1], atol=1e-6)
