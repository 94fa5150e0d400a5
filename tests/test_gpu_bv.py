"""Tier-2 boundary: the granular BatchVector ops (gm_bv_*, euclidean.rs:447-534)
on device buffers. Each op is checked against the oracle / IEEE arithmetic,
and the reference's own step loop (BatchedGenericHMC::step,
batched_hmc.rs:129-190) composed from them must reproduce the oracle's
reference-structure leapfrog bit for bit; the one-kernel leapfrog
(gm_bv_leapfrog) reproduces the fused kernel."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bv(gm):
    return gm.batch_vector


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_elementwise_ops_ieee(bv, dtype):
    rng = np.random.default_rng(3)
    C, D = 37, 11
    x = rng.standard_normal((C, D)).astype(dtype)
    o = rng.standard_normal((C, D)).astype(dtype)
    dx, do = bv.DeviceMatrix.from_host(x), bv.DeviceMatrix.from_host(o)
    alpha = dtype(0.5) * dtype(0.013)
    bv.add_scaled_assign(dx, do, alpha)
    np.testing.assert_array_equal(dx.to_host(), x + o * alpha)  # two roundings (euclidean.rs:392-394)
    mask = (rng.random(C) < 0.5).astype(np.uint8)
    y = dx.to_host()
    bv.masked_assign(dx, do, bv.DeviceMatrix.from_host(mask))
    np.testing.assert_array_equal(dx.to_host(), np.where(mask[:, None] == 1, o, y))
    a = rng.standard_normal(C).astype(dtype)
    b = rng.standard_normal(C).astype(dtype)
    da, db = bv.DeviceMatrix.from_host(a), bv.DeviceMatrix.from_host(b)
    np.testing.assert_array_equal(bv.energy_sub(da, db).to_host(), a - b)
    np.testing.assert_array_equal(bv.energy_add(da, db).to_host(), a + b)
    np.testing.assert_array_equal(bv.energy_neg(da).to_host(), -a)
    la = np.array([0.0, -1.0, np.nan, 2.0, -np.inf], dtype=dtype)
    lu = np.array([0.0, -0.5, -1.0, np.nan, -np.inf], dtype=dtype)
    m = bv.accept_mask(bv.DeviceMatrix.from_host(la), bv.DeviceMatrix.from_host(lu)).to_host()
    np.testing.assert_array_equal(m, [1, 0, 0, 0, 1])  # >=, NaN rejects (euclidean.rs:532)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_random_fills_and_ln_match_oracle(bv, oracle, dtype):
    C, D, seed, step, off = 9, 5, 77, 13, 100
    z = bv.DeviceMatrix((C, D), dtype)
    bv.fill_random_normal(z, seed, step, chain_offset=off)
    sfx = "f" if dtype == np.float32 else "d"
    nrm = getattr(oracle.lib, f"or_mom_normal_{sfx}")  # the HMC momentum draws (f32: spec v5 tables)
    exp = np.array([[nrm(seed, off + c, step, 2, j) for j in range(D)] for c in range(C)], dtype=dtype)
    np.testing.assert_array_equal(z.to_host(), exp)
    u = bv.sample_uniform(C, dtype, seed, step, chain_offset=off)
    uni = getattr(oracle.lib, f"or_uniform_co_{sfx}")
    ue = np.array([uni(seed, off + c, step, 3, 0) for c in range(C)], dtype=dtype)
    np.testing.assert_array_equal(u.to_host(), ue)
    lg = getattr(oracle.lib, f"or_log_{sfx}")
    np.testing.assert_array_equal(bv.energy_ln(u).to_host(), np.array([lg(v) for v in ue], dtype=dtype))


@pytest.mark.parametrize("D", [1, 7, 64, 100, 300])
def test_kinetic_energy_canonical_order(gm, bv, oracle, D):
    """K(p) = (sum p^2)*0.5 equals -logp of IsotropicGaussian(1) in the same
    canonical summation order (scaling by 0.5 and dividing by 1 are exact)."""
    rng = np.random.default_rng(D)
    p = rng.standard_normal((17, D)).astype(np.float32)
    ke = bv.kinetic_energy(bv.DeviceMatrix.from_host(p)).to_host()
    s = gm.HMC(gm.IsotropicGaussian(1.0), p, 0.1, 1)
    lanes, elems = s.layout()
    lp, _ = oracle.logp_grad(Target(2, D, std=1.0), p, lanes, elems, np.float32)
    np.testing.assert_array_equal(ke, -lp)


def test_logp_and_grad_device(gm, bv, oracle):
    rng = np.random.default_rng(5)
    x = rng.standard_normal((33, 64)).astype(np.float32)
    t = bv.BatchTarget(gm.RosenbrockND(), 64, np.float32)
    dx = bv.DeviceMatrix.from_host(x)
    g = bv.DeviceMatrix.like(dx)
    lp = t.logp_and_grad(dx, g).to_host()
    elp, eg = oracle.logp_grad(Target(1, 64), x, 64, 1, np.float32)
    np.testing.assert_array_equal(lp, elp)
    np.testing.assert_array_equal(g.to_host(), eg)


CASES = [
    ("rosen64_f32", lambda gm: gm.RosenbrockND(), 64, np.float32, 0.01, 7),
    ("rosen10_f64", lambda gm: gm.RosenbrockND(), 10, np.float64, 0.02, 5),
    ("rosen100_f32", lambda gm: gm.RosenbrockND(), 100, np.float32, 0.005, 4),
    ("iso7_f32", lambda gm: gm.IsotropicGaussian(1.5), 7, np.float32, 0.3, 6),
    ("gauss2d_f64", lambda gm: gm.DiffableGaussian2D([0.0, 1.0], [[4.0, 2.0], [2.0, 3.0]]), 2,
     np.float64, 0.1, 10),
]


def _oracle_runs(gm, oracle, mk, x0, D, dtype, eps, L, off, form):
    """the oracle's two calls matching run(3, 0) then run(4, 2), at the
    layout the sampler and the tier-2 target pick for this dim"""
    lay = gm.HMC(mk(gm), x0, eps, L, dtype=dtype).layout()
    t = Target.from_product(mk(gm), D)
    q, s1, _ = oracle.hmc_run(t, x0, eps, L, 9, 0, 3, 0, *lay, chain_offset=off, form=form)
    q, s2, _ = oracle.hmc_run(t, q, eps, L, 9, 3, 6, 2, *lay, chain_offset=off, form=form)
    return s1.transpose(1, 0, 2), s2.transpose(1, 0, 2), q


@pytest.mark.parametrize("name,mk,D,dtype,eps,L", CASES, ids=[c[0] for c in CASES])
def test_composed_step_equals_reference_op_structure(gm, bv, oracle, name, mk, D, dtype, eps, L):
    """batched_hmc.rs:129-190 op by op (add_scaled_assign rounds the product
    and the sum separately, euclidean.rs:392-394) == the oracle's
    reference-structure form, bitwise, including a chain offset (sharded
    streams) and a mid-block start (step 3); the fused kernel == the oracle's
    engine form (fused multiply-add kicks and drift), and the two forms agree
    to rounding."""
    C, off = 48, 1000
    x0 = gm.init_with_seed(C, D, 11, dtype)
    composed = bv.BatchedGenericHMC(mk(gm), x0, eps, L, seed=9, chain_offset=off)
    fused = gm.HMC(mk(gm), x0, eps, L, dtype=dtype, chain_offset=off).set_seed(9)
    a1, a2 = composed.run(3, 0), composed.run(4, 2)
    b1, b2 = fused.run(3, 0), fused.run(4, 2)
    r1, r2, rq = _oracle_runs(gm, oracle, mk, x0, D, dtype, eps, L, off, form=1)
    np.testing.assert_array_equal(a1, r1)
    np.testing.assert_array_equal(a2, r2)
    np.testing.assert_array_equal(composed.positions(), rq)
    e1, e2, eq = _oracle_runs(gm, oracle, mk, x0, D, dtype, eps, L, off, form=0)
    np.testing.assert_array_equal(b1, e1)
    np.testing.assert_array_equal(b2, e2)
    np.testing.assert_array_equal(fused.positions(), eq)
    # the same chains to rounding: the first transition's draws (accept
    # decisions can flip on a rounding-level difference later on)
    tol = 1e-4 if dtype == np.float32 else 1e-10
    np.testing.assert_allclose(a1[:, 0], b1[:, 0], rtol=tol, atol=tol)


@pytest.mark.parametrize("name,mk,D,dtype,eps,L", CASES, ids=[c[0] for c in CASES])
def test_hbm_leapfrog_equals_fused_kernel(gm, bv, name, mk, D, dtype, eps, L):
    """gm_bv_leapfrog (one kernel per leapfrog, state in HBM) == the fused
    kernel, bitwise (the same fused multiply-add kicks and drift)."""
    C, off = 48, 1000
    x0 = gm.init_with_seed(C, D, 11, dtype)
    per_lf = bv.BatchedGenericHMC(mk(gm), x0, eps, L, seed=9, chain_offset=off, fused_leapfrog=True)
    fused = gm.HMC(mk(gm), x0, eps, L, dtype=dtype, chain_offset=off).set_seed(9)
    np.testing.assert_array_equal(per_lf.run(3, 1), fused.run(3, 1))


@pytest.mark.parametrize("D,dtype", [(64, np.float32), (32, np.float64), (16, np.float32), (128, np.float32),
                                     (256, np.float64)])
@pytest.mark.parametrize("C", [1, 5, 50, 1001])
def test_hbm_leapfrog_ragged(gm, bv, D, dtype, C):
    """gm_bv_leapfrog with a partial last block (C not a multiple of the
    chains per block) == the fused kernel, bitwise."""
    x0 = gm.init_with_seed(C, D, 5, dtype)
    per_lf = bv.BatchedGenericHMC(gm.RosenbrockND(), x0, 0.01, 3, seed=2, fused_leapfrog=True)
    fused = gm.HMC(gm.RosenbrockND(), x0, 0.01, 3, dtype=dtype).set_seed(2)
    np.testing.assert_array_equal(per_lf.run(2, 1), fused.run(2, 1))


def test_bv_rejects_bad_arguments(gm, bv):
    a = bv.DeviceMatrix((4, 3), np.float32)
    b = bv.DeviceMatrix((4, 2), np.float32)
    with pytest.raises(ValueError):
        bv.add_scaled_assign(a, b, 1.0)
    lib = gm._lib.load()
    assert lib.gm_bv_kinetic_energy(7, 4, 3, None, None) == gm._lib.GM_EINVAL  # bad dtype


def test_writers_stream_device_samples(gm, tmp_path, monkeypatch):
    """io writers on DeviceSamples (streamed by blocks) == on the host copy."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    import general_mcmc_amd.io as gio
    s = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(37, 5, 3, np.float32), 0.02, 4).set_seed(2)
    ds = s.run_positions(11, 2)
    host = ds.to_host()  # [C, N, D]
    np.testing.assert_array_equal(ds.block(3, 4, 5, 9), host[5:14, 3:7].transpose(1, 0, 2))
    monkeypatch.setattr(gio, "_CHAIN_BLOCK_BYTES", 700)  # several blocks
    for name, fn in (("a.arrow", gio.save_arrow), ("p.parquet", gio.save_parquet), ("c.csv", gio.save_csv)):
        fn(ds, str(tmp_path / ("d" + name)))
        fn(host, str(tmp_path / ("h" + name)))
    assert (tmp_path / "dc.csv").read_text() == (tmp_path / "hc.csv").read_text()
    assert pa.ipc.open_file(str(tmp_path / "da.arrow")).read_all().equals(
        pa.ipc.open_file(str(tmp_path / "ha.arrow")).read_all())
    assert pq.read_table(str(tmp_path / "dp.parquet")).equals(pq.read_table(str(tmp_path / "hp.parquet")))
    gio.save_parquet_tensor(ds, str(tmp_path / "dt.parquet"))
    gio.save_parquet_tensor(host.transpose(1, 0, 2), str(tmp_path / "ht.parquet"))
    assert pq.read_table(str(tmp_path / "dt.parquet")).equals(pq.read_table(str(tmp_path / "ht.parquet")))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_euclidean_scale_fill_dot(bv, dtype):
    """EuclideanVector's remaining ops (euclidean.rs:11-56) the Rust seam of
    INTEGRATION.md binds: scale_assign bitwise, fill, and dot against a float64
    sum (summation order is the engine's: 1024 strided partials, then a tree)."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal((129, 33)).astype(dtype)
    y = rng.standard_normal((129, 33)).astype(dtype)
    dx, dy = bv.DeviceMatrix.from_host(x), bv.DeviceMatrix.from_host(y)
    a = dtype(0.37)
    bv.scale_assign(dx, a)
    np.testing.assert_array_equal(dx.to_host(), x * a)
    got = bv.dot(dx, dy)
    ref = float(np.sum((x * a).astype(np.float64) * y.astype(np.float64)))
    assert abs(got - ref) <= (1e-4 if dtype == np.float32 else 1e-12) * max(1.0, abs(ref))
    bv.fill(dy, 0.0)
    assert not dy.to_host().any()
    bv.fill(dy, 2.5)
    assert (dy.to_host() == dtype(2.5)).all()
    assert bv.dot(bv.DeviceMatrix((0,), dtype), bv.DeviceMatrix((0,), dtype)) == 0.0


@pytest.mark.parametrize("nbytes,off", [(16, 0), (4096 * 16 + 16, 0), ((1 << 24) + 48, 0), (1000, 0), (4096, 8),
                                        (17, 3)])
def test_memcpy_dtod_sizes_and_alignment(gm, nbytes, off):
    """assign (euclidean.rs:380-382) through gm_memcpy_dtod: the 16-byte copy
    kernel for aligned whole-word buffers (partial last pass included), the
    runtime copy otherwise (odd sizes, 8-byte offsets); every byte equal."""
    import ctypes as C
    lib, _lib = gm._lib.load(), gm._lib
    rng = np.random.default_rng(nbytes)
    h = rng.integers(0, 256, nbytes + off, dtype=np.uint8)
    src, dst = C.c_void_p(), C.c_void_p()
    _lib.check(lib.gm_malloc(C.byref(src), nbytes + off))
    _lib.check(lib.gm_malloc(C.byref(dst), nbytes + off))
    try:
        _lib.check(lib.gm_memcpy_htod(src, h.ctypes.data, nbytes + off))
        _lib.check(lib.gm_memcpy_dtod(C.c_void_p(dst.value + off), C.c_void_p(src.value + off), nbytes))
        _lib.check(lib.gm_device_synchronize())
        out = np.zeros(nbytes + off, np.uint8)
        _lib.check(lib.gm_memcpy_dtoh(out.ctypes.data, C.c_void_p(dst.value + off), nbytes))
        np.testing.assert_array_equal(out[:nbytes], h[off:off + nbytes])
    finally:
        lib.gm_free(src)
        lib.gm_free(dst)
