"""GPU parity: every kernel result compared with the CPU oracle on the same
seeded inputs through the C ABI. Integer/RNG-driven control flow must agree
exactly; floating-point results are compared BIT-FOR-BIT (kernels and oracle
share the declared operation order, no FMA contraction, the same Philox
streams and the same log/exp/cos implementations)."""
import numpy as np
import pytest

from tests._oracle import Target

pytestmark = pytest.mark.gpu

DTYPES = [np.float32, np.float64]


def targets(g, dim):
    rng = np.random.default_rng(dim)
    a = rng.standard_normal((dim, dim))
    cov = a @ a.T / dim + np.eye(dim)
    mean = rng.standard_normal(dim)
    out = [("rosenbrock", g.RosenbrockND()), ("iso", g.IsotropicGaussian(1.7)),
           ("gauss", g.DenseGaussian(mean, cov))]
    if dim == 2:
        out.append(("rosen2d", g.Rosenbrock2D(0.7, 20.0)))
    return out


def start(g, n, d, dtype, scale=0.5):
    return (g.init_with_seed(n, d, 3, np.float64) * scale).astype(dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("dim", [1, 2, 3, 7, 64, 100, 128, 300, 1000])
def test_target_logp_grad_bitwise(gm, oracle, dtype, dim):
    x = start(gm, 37, dim, dtype, 1.3)
    for name, t in targets(gm, dim):
        lp, g = t.unnorm_logp_and_grad_batch(x, dtype)
        olp, og = oracle.logp_grad(Target.from_product(t, dim), x, *_default_layout(dim), dtype)
        np.testing.assert_array_equal(lp, olp, err_msg=f"{name} logp")
        np.testing.assert_array_equal(g, og, err_msg=f"{name} grad")


def _default_layout(dim):
    if dim <= 64:
        p = 1
        while p < dim:
            p <<= 1
        return p, 1
    if dim <= 128:
        return 64, 2
    if dim <= 256:
        return 64, 4
    if dim <= 512:
        return 64, 8
    return 64, 16


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("dim,lay", [(2, (2, 1)), (3, (4, 1)), (33, (64, 1)), (64, (64, 1)),
                                     (64, (16, 4)), (64, (32, 2)), (100, (64, 2)), (128, (32, 4))])
def test_hmc_samples_bitwise(gm, oracle, dtype, dim, lay):
    n_chains, L, eps = 24, 7, 0.01
    x0 = start(gm, n_chains, dim, dtype)
    for name, t in targets(gm, dim):
        s = gm.HMC(t, x0, eps, L, dtype=dtype).set_seed(11)
        s.set_layout(*lay)
        s.set_steps_per_launch(4)  # exercise state hand-off across launches
        out = s.run(6, 3)  # [C, 6, D]
        q, samples, acc = oracle.hmc_run(Target.from_product(t, dim), x0, eps, L, 11, 0, 9, 3, *lay)
        np.testing.assert_array_equal(out, samples.transpose(1, 0, 2), err_msg=name)
        np.testing.assert_array_equal(s.positions(), q, err_msg=name)
        np.testing.assert_array_equal(s.accept_counts(), acc, err_msg=name)
        # second run continues the same streams
        out2 = s.run(2, 0)
        _, samples2, _ = oracle.hmc_run(Target.from_product(t, dim), q, eps, L, 11, 9, 2, 0, *lay)
        np.testing.assert_array_equal(out2, samples2.transpose(1, 0, 2), err_msg=name)
        s.close()


@pytest.mark.parametrize("unroll", [1, 2, 4])
@pytest.mark.parametrize("L", [7, 8, 1])
@pytest.mark.parametrize("dim,lay,dtype", [(64, (64, 1), np.float32), (128, (64, 2), np.float32),
                                           (32, (16, 2), np.float64)])
def test_hmc_unroll_forms_bitwise(gm, oracle, unroll, L, dim, lay, dtype):
    """The fused kernel's leapfrog loop unrolled x1, x2 and x4 (chosen by the
    launch's waves per SIMD; forced here with gm_sampler_set_unroll), odd,
    even and single leapfrog counts: the oracle's bits in every form."""
    n_chains, eps = 24, 0.01
    x0 = start(gm, n_chains, dim, dtype)
    t = gm.RosenbrockND()
    s = gm.HMC(t, x0, eps, L, dtype=dtype).set_seed(5)
    s.set_layout(*lay)
    s.set_unroll(unroll)
    out = s.run(3, 2)
    q, samples, acc = oracle.hmc_run(Target.from_product(t, dim), x0, eps, L, 5, 0, 5, 2, *lay)
    np.testing.assert_array_equal(out, samples.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.accept_counts(), acc)


@pytest.mark.parametrize("dim,elems", [(33, 1), (50, 1), (64, 1), (65, 2), (100, 2), (128, 2)])
@pytest.mark.parametrize("n_chains,offset", [(2, 0), (10, 7), (11, 3), (64, 1)])
def test_hmc_64lane_rosenbrock_bitwise(gm, oracle, dim, elems, n_chains, offset):
    """RosenbrockND f32 at 64 x 1 and 64 x 2 (cfg2's and cfg4's layouts, the
    64-lane gradient form): the oracle's bits for padded dims, even and odd
    chain counts, odd global chain offsets and launches that start mid draw
    block."""
    x0 = start(gm, n_chains, dim, np.float32, 0.8)
    t = gm.RosenbrockND()
    s = gm.HMC(t, x0, 0.02, 9, dtype=np.float32, chain_offset=offset).set_seed(21)
    s.set_layout(64, elems)
    s.set_steps_per_launch(3)
    out = s.run(5, 2)
    q, samples, acc = oracle.hmc_run(Target.from_product(t, dim), x0, 0.02, 9, 21, 0, 7, 2, 64, elems,
                                     chain_offset=offset)
    np.testing.assert_array_equal(out, samples.transpose(1, 0, 2))
    np.testing.assert_array_equal(s.positions(), q)
    np.testing.assert_array_equal(s.accept_counts(), acc)
    s.close()


@pytest.mark.parametrize("dtype", DTYPES)
def test_hmc_sharding_invariance(gm, dtype):
    """Chains keyed by global id: one sampler over 48 chains == two shards."""
    x0 = start(gm, 48, 16, dtype)
    t = gm.RosenbrockND()
    full = gm.HMC(t, x0, 0.02, 5, dtype=dtype).set_seed(5).run(4, 2)
    a = gm.HMC(t, x0[:20], 0.02, 5, dtype=dtype, chain_offset=0).set_seed(5).run(4, 2)
    b = gm.HMC(t, x0[20:], 0.02, 5, dtype=dtype, chain_offset=20).set_seed(5).run(4, 2)
    np.testing.assert_array_equal(full, np.concatenate([a, b], axis=0))


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("dim,lay", [(2, (2, 1)), (5, (8, 1)), (64, (64, 1)), (256, (64, 4)),
                                     (256, (32, 8))])
def test_mh_samples_bitwise(gm, oracle, dtype, dim, lay):
    n_chains = 20
    x0 = start(gm, n_chains, dim, dtype, 1.0)
    for name, t in targets(gm, dim):
        prop = gm.IsotropicGaussian(2.38 / np.sqrt(dim))
        s = gm.MetropolisHastings(t, prop, x0, dtype=dtype).seed(3)
        s.set_layout(*lay)
        s.set_steps_per_launch(5)
        out = s.run(8, 4)
        q, samples, acc = oracle.mh_run(Target.from_product(t, dim), x0, prop.std, 3, 0, 12, 4, *lay)
        np.testing.assert_array_equal(out, samples.transpose(1, 0, 2).astype(np.float64), err_msg=name)
        np.testing.assert_array_equal(s.accept_counts(), acc, err_msg=name)
        s.close()


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("std", [1e-30, 1e-6, 3.0])
def test_mh_exact_quotient_edges_bitwise(gm, oracle, dtype, std):
    """The proposal density's -(d*d)/(2 sd^2) outside the fast quotient's
    proven range takes the IEEE division (mh_device.h, div_by_const_q): sd
    1e-30 gives d = 0 (x + n sd == x) for every coordinate, so every step
    divides -0 (and in f32 sd^2 underflows to 0, so the quotient is NaN);
    1e-6 and 3 are in-range controls. 64 x 4 and 32 x 8 at 256 dimensions,
    as cfg5."""
    dim, n_chains = 256, 12
    x0 = start(gm, n_chains, dim, dtype, 1.0)
    t = gm.IsotropicGaussian(1.0)
    prop = gm.IsotropicGaussian(std)
    for lay in ((64, 4), (32, 8)):
        s = gm.MetropolisHastings(t, prop, x0, dtype=dtype).seed(11)
        s.set_layout(*lay)
        out = s.run(6, 3)
        q, samples, acc = oracle.mh_run(Target.from_product(t, dim), x0, prop.std, 11, 0, 9, 3, *lay)
        np.testing.assert_array_equal(out, samples.transpose(1, 0, 2).astype(np.float64), err_msg=str(lay))
        np.testing.assert_array_equal(s.accept_counts(), acc, err_msg=str(lay))
        s.close()


@pytest.mark.parametrize("dtype,std", [(np.float32, 1e-16), (np.float64, 1e-150)])
@pytest.mark.parametrize("lay", [(32, 1), (16, 2), (8, 4)])
def test_isogauss_target_tiny_std_bitwise(gm, oracle, dtype, std, lay):
    """An IsotropicGaussian target so narrow that the log-density's dividend
    -0.5 sum x^2 falls below the fast quotient's safe range (f32 ~2^-102 <
    2^-100, f64 ~2^-993 < 2^-968; div_by_const_q's per-divisor bound, where
    the remainder a - b q could round in the subnormal range): HMC, NUTS and
    MH equal the oracle's IEEE divisions bit for bit."""
    dim, n_chains = 32, 12
    x0 = (start(gm, n_chains, dim, np.float64, 1.0) * std).astype(dtype)
    t = gm.IsotropicGaussian(std)
    ot = Target.from_product(t, dim)
    h = gm.HMC(t, x0, 0.2 * std, 5, dtype=dtype).set_seed(4)
    h.set_layout(*lay)
    out = h.run(4, 2)
    _, smp, acc = oracle.hmc_run(ot, x0, 0.2 * std, 5, 4, 0, 6, 2, *lay)
    np.testing.assert_array_equal(out, smp.transpose(1, 0, 2))
    np.testing.assert_array_equal(h.accept_counts(), acc)
    assert 0 < acc.sum()
    n = gm.NUTS(t, x0, 0.8, dtype=dtype, max_depth=6).set_seed(5)
    n.set_layout(*lay)
    out = n.run(4, 3)
    st = oracle.nuts_state(n_chains, dtype)
    _, smp, acc, nlf = oracle.nuts_run(ot, x0, st, 0.8, 6, 5, 0, 4, 3, False, *lay)
    np.testing.assert_array_equal(out, smp.transpose(1, 0, 2))
    np.testing.assert_array_equal(n.leapfrog_counts(), nlf)
    eps, _ = n.step_sizes()
    np.testing.assert_array_equal(eps.astype(dtype), st["eps"])
    m = gm.MetropolisHastings(t, gm.IsotropicGaussian(0.7 * std), x0, dtype=dtype).seed(6)
    m.set_layout(*lay)
    out = m.run(5, 2)
    _, smp, acc = oracle.mh_run(ot, x0, 0.7 * std, 6, 0, 7, 2, *lay)
    np.testing.assert_array_equal(out, smp.transpose(1, 0, 2).astype(np.float64))
    np.testing.assert_array_equal(m.accept_counts(), acc)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("dim,lay", [(2, (2, 1)), (5, (8, 1)), (32, (32, 1)), (32, (16, 2))])
@pytest.mark.parametrize("progress", [False, True])
@pytest.mark.parametrize("lds_levels", [-1, 0, 2])  # subtree stack in LDS / HBM / split
def test_nuts_samples_bitwise(gm, oracle, dtype, dim, lay, progress, lds_levels):
    n_chains = 12
    x0 = start(gm, n_chains, dim, dtype, 0.5)
    for name, t in targets(gm, dim):
        if name.startswith("rosen") and dim > 5:
            continue  # deep trees on high-dim Rosenbrock: slow oracle, same code path
        s = gm.NUTS(t, x0, 0.8, dtype=dtype, max_depth=6).set_seed(9)
        s.set_layout(*lay)
        s.set_lds_levels(lds_levels)
        s.set_steps_per_launch(3)
        n_collect, n_discard = 5, 4
        if progress:
            out, _ = s.run_progress(n_collect, n_discard)
        else:
            out = s.run(n_collect, n_discard)
        st = oracle.nuts_state(n_chains, dtype)
        q, samples, acc, nlf = oracle.nuts_run(Target.from_product(t, dim), x0, st, 0.8, 6, 9, 0,
                                               n_collect, n_discard, progress, *lay)
        np.testing.assert_array_equal(out, samples.transpose(1, 0, 2), err_msg=name)
        np.testing.assert_array_equal(s.accept_counts(), acc, err_msg=name)
        np.testing.assert_array_equal(s.leapfrog_counts(), nlf, err_msg=name)
        eps, bar = s.step_sizes()
        np.testing.assert_array_equal(eps.astype(dtype), st["eps"], err_msg=name)
        np.testing.assert_array_equal(bar.astype(dtype), st["eps_bar"], err_msg=name)
        s.close()


def test_nuts_chain_1_kat(gm):
    """test_chain_1 (nuts.rs:588-601): n_collect=1, n_discard=0 -> the start."""
    t = gm.DiffableGaussian2D([0.0, 1.0], [[4.0, 2.0], [2.0, 3.0]])
    c = gm.NUTSChain(t, np.array([0.0, 1.0]), 0.8).set_seed(42)
    np.testing.assert_array_equal(c.run(1, 0), [[0.0, 1.0]])


# h = N/2 <= 64 runs the matrix-core Gram kernel (chain groups, 8-parameter
# tiles: C and P chosen off those multiples), larger h the register-window lag
# kernel (up to 8-parameter blocks, fewer when a long series fills the LDS;
# h > 512 takes further passes over the lags)
@pytest.mark.parametrize("shape", [(4, 100, 3), (7, 41, 2), (64, 300, 5), (3, 1000, 1),
                                   (100, 128, 37), (33, 129, 17), (517, 60, 9), (9, 131, 3),
                                   (5, 1100, 3), (20, 200, 19), (3, 8000, 2), (2, 10400, 1)])
@pytest.mark.parametrize("dtype", DTYPES)
def test_split_rhat_ess_matches_oracle(gm, oracle, shape, dtype):
    rng = np.random.default_rng(sum(shape))
    x = rng.standard_normal(shape)
    x = np.cumsum(x, axis=1) * 0.1 + rng.standard_normal(shape)  # autocorrelated
    x = x.astype(dtype)
    r, e = gm.split_rhat_mean_ess(x)
    orr, oe = oracle.split_rhat_ess(x)
    np.testing.assert_allclose(r, orr, atol=1e-3)  # north-star tolerance: R-hat within 1e-3
    np.testing.assert_allclose(e, oe, rtol=1e-3)



@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("dim,lay", [(32, (16, 2)), (7, (8, 1)), (300, (256, 2))])
def test_nuts_momentum_pass_forms_bitwise(gm, oracle, dtype, dim, lay):
    """The transition momenta drawn in one parallel pass per launch (the
    default, nuts_momenta_kernel) or inside the tree kernel: the oracle's bits
    either way, across launches of a run (steps_per_launch) and a second run."""
    n_chains = 10
    x0 = start(gm, n_chains, dim, dtype, 0.5)
    t = gm.IsotropicGaussian(1.2)
    outs = []
    for on in (True, False):
        s = gm.NUTS(t, x0, 0.8, dtype=dtype, max_depth=6).set_seed(21)
        s.set_layout(*lay)
        s.set_momentum_pass(on)
        s.set_steps_per_launch(4)
        outs.append((s.run(5, 6), s.run(3, 0)))
    st = oracle.nuts_state(n_chains, dtype)
    q, s1, _, _ = oracle.nuts_run(Target.from_product(t, dim), x0, st, 0.8, 6, 21, 0, 5, 6, False, *lay)
    _, s2, _, _ = oracle.nuts_run(Target.from_product(t, dim), q, st, 0.8, 6, 21, 11, 3, 0, False, *lay)
    for a, b in outs:
        np.testing.assert_array_equal(a, s1.transpose(1, 0, 2))
        np.testing.assert_array_equal(b, s2.transpose(1, 0, 2))
