"""Locate the first GPU/oracle divergence of NUTS mass warm-up: fresh
samplers, run(1, nd) for increasing nd, compare state."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402
from tests import _oracle  # noqa: E402
from tests._oracle import Target  # noqa: E402

o = _oracle.load()
dtype = np.float64
cov = np.diag([0.04, 1.0, 4.0, 0.5])
t = gm.DenseGaussian(np.zeros(4), cov)
x0 = gm.init_with_seed(24, 4, 3, dtype)
cfg = dict(start_buffer=5, end_buffer=5, initial_window=10)
MODE = int(os.environ.get("MODE", "1"))
for nd in [1, 2, 3, 4, 5, 10]:
    s = gm.NUTS.new_with_mass_matrix(t, x0, 0.8, gm.NUTSMassMatrixConfig(["none", "diagonal"][MODE], **cfg),
                                     dtype=dtype).set_seed(11)
    lanes, elems = s.layout()
    s.run(1, nd)
    st = o.nuts_state(24, dtype)
    om = o.nuts_mass(MODE, 24, 4, dtype, **cfg)
    q, smp, _, _ = o.nuts_mass_run(Target.from_product(t, 4), x0, st, om, 0.8, 10, 11, 0, 1, nd, False, lanes, elems)
    pos = s.positions()
    eps, bar = s.step_sizes()
    m = s.mass_matrix()
    bad_pos = np.where(np.any(pos != q, axis=1))[0]
    bad_eps = np.where(eps != st["eps"])[0]
    bad_bar = np.where(bar != st["eps_bar"])[0]
    bad_kind = np.where(m.kind != om.kind)[0]
    bad_inv = np.where(np.any(m.diag_inv != om.dinv, axis=1))[0] if MODE else []
    st2 = o.nuts_state(24, dtype)
    _ = o.nuts_run(Target.from_product(t, 4), x0, st2, 0.8, 10, 11, 0, 1, nd, False, lanes, elems)
    print("   plain-oracle vs mass-oracle eps equal:", np.array_equal(st2["eps"], st["eps"]))
    print(f"nd={nd:3d} pos {list(bad_pos)[:8]} eps {list(bad_eps)[:8]} bar {list(bad_bar)[:8]} "
          f"kind {list(bad_kind)[:8]} inv {list(bad_inv)[:8]}", flush=True)
    if len(bad_eps):
        c = bad_eps[0]
        print("   chain", c, "gpu eps", eps[c], "oracle", st["eps"][c], "gpu inv", m.diag_inv[c],
              "oracle inv", om.dinv[c], "kinds", m.kind[c], om.kind[c], flush=True)
