"""HMC transitions without leapfrogs (L = 0) and with L = 50, 4096 x 64 f32:
a fixed workload for PMC counter passes (rocprofv3 --pmc ...)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import general_mcmc_amd as gm  # noqa: E402

for L in (0, 50):
    s = gm.HMC(gm.RosenbrockND(), gm.init_with_seed(4096, 64, 42, np.float32), 0.01, L).set_seed(1)
    s.run_positions(0, 4)
    s.run_positions(200, 0)
    print(L, s.last_run_stats())
