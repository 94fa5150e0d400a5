#!/bin/bash
# Round-6 call B: the NUTS leaf's division-free exp (leaf_alpha_tab) --
# the GPU suite on the new tree, then cfg3 identity and dense A/Bs of the
# previous tree (abrun/base), the new tree and its pinned-constant variant.
source tools/gpu_check.sh
L=general-mcmc_amd/lib/libgmcmc.so
run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
AB_ROUNDS=3 run ab_nuts 400 python tools/ab_nuts.py abrun/base/libgmcmc.so $L abrun/lexp_pin1/libgmcmc.so || exit $?
AB_ARGS="--nuts-mass dense" AB_ROUNDS=2 run ab_dense 450 python tools/ab_nuts.py abrun/base/libgmcmc.so $L \
  abrun/lexp_pin1/libgmcmc.so || exit $?
tail -n 12 gpurun_out/ab_nuts.log gpurun_out/ab_dense.log
