#!/bin/bash
# Round-6 A/B call 1 (libraries under abrun/, each a whole libgmcmc.so):
#   MH f64 draw forms: mh_f0 (per-coordinate draws), mh_f1 (one basic block),
#     the tree's form 2 (draw_blocks_v / normals_tab_n);
#   NUTS cfg3 identity: nuts_u0 (per-chain climb) vs the tree (wave-uniform)
#     and the stack-slab builds pf0 / pf1 / pf2 (touch-prefetch depth);
#   NUTS cfg3 dense metric: the tree vs pf0 / pf1 / pf2.
source tools/gpu_check.sh
L=general-mcmc_amd/lib/libgmcmc.so
AB_ROUNDS=3 run ab_mh 300 python tools/ab_mh.py abrun/mh_f0/libgmcmc.so abrun/mh_f1/libgmcmc.so $L || exit $?
AB_ROUNDS=3 run ab_nuts 400 python tools/ab_nuts.py abrun/nuts_u0/libgmcmc.so $L abrun/pf0/libgmcmc.so \
  abrun/pf1/libgmcmc.so abrun/pf2/libgmcmc.so || exit $?
AB_ARGS="--nuts-mass dense" AB_ROUNDS=2 run ab_dense 450 python tools/ab_nuts.py $L abrun/pf0/libgmcmc.so \
  abrun/pf1/libgmcmc.so abrun/pf2/libgmcmc.so || exit $?
run forms_tests 300 python -u -m pytest tests/test_gpu_forms.py -x -v -s --timeout 200 --timeout-method thread || exit $?
tail -n 6 gpurun_out/ab_mh.log gpurun_out/ab_nuts.log gpurun_out/ab_dense.log
