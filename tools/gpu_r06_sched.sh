#!/bin/bash
# Round-6 A/B: compiler scheduling variants of the whole library (same bits;
# tools/ab_variants.sh): ilp (-mllvm -amdgpu-sched-strategy=gcn-max-ilp) and
# prio (-mllvm -amdgpu-set-wave-priority) against the tree, on the headline
# HMC launch, NUTS cfg3 (identity and dense metric) and MH cfg5.
source tools/gpu_check.sh
L=general-mcmc_amd/lib/libgmcmc.so
V="abrun/ilp/libgmcmc.so abrun/prio/libgmcmc.so"
AB_ROUNDS=3 AB_ARGS="--layouts 64x1 --rounds 3 --steps 20" run ab_sched_hmc 400 python tools/ab_run.py $L $V || exit $?
AB_ROUNDS=2 run ab_sched_nuts 400 python tools/ab_nuts.py $L $V || exit $?
AB_ROUNDS=2 AB_ARGS="--nuts-mass dense" run ab_sched_dense 500 python tools/ab_nuts.py $L $V || exit $?
AB_ROUNDS=2 run ab_sched_mh 400 python tools/ab_mh.py $L $V || exit $?
tail -n 12 gpurun_out/ab_sched_*.log
