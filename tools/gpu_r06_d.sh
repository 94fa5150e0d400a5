#!/bin/bash
# Round-6 call D: NUTS start records from the momentum pre-pass
# (nuts_starts_kernel) -- the GPU suite on the new tree, cfg3 identity and
# dense A/Bs of the previous tree (abrun/prev: leaf exp + MH cancel), the new
# tree, and the new tree without the records in the frozen-dense kernel
# (abrun/srec_d0); the host-path probe of the bench's timed call; MH with
# the steps of a normal pair taken in turn (no per-step select), against prev.
source tools/gpu_check.sh
L=general-mcmc_amd/lib/libgmcmc.so
run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
AB_ROUNDS=3 run ab_nuts 400 python tools/ab_nuts.py abrun/prev/libgmcmc.so $L || exit $?
AB_ARGS="--nuts-mass dense" AB_ROUNDS=2 run ab_dense 450 python tools/ab_nuts.py abrun/prev/libgmcmc.so $L \
  abrun/srec_d0/libgmcmc.so || exit $?
run host_path 120 python tools/probe_host_path.py || exit $?
tail -n 12 gpurun_out/ab_nuts.log gpurun_out/ab_dense.log
AB_ROUNDS=3 run ab_mh 400 python tools/ab_mh.py abrun/prev/libgmcmc.so $L || exit $?
tail -n 12 gpurun_out/ab_mh.log
