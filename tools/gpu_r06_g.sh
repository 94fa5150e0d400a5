#!/bin/bash
# Round-6 call G: NUTS change vs the previous tree (abrun/prev) -- NUTS GPU tests,
# then cfg3 and dense A/B (latest: the doublings' top-level uniforms from the
# pre-pass, each loaded at the previous doubling's end).

source tools/gpu_check.sh
L=general-mcmc_amd/lib/libgmcmc.so
run nuts_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mfma_gauss.py tests/test_gpu_nuts_truncation.py tests/test_gpu_nuts_mass.py tests/test_gpu_fullsize_edge.py tests/test_gpu_checkpoint.py tests/test_gpu_step.py tests/test_gpu_nuts_wide.py -x -q -k "nuts or NUTS or cfg3 or mfma" --timeout 120 --timeout-method thread || exit $?
AB_ROUNDS=3 run ab_nuts 400 python tools/ab_nuts.py abrun/prev/libgmcmc.so $L || exit $?
AB_ARGS="--nuts-mass dense" AB_ROUNDS=2 run ab_dense 450 python tools/ab_nuts.py abrun/prev/libgmcmc.so $L || exit $?
tail -n 10 gpurun_out/ab_nuts.log gpurun_out/ab_dense.log
