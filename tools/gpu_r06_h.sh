#!/bin/bash
# Round-6 call H: NUTS -- the level-0 merge's U-turn dots reduced with the
# leaf's sums (GM_NUTS_L0UT) and the merge uniforms by a Weyl walk
# (GM_NUTS_WEYL): NUTS GPU tests (bitwise vs the unchanged oracle), cfg3 A/B of
# the previous tree (abrun/prev), both (the tree), each alone (abrun/l0ut0 =
# Weyl only, abrun/weyl0 = L0UT only); dense A/B; an LDS-counter pass of cfg3.
source tools/gpu_check.sh
L=general-mcmc_amd/lib/libgmcmc.so
run nuts_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mfma_gauss.py tests/test_gpu_nuts_truncation.py tests/test_gpu_nuts_mass.py tests/test_gpu_fullsize_edge.py tests/test_gpu_checkpoint.py tests/test_gpu_step.py tests/test_gpu_nuts_wide.py -x -q -k "nuts or NUTS or cfg3 or mfma" --timeout 120 --timeout-method thread || exit $?
AB_ROUNDS=3 run ab_nuts 500 python tools/ab_nuts.py abrun/prev/libgmcmc.so $L abrun/l0ut0/libgmcmc.so abrun/weyl0/libgmcmc.so || exit $?
AB_ARGS="--nuts-mass dense" AB_ROUNDS=2 run ab_dense 450 python tools/ab_nuts.py abrun/prev/libgmcmc.so $L || exit $?
run lds_pmc 90 timeout -s KILL 80 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT -d gpurun_out/lds_pmc -o run --output-format csv -- python3 tools/bench_configs.py --which 3 || true
tail -n 14 gpurun_out/ab_nuts.log
