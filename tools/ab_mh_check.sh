#!/bin/bash
# One GPU call: MH parity and statistical tests on the working-tree library,
# then an alternating-process A/B of cfg5 against ${AB_BASE:-abtest/cur}
# (tools/ab_mh.py; extra variants in AB_EXTRA).
source tools/gpu_check.sh
run mh_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_edge.py tests/test_gpu_tracker.py tests/test_gpu_custom.py tests/test_gpu_mfma_gauss.py tests/test_gpu_statistical.py tests/test_gpu_checkpoint.py -x -q -k "mh or MH or cfg5 or Metropolis or tracker or custom" --timeout 120 --timeout-method thread || exit $?
AB_ROUNDS=${AB_ROUNDS:-4} run ab_mh 600 python tools/ab_mh.py ${AB_BASE:-abtest/cur/libgmcmc.so} general-mcmc_amd/lib/libgmcmc.so ${AB_EXTRA} || exit $?
tail -16 gpurun_out/ab_mh.log
