#!/bin/bash
# One GPU call: MH parity tests on the working-tree library, then an
# alternating-process A/B of cfg5 against abtest/base (tools/ab_mh.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_edge.py tests/test_gpu_tracker.py tests/test_gpu_custom.py -x -q -k "mh or MH or cfg5 or Metropolis or tracker or custom" --timeout 120 --timeout-method thread > gpurun_out/ab_mh_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_mh_tests.log; [ $rc -ne 0 ] && exit $rc
AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 600 python tools/ab_mh.py abtest/base/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so ${AB_EXTRA} > gpurun_out/ab_mh.log 2>&1
rc=$?; tail -12 gpurun_out/ab_mh.log; exit $rc
