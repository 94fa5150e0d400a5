#!/bin/bash
# One GPU call: NUTS/MFMA parity tests on the working-tree library, then an
# alternating-process A/B of cfg3 against abtest/base (tools/ab_nuts.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma_gauss.py tests/test_gpu_parity.py tests/test_gpu_nuts_truncation.py tests/test_gpu_nuts_mass.py tests/test_gpu_fullsize_edge.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 600 python tools/ab_nuts.py ${AB_BASE:-abtest/base/libgmcmc.so} general-mcmc_amd/lib/libgmcmc.so ${AB_EXTRA} > gpurun_out/ab_nuts.log 2>&1
rc=$?; tail -12 gpurun_out/ab_nuts.log; exit $rc
