#!/bin/bash
# One GPU call: dense-metric NUTS tests on the working-tree library and on the
# pipelined-product variants (GMCMC_LIB), then an alternating-process A/B of
# cfg3 with dense adaptation (tools/ab_nuts.py) against abtest/base.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for L in general-mcmc_amd/lib/libgmcmc.so ${AB_VARIANTS}; do
  GMCMC_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_nuts_mass.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_dense_tests.log 2>&1
  rc=$?; echo "$L: $(tail -1 gpurun_out/ab_dense_tests.log)"; [ $rc -ne 0 ] && exit $rc
done
AB_ARGS="--nuts-mass dense" AB_ROUNDS=${AB_ROUNDS:-2} timeout -k 10 700 python tools/ab_nuts.py abtest/base/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so ${AB_VARIANTS} > gpurun_out/ab_chol.log 2>&1
rc=$?; tail -24 gpurun_out/ab_chol.log; exit $rc
