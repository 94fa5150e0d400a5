#!/bin/bash
# One GPU call: dense-metric NUTS parity tests on the working-tree library,
# then an alternating-process A/B of cfg3 with dense adaptation against
# abtest/base (tools/ab_nuts.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
[ -x tools/probes/bin/row_share_probe ] && timeout -k 5 30 tools/probes/bin/row_share_probe > gpurun_out/row_share_probe.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_nuts_mass.py tests/test_gpu_mfma_gauss.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_dense_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_dense_tests.log; [ $rc -ne 0 ] && exit $rc
AB_ARGS="--nuts-mass dense" AB_ROUNDS=${AB_ROUNDS:-2} timeout -k 10 600 python tools/ab_nuts.py abtest/base/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so > gpurun_out/ab_dense.log 2>&1
rc=$?; tail -12 gpurun_out/ab_dense.log; [ $rc -ne 0 ] && exit $rc
for v in ${AB_MINV:-1 2 1 2}; do
  GMCMC_NUTS_DEBUG=1 GMCMC_NUTS_MINV_LDS=$v timeout -k 10 200 python tools/bench_configs.py --which 3 --nuts-mass dense > gpurun_out/dense_minv$v.log 2>&1 || exit $?
  echo "minv_lds=$v $(grep -o 'M^-1 in LDS [0-9]* at [0-9]*, L [01] at [0-9]*' gpurun_out/dense_minv$v.log | tail -1) $(grep -o 'stack levels in LDS [0-9]*' gpurun_out/dense_minv$v.log | tail -1) $(grep -o '"leapfrog_per_s": [0-9.e+]*' gpurun_out/dense_minv$v.log)"
done
