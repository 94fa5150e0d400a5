source tools/gpu_check.sh
run mh_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_edge.py tests/test_gpu_tracker.py tests/test_gpu_custom.py tests/test_gpu_mfma_gauss.py -x -q -k "mh or MH or cfg5 or Metropolis or tracker or custom" --timeout 120 --timeout-method thread || exit $?
AB_ROUNDS=4 run ab_mh 600 python tools/ab_mh.py abtest/cur/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so || exit $?
tail -12 gpurun_out/ab_mh.log
