source tools/gpu_check.sh
#run mh_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_edge.py tests/test_gpu_tracker.py tests/test_gpu_custom.py tests/test_gpu_mfma_gauss.py tests/test_gpu_statistical.py tests/test_gpu_checkpoint.py -x -q -k "mh or MH or cfg5 or Metropolis or tracker or custom" --timeout 120 --timeout-method thread || exit $?
#run nuts_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mfma_gauss.py tests/test_gpu_nuts_truncation.py tests/test_gpu_nuts_mass.py tests/test_gpu_fullsize_edge.py tests/test_gpu_checkpoint.py tests/test_gpu_step.py tests/test_gpu_nuts_wide.py -x -q -k "nuts or NUTS or cfg3 or mfma" --timeout 120 --timeout-method thread || exit $?
run edge_tests 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tiny_std or exact_quotient" --timeout 120 --timeout-method thread || exit $?
run forms_tests 400 python -u -m pytest tests/test_gpu_forms.py -x -v -s --timeout 200 --timeout-method thread || exit $?
AB_ROUNDS=3 run ab_mh 400 python tools/ab_mh.py abtest/mh_f0/libgmcmc.so abtest/mh_f1/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so || exit $?
AB_ROUNDS=3 run ab_nuts 300 python tools/ab_nuts.py abtest/nuts_u0/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so || exit $?
AB_ARGS="--nuts-mass dense" AB_ROUNDS=2 run ab_dense 300 python tools/ab_nuts.py abtest/nuts_u0/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so || exit $?
tail -n 8 gpurun_out/ab_mh.log gpurun_out/ab_nuts.log gpurun_out/ab_dense.log
