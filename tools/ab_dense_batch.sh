cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
AB_ARGS="--nuts-mass dense" AB_ROUNDS=2 timeout -k 10 600 python tools/ab_nuts.py abtest/nb8/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so abtest/nb32/libgmcmc.so > gpurun_out/ab_nb.log 2>&1
rc=$?; tail -16 gpurun_out/ab_nb.log; exit $rc
