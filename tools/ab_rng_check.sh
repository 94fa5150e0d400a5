#!/bin/bash
# One GPU call: the whole GPU suite on the working tree, then A/B of the MH
# (cfg5) and HMC (cfg2 shape) kernels against variants built from another
# source tree (abtest/v3mh, abtest/v3hmc: tools/ab_build_unit.sh).
source tools/gpu_check.sh
run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
AB_ROUNDS=3 run ab_mh 600 python tools/ab_mh.py abtest/v3mh/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so || exit $?
AB_ROUNDS=3 AB_ARGS="--layouts 64x1 --rounds 3 --steps 20" run ab_hmc 600 python tools/ab_run.py abtest/v3hmc/libgmcmc.so general-mcmc_amd/lib/libgmcmc.so || exit $?
tail -12 gpurun_out/ab_mh.log; tail -12 gpurun_out/ab_hmc.log
