#!/bin/bash
# Round-6 call C: MH with the symmetric proposal's log q terms cancelled
# (mh_device.h `cancel`) -- the GPU suite (parity, forms ties) on the new
# tree, then the cfg5 A/B of the previous tree (abrun/base) and the new one.
source tools/gpu_check.sh
L=general-mcmc_amd/lib/libgmcmc.so
run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
run forms_tests 400 python -u -m pytest tests/test_gpu_forms.py -x -v -s --timeout 300 --timeout-method thread || exit $?
AB_ROUNDS=3 run ab_mh 400 python tools/ab_mh.py abrun/base/libgmcmc.so $L || exit $?
tail -n 12 gpurun_out/ab_mh.log
