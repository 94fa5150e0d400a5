#!/bin/bash
# Round-6 call I: MH without a run_progress tracker takes a TRACK = false
# instantiation; at 64 x 4 f64 its draws go in two halves and the kernel
# fits 5 waves per SIMD (93 VGPRs). MH GPU tests, then cfg5 A/B of the
# previous tree (abrun/prev), the tree, and the tree without the halves / 5-wave
# bound (abrun/mh_nohalves: the tracker-free instantiation alone, 4 waves);
# the dense NUTS leg of the tree (start-record pass skipped for frozen-dense
# launches) against prev.
source tools/gpu_check.sh
L=general-mcmc_amd/lib/libgmcmc.so
run mh_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_edge.py tests/test_gpu_tracker.py tests/test_gpu_custom.py tests/test_gpu_checkpoint.py tests/test_gpu_statistical.py tests/test_gpu_forms.py -x -q -k "mh or MH or cfg5 or Metropolis or tracker or custom" --timeout 200 --timeout-method thread || exit $?
run nuts_mass_tests 300 python -u -m pytest tests/test_gpu_nuts_mass.py -x -q --timeout 200 --timeout-method thread || exit $?
AB_ROUNDS=3 run ab_mh 400 python tools/ab_mh.py abrun/prev/libgmcmc.so $L abrun/mh_nohalves/libgmcmc.so || exit $?
AB_ARGS="--nuts-mass dense" AB_ROUNDS=2 run ab_dense 450 python tools/ab_nuts.py abrun/prev/libgmcmc.so $L || exit $?
tail -n 14 gpurun_out/ab_mh.log
