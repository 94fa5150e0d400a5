#!/bin/bash
# Round-6 call F: iteration profiles (measurement build abrun/nprof) and the
# rocprofv3 passes of the bench command over the current tree.
source tools/gpu_check.sh
run nprof_cfg3 120 env GMCMC_LIB=abrun/nprof/libgmcmc.so python tools/probe_nuts_prof.py || exit $?
run nprof_dense 200 env MASS=dense GMCMC_LIB=abrun/nprof/libgmcmc.so python tools/probe_nuts_prof.py || exit $?
PMC_OUT=gpurun_out/pmc_r06 K=20 bash tools/profile_r06.sh
