#!/bin/bash
# rocprofv3 passes (trace, FETCH_SIZE, WRITE_SIZE, SQ mix, GRBM) of the cfg3
# dense-metric leg (tools/bench_configs.py --which 3 --nuts-mass dense) for
# each library given as NAME=PATH, one run per pass; tools/pmc_dispatch.py
# reduces the frozen-dense sampling launch of each into $OUT (key NAME).
#   bash tools/profile_dense_prep.sh tree=general-mcmc_amd/lib/libgmcmc.so noprep=abrun/noprep/libgmcmc.so
source tools/gpu_check.sh
OUT=${OUT:-gpurun_out/pmc_dense_prep.json}
ARGS="tools/bench_configs.py --which 3 --nuts-mass dense"
for nl in "$@"; do
  n=${nl%%=*}; l=$(pwd)/${nl#*=}
  O=gpurun_out/dprep_$n
  export GMCMC_LIB=$l
  run dp_trace_$n 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $ARGS &&
  run dp_fetch_$n 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $ARGS &&
  run dp_write_$n 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $ARGS &&
  run dp_sq_$n 300 timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/sq -o run --output-format csv -- python3 $ARGS &&
  run dp_grbm_$n 300 timeout -s KILL 280 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/grbm -o run --output-format csv -- python3 $ARGS &&
  python3 tools/pmc_dispatch.py $O --kernel "GaussT<double>, 3>" --grid 131072 --ordinal -1 --key $n --steps 499 --out $OUT >&2 || exit $?
  unset GMCMC_LIB
done
