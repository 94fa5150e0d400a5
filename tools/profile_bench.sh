#!/bin/bash
# rocprofv3 passes over the default bench.py run (on the GPU box):
#   1. kernel trace + stats;  2. FETCH_SIZE;  3. WRITE_SIZE
# (separate PMC passes: the two TCC counters do not fit one pass, and PMC is
# never combined with runtime/sys tracing). Outputs under gpurun_out/prof_$TAG.
# Usage: TAG=r01b bash tools/profile_bench.sh [extra bench.py args]
source tools/gpu_check.sh
OUT=gpurun_out/prof_${TAG:-r01}
ARGS="--cpu-seconds 0 $*"
run prof_trace 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_fetch 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_write 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS &&
python3 tools/pmc_traffic.py $OUT >&2
