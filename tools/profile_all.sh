#!/bin/bash
# All rocprofv3 captures of the default bench.py run, each its own pass:
# kernel trace + stats, FETCH_SIZE, WRITE_SIZE, two SQ instruction-mix
# passes and GRBM_GUI_ACTIVE. Outputs under gpurun_out/prof_$TAG; summarise
# with tools/pmc_traffic.py and tools/pmc_valu.py (on the dev box).
# Usage (GPU box): TAG=r01d bash tools/profile_all.sh
source tools/gpu_check.sh
export TMPDIR=/tmp
O=gpurun_out/prof_${TAG:-r01}
B="python3 bench.py --cpu-seconds 0"
run prof_trace 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B &&
run prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B &&
run prof_write 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B &&
run pmc_sq_a 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmca -o run --output-format csv -- $B &&
run pmc_sq_b 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $O/pmcb -o run --output-format csv -- $B &&
run pmc_grbm 300 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/grbm -o run --output-format csv -- $B &&
run bench 300 python3 bench.py
