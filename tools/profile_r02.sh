#!/bin/bash
# rocprofv3 passes over the driver's bench command at K transitions (GPU box):
# kernel trace + stats, FETCH_SIZE, WRITE_SIZE, SQ instruction mix, GRBM busy
# cycles, VALU FLOPS -- each in its own run (PMC never beside runtime tracing; counter
# blocks within one pass stay inside their slot limits). Output under
# gpurun_out/prof_r02_K$K; tools/pmc_hmc.py turns it into profiles/r02/pmc_hmc.json.
#   K=20 bash tools/profile_r02.sh
source tools/gpu_check.sh
K=${K:-20}
W=${W:-5}
O=gpurun_out/prof_r02_K$K
ARGS="--steps $K --warmup $W --cpu-seconds 0 --ess-long-discard 0"
run prof_trace_$K 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_fetch_$K 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_write_$K 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_sq_$K 300 timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $O/sq -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_grbm_$K 300 timeout -s KILL 280 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/grbm -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_flops_$K 300 timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 -d $O/flops -o run --output-format csv -- python3 bench.py $ARGS &&
python3 tools/pmc_hmc.py $O --steps $K >&2
