#!/bin/bash
# rocprofv3 passes over the driver's bench command (GPU box): kernel trace +
# stats, FETCH_SIZE, WRITE_SIZE, SQ instruction mix (VALU and SALU), GRBM busy
# cycles -- each in its own run (PMC never beside runtime tracing; counter
# blocks within one pass stay inside their slot limits). The bench command
# includes the config legs (cfg3 NUTS, cfg4 HMC, cfg5 MH), so one set of
# passes covers every kernel; tools/pmc_dispatch.py picks each dispatch by
# kernel name and grid. Output under gpurun_out/prof_r03_K$K.
#   K=20 bash tools/profile_r03.sh
source tools/gpu_check.sh
K=${K:-20}
W=${W:-5}
O=gpurun_out/prof_r03_K$K
ARGS="--steps $K --warmup $W --cpu-seconds 0 --ess-long-discard 0 --no-north-star"
run prof_trace_$K 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_fetch_$K 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_write_$K 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_sq_$K 300 timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $O/sq -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_grbm_$K 300 timeout -s KILL 280 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/grbm -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_flops_$K 300 timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 -d $O/flops -o run --output-format csv -- python3 bench.py $ARGS &&
P=profiles/r03 &&
python3 tools/pmc_dispatch.py $O --kernel hmc_kernel --grid 262144 --ordinal -4 --key C4096_D64_L50_f32 --steps $K --out $P/pmc_hmc.json >&2 &&
python3 tools/pmc_dispatch.py $O --kernel hmc_kernel --grid 524288 --ordinal 0 --key cfg4_C8192_D128_L50_f32 --steps 200 --out $P/pmc_configs.json >&2 &&
python3 tools/pmc_dispatch.py $O --kernel nuts_kernel --grid 131072 --ordinal -1 --key cfg3_C8192_D32_f64 --steps 999 --out $P/pmc_configs.json >&2 &&
python3 tools/pmc_dispatch.py $O --kernel mh_kernel --grid 1048576 --ordinal 0 --key cfg5_C16384_D256_f64 --steps 1000 --out $P/pmc_configs.json >&2
