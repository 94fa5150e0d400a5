#!/bin/bash
# rocprofv3 passes over the driver's bench command (GPU box): kernel trace +
# stats, FETCH_SIZE, WRITE_SIZE, SQ instruction mix (VALU, SALU, LDS), GRBM
# busy cycles and the FLOPS counters -- each in its own run (PMC never beside
# runtime tracing; counter blocks within one pass stay inside their slot
# limits). The bench command includes the config legs (cfg3 NUTS identity
# and dense metric, cfg4 HMC, cfg5 MH), so one set of passes covers every
# kernel the bench line reports (round 5+: the cfg3_dense sampling launch is
# the frozen-dense kernel, MASS 3); tools/pmc_dispatch.py picks each dispatch by
# kernel name and grid into profiles/r06/pmc_hmc.json (the headline's
# `traffic` and `valu_issue`) and profiles/r06/pmc_configs.json (each leg's).
#   K=20 bash tools/profile_r06.sh
source tools/gpu_check.sh
K=${K:-20}
W=${W:-5}
O=gpurun_out/prof_r06_K$K
ARGS="--steps $K --warmup $W --cpu-seconds 0 --cpu-config-seconds 0 --ess-long-discard 0 --no-north-star"
run prof_trace_$K 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_fetch_$K 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_write_$K 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_sq_$K 300 timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/sq -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_grbm_$K 300 timeout -s KILL 280 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/grbm -o run --output-format csv -- python3 bench.py $ARGS &&
run prof_flops_$K 300 timeout -s KILL 280 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 -d $O/flops -o run --output-format csv -- python3 bench.py $ARGS &&
P=${PMC_OUT:-profiles/r06} && mkdir -p $P &&
python3 tools/pmc_dispatch.py $O --kernel hmc_kernel --grid 262144 --ordinal -4 --key C4096_D64_L50_f32 --steps $K --out $P/pmc_hmc.json >&2 &&
python3 tools/pmc_dispatch.py $O --kernel hmc_kernel --grid 524288 --ordinal -1 --key cfg4 --steps 200 --out $P/pmc_configs.json >&2 &&
python3 tools/pmc_dispatch.py $O --kernel "GaussT<double>, 0>" --grid 131072 --ordinal -1 --key cfg3 --steps 499 --out $P/pmc_configs.json >&2 &&
python3 tools/pmc_dispatch.py $O --kernel "GaussT<double>, 3>" --grid 131072 --ordinal -1 --key cfg3_dense --steps 499 --out $P/pmc_configs.json >&2 &&
python3 tools/pmc_dispatch.py $O --kernel mh_kernel --grid 1048576 --ordinal -2 --key cfg5 --steps 1000 --out $P/pmc_configs.json >&2 &&
cp $O/trace/*kernel_stats.csv $P/kernel_stats_K$K.csv 2>/dev/null; ls $O/trace >&2
