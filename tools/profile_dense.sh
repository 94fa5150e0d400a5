#!/bin/bash
# rocprofv3 passes over the dense-metric NUTS run (cfg3 with dense mass-matrix
# adaptation, tools/bench_configs.py --which 3 --nuts-mass dense): kernel trace
# + stats, SQ instruction mix, GRBM busy cycles -- each in its own run.
# Output under gpurun_out/prof_r03_dense; summary by tools/pmc_dispatch.py.
source tools/gpu_check.sh
O=gpurun_out/prof_r03_dense
CMD="python3 tools/bench_configs.py --which 3 --nuts-mass dense"
run profd_trace 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $CMD &&
run profd_fetch 300 timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $CMD &&
run profd_write 300 timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $CMD &&
run profd_sq 300 timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $O/sq -o run --output-format csv -- $CMD &&
run profd_grbm 300 timeout -s KILL 280 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/grbm -o run --output-format csv -- $CMD &&
python3 tools/pmc_dispatch.py $O --kernel nuts_kernel --grid 131072 --ordinal -1 --key cfg3_dense_C8192_D32_f64 --steps 500 --out profiles/r03/pmc_configs.json >&2
