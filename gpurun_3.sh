#!/bin/bash
source tools/gpu_check.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -m pytest tests -m gpu -q --maxfail=10 -p no:cacheprovider || exit 1
run sweep 300 python tools/sweep_hmc.py --layouts 64x1,32x2,16x4 --rounds 5
cat gpurun_out/sweep.log >&2
run sweep_big 300 python tools/sweep_hmc.py --chains 65536 --layouts 64x1,32x2,16x4,16x8 --rounds 3 --steps 20
cat gpurun_out/sweep_big.log >&2
run bench 300 python bench.py --cpu-seconds 10
run prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python bench.py --cpu-seconds 0
run prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python bench.py --cpu-seconds 0
run prof_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python bench.py --cpu-seconds 0
find gpurun_out -name "*.csv" | head -20 >&2
