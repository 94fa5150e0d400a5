#!/bin/bash
source tools/gpu_check.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -m pytest tests -m gpu -q --maxfail=10 -p no:cacheprovider || exit 1
run sweep 300 python tools/sweep_hmc.py --layouts 64x1,32x2,16x4 --rounds 5
cat gpurun_out/sweep.log >&2
run configs 900 python tools/bench_configs.py --which 4,5,3
cat gpurun_out/configs.log >&2
run bench 300 python bench.py --cpu-seconds 10
