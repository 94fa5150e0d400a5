#!/bin/bash
source tools/gpu_check.sh
export TMPDIR=/tmp
run pytest_gpu 1200 python -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider
run bench 300 python bench.py --cpu-seconds 5
