#!/bin/bash
# Round-6 call E: validation of the tree (GPU suite, smoke) and its bench line
# (default command and the driver's --steps 20 --warmup 5).
source tools/gpu_check.sh
run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench20 400 python bench.py --steps 20 --warmup 5 || exit $?
grep '^{' gpurun_out/bench20.log | tail -1 > gpurun_out/bench20_line.json
