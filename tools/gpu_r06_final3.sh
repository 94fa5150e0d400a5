#!/bin/bash
# Round-6 final call (after the dense pre-pass): the tree's GPU suite and smoke, its bench lines (the
# driver's default command and --steps 20 --warmup 5, twice), the NUTS
# of the bench command (tools/profile_r06.sh).
source tools/gpu_check.sh
run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench_default 400 python bench.py || exit $?
grep '^{' gpurun_out/bench_default.log | tail -n 1 > gpurun_out/bench_default_line.json
for r in 1 2; do
  run bench20 400 python bench.py --steps 20 --warmup 5 || exit $?
  grep '^{' gpurun_out/bench20.log | tail -n 1 >> gpurun_out/bench20_lines.jsonl
done
PMC_OUT=gpurun_out/pmc_r06c K=20 bash tools/profile_r06.sh
