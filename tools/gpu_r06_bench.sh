#!/bin/bash
# Round-6: bench lines of the current tree (the driver's default command and
# --steps 20 --warmup 5, twice) and the smoke.
source tools/gpu_check.sh
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench_default 400 python bench.py || exit $?
grep '^{' gpurun_out/bench_default.log | tail -n 1 > gpurun_out/bench_default_line.json
for r in 1 2; do
  run bench20 400 python bench.py --steps 20 --warmup 5 || exit $?
  grep '^{' gpurun_out/bench20.log | tail -n 1 >> gpurun_out/bench20_lines.jsonl
done
