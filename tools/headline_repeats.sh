#!/bin/bash
# The driver's bench command (--steps 20 --warmup 5) repeated in fresh
# processes on one box, CPU-baseline and ESS legs off, to state the
# headline's process-to-process spread: gpurun_out/headline_repeats.jsonl.
source tools/gpu_check.sh
N=${N:-8}
rm -f gpurun_out/headline_repeats.jsonl
for r in $(seq 1 $N); do
  run headline_rep 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --cpu-config-seconds 0 --ess-long-discard 0 --no-north-star || exit $?
  grep '^{' gpurun_out/headline_rep.log | tail -n 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'value': d['value'], 'kernel_ms': d['timing']['kernel_ms'], 'wall_ms': d['timing']['wall_ms'],
                  'host_overhead_ms': d['timing']['host_overhead_ms'], 'frac': d['roofline']['frac'],
                  'cfg3': d['configs']['cfg3']['value'], 'cfg3_dense': d['configs']['cfg3_dense']['value'],
                  'cfg4': d['configs']['cfg4']['value'], 'cfg5': d['configs']['cfg5']['value']}))" >> gpurun_out/headline_repeats.jsonl
done
