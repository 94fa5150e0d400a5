#!/bin/bash
# The headline with the bench's device warm-up at 50 ms (default) and 300 ms,
# alternating fresh processes: does a longer clock ramp move the timed launch?
source tools/gpu_check.sh
rm -f gpurun_out/ab_warmup_ms.jsonl
for r in 1 2 3 4; do
  for w in 50 300; do
    run warm_rep 200 python bench.py --steps 20 --warmup 5 --device-warmup-ms $w --cpu-seconds 0 --cpu-config-seconds 0 --ess-long-discard 0 --no-north-star --configs "" || exit $?
    grep '^{' gpurun_out/warm_rep.log | tail -n 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(json.dumps({'warmup_ms': $w, 'value': d['value'], 'kernel_ms': d['timing']['kernel_ms'], 'host_overhead_ms': d['timing']['host_overhead_ms']}))" >> gpurun_out/ab_warmup_ms.jsonl
  done
done
