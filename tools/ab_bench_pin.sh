#!/bin/bash
# The headline's timed call with and without the host thread pinned to one
# CPU (BENCH_PIN_CPU=1, now the default), alternating processes, 5 rounds: wall, kernel and
# host-path times of each --steps 20 --warmup 5 line into
# gpurun_out/ab_bench_pin.jsonl (no CPU baseline, no config legs).
source tools/gpu_check.sh
ARGS="--steps 20 --warmup 5 --cpu-seconds 0 --cpu-config-seconds 0 --ess-long-discard 0 --no-north-star --configs="
for r in 1 2 3 4 5; do
  for pin in 0 1; do
    run bench_pin 200 env BENCH_PIN_CPU=$pin python bench.py $ARGS || exit $?
    grep '^{' gpurun_out/bench_pin.log | tail -n 1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); t=d['timing']
print(json.dumps({'pin': $pin, 'round': $r, 'value': d['value'], 'wall_us': t['wall_ms']*1e3, 'kernel_us': t['kernel_ms']*1e3, 'host_us': t['host_overhead_ms']*1e3}))" >> gpurun_out/ab_bench_pin.jsonl
  done
done
