#!/bin/bash
# cfg5 MH (16384 chains x 256-D f64) throughput per compiled layout, one process each.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for L in ${MH_LAYOUTS:-64x4 32x8 64x8 16x16 64x16 64x4}; do
  timeout -k 10 120 python tools/bench_configs.py --which 5 --mh-layout $L >> gpurun_out/mh_layouts.jsonl 2>&1 || echo "layout $L failed" >> gpurun_out/mh_layouts.jsonl
done
grep -h chain_steps_per_s gpurun_out/mh_layouts.jsonl | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['layout'], '%.3e' % d['chain_steps_per_s'])"
