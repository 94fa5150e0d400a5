#!/bin/bash
# cfg4 (HMC RosenbrockND 128-D f32, 8192 chains) across layouts and leapfrog
# unrolls: the clock/occupancy trade-off (8 waves per SIMD at 64x2, 4 at 32x4,
# 2 at 16x8), two rounds, one line per run into gpurun_out/cfg4_layouts.jsonl.
source tools/gpu_check.sh
for r in 1 2; do
  for lay in 64x2 32x4 16x8; do
    for u in 1 2 4; do
      run cfg4_lay 120 python tools/bench_configs.py --which 4 --hmc128-layout $lay --hmc128-unroll $u || exit $?
      grep '^{' gpurun_out/cfg4_lay.log | sed "s|^{|{\"round\": $r, \"unroll\": $u, |" >> gpurun_out/cfg4_layouts.jsonl
    done
  done
done
