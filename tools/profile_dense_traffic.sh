#!/bin/bash
# HBM traffic of the dense-metric NUTS sampling launch per dense form (full vs packed M^-1):
# FETCH_SIZE, WRITE_SIZE and a kernel trace of tools/bench_configs.py cfg3 --nuts-mass dense, one rocprofv3
# run each; reduced into profiles/r04/dense_traffic.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for f in 2,1 1,0; do
  t=${f/,/_}
  timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/dtr_$t/fetch -o run --output-format csv -- python3 tools/bench_configs.py --which 3 --nuts-mass dense --nuts-dense-forms $f > gpurun_out/dtr_fetch_$t.log 2>&1 || exit 3
  timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/dtr_$t/write -o run --output-format csv -- python3 tools/bench_configs.py --which 3 --nuts-mass dense --nuts-dense-forms $f > gpurun_out/dtr_write_$t.log 2>&1 || exit 4
  timeout -s KILL 280 rocprofv3 --kernel-trace --stats -d gpurun_out/dtr_$t/trace -o run --output-format csv -- python3 tools/bench_configs.py --which 3 --nuts-mass dense --nuts-dense-forms $f > gpurun_out/dtr_trace_$t.log 2>&1 || exit 5
done
