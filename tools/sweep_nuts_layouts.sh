cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for L in 16x2 8x4 32x1 4x8 16x2; do
  timeout -k 10 120 python tools/bench_configs.py --which 3 --nuts-layout $L >> gpurun_out/nuts_layouts.jsonl 2>&1 || exit $?
done
