#!/bin/bash
# One GPU session: probes, tests, smoke, bench. Each GPU step has its own time
# limit; a crash/abort/timeout (status >= 124 or signal) ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "fatal step $name ($rc), stopping" >&2; exit $rc; fi
  return $rc
}
for step in "$@"; do
  case $step in
    mfma) run mfma_probe 60 ./tools/probes/bin/gemv_mfma_probe 8192 200 ;;
    tests) run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    mfmatest) run mfma_tests 300 python -u -m pytest tests/test_gpu_mfma_gauss.py -x -q --timeout 120 --timeout-method thread ;;
    fixed) run hmc_fixed 120 python tools/probe_hmc_fixed.py ;;
    essburn) run ess_burnin 300 python tools/probe_ess_burnin.py ;;
    fixed2) run hmc_fixed2 120 python tools/probe_hmc_fixed2.py ;;
    abhmc) run ab_hmc100 300 python tools/ab_run.py general-mcmc_amd/lib/libgmcmc.so $AB_LIBS &&
           AB_ARGS="--layouts 64x1 --rounds 3 --steps 20" run ab_hmc20 300 python tools/ab_run.py general-mcmc_amd/lib/libgmcmc.so $AB_LIBS ;;
    diag) run diag_fullsize 600 python -u tools/diag_fullsize.py gpurun_out/diag_fullsize.jsonl ;;
    diagtest) run diag_tests 600 python -u -m pytest tests/test_gpu_diag_fullsize.py -x -v --timeout 300 --timeout-method thread ;;
    abmh) AB_ROUNDS=${AB_ROUNDS:-3} run ab_mh 600 python tools/ab_mh.py ${AB_LIBS} ;;
    abnuts) AB_ROUNDS=${AB_ROUNDS:-3} run ab_nuts 900 python tools/ab_nuts.py general-mcmc_amd/lib/libgmcmc.so ${AB_LIBS} ;;
    nlevels) run nuts_levels 300 python tools/probe_nuts_levels.py ;;
    nutstest) run nuts_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mfma_gauss.py tests/test_gpu_nuts_truncation.py tests/test_gpu_nuts_mass.py tests/test_gpu_fullsize_edge.py tests/test_gpu_checkpoint.py tests/test_gpu_step.py -x -q -k "nuts or NUTS or cfg3 or mfma" --timeout 120 --timeout-method thread ;;
    masstest) run mass_tests 300 python -u -m pytest tests/test_gpu_nuts_mass.py tests/test_gpu_mfma_gauss.py tests/test_gpu_nuts_truncation.py -x -q --timeout 120 --timeout-method thread ;;
    densemass) run dense_lds0 300 python tools/bench_configs.py --which 3 --nuts-mass dense --nuts-dense-forms 0,0 &&
               run dense_lds1 300 python tools/bench_configs.py --which 3 --nuts-mass dense --nuts-dense-forms 1,1  ;;
    abbench) AB_ROUNDS=${AB_ROUNDS:-4} run ab_bench 600 python tools/ab_bench.py general-mcmc_amd/lib/libgmcmc.so ${AB_LIBS} ;;
    denseforms)
      for r in 1 2; do for f in 2,1 1,0 1,1; do
        run dense_forms 300 python tools/bench_configs.py --which 3 --nuts-mass dense --nuts-dense-forms $f &&
          sed "s|^{|{\"forms\": \"$f\", |" gpurun_out/dense_forms.log | grep '^{' >> gpurun_out/dense_forms.jsonl
      done; done ;;
    mhtest) run mh_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_edge.py tests/test_gpu_tracker.py -x -q -k "mh or MH or cfg5 or Metropolis or tracker" --timeout 120 --timeout-method thread ;;
    warmup) run warmup_probe 300 python tools/probe_warmup.py ;;
    hostpath) run host_path 120 python tools/probe_host_path.py ;;
    steptests) run step_tests 300 python -u -m pytest tests/test_gpu_step.py -x -v --timeout 120 --timeout-method thread ;;
    benchn) run bench_new 600 python bench.py --steps 20 --warmup 5 ;;
    smoke) run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench20) run bench20 300 python bench.py --steps 20 --warmup 5 ;;
    bench) run bench 300 python bench.py ;;
    configs) run configs 300 python tools/bench_configs.py ;;
    mfma64) run mfma_f64_probe 60 ./tools/probes/bin/mfma_f64_probe ;;
    first)
      for v in ${FIRST_VARIANTS:-"--warm-collect --scratch-warm 2" "--warm-collect --scratch-warm 2" "--warm-collect --scratch-warm 2"}; do
        run first_call 60 python tools/probe_bench_first.py --repeat 4 $v && cat gpurun_out/first_call.log >> gpurun_out/first_calls.jsonl
      done ;;
    abhd)
      for r in 1 2; do for l in general-mcmc_amd/lib/libgmcmc.so $AB_LIBS; do
        run nuts_highdim 300 env GMCMC_LIB=$(pwd)/$l python tools/probe_nuts_highdim.py &&
          sed "s|^{|{\"lib\": \"$l\", |" gpurun_out/nuts_highdim.log >> gpurun_out/nuts_highdim.jsonl
      done; done ;;
    abdense) AB_ARGS="--nuts-mass dense" AB_ROUNDS=${AB_ROUNDS:-2} run ab_dense 900 python tools/ab_nuts.py general-mcmc_amd/lib/libgmcmc.so ${AB_LIBS} ;;
    nprof) run nuts_prof 120 env GMCMC_LIB=abtest/nprof/libgmcmc.so python tools/probe_nuts_prof.py ;;
  esac
done
