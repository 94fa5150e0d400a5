#!/bin/bash
# rocprofv3 passes over the other configs' kernels (GPU box), one run per pass
# (kernel trace + stats; FETCH_SIZE; WRITE_SIZE; SQ instruction mix; GRBM busy
# cycles; VALU FLOPS), for tools/pmc_kernels.py -> profiles/r02/kernels_pmc.json:
#   cfg3  nuts_kernel<f64,16,2,Gauss>    tools/bench_configs.py --which 3
#   cfg4  hmc_kernel<f32,64,2,Rosenbrock> tools/bench_configs.py --which 4
#   cfg5  mh_kernel<f64,64,4,IsoGauss>   tools/bench_configs.py --which 5
#   hbm   leapfrog_hbm_kernel, 2^20 chains  tools/hbm_leapfrog.py
#   WHICH="cfg3 cfg4" bash tools/profile_kernels.sh
source tools/gpu_check.sh
O=gpurun_out/prof_kernels
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU"
FLOPS="SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64"
st=0
for w in ${WHICH:-cfg3 cfg4 cfg5 hbm}; do
  case $w in
    cfg3) CMD="tools/bench_configs.py --which 3 --nuts-discard 200 --nuts-collect 200" ;;
    cfg4) CMD="tools/bench_configs.py --which 4" ;;
    cfg5) CMD="tools/bench_configs.py --which 5" ;;
    hbm)  CMD="tools/hbm_leapfrog.py --reps 5" ;;
  esac
  run ${w}_trace 240 rocprofv3 --kernel-trace --stats -d $O/$w/trace -o run --output-format csv -- python3 $CMD &&
  run ${w}_fetch 240 timeout -s KILL 230 rocprofv3 --pmc FETCH_SIZE -d $O/$w/fetch -o run --output-format csv -- python3 $CMD &&
  run ${w}_write 240 timeout -s KILL 230 rocprofv3 --pmc WRITE_SIZE -d $O/$w/write -o run --output-format csv -- python3 $CMD &&
  run ${w}_sq 240 timeout -s KILL 230 rocprofv3 --pmc $SQ -d $O/$w/sq -o run --output-format csv -- python3 $CMD &&
  run ${w}_grbm 240 timeout -s KILL 230 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/$w/grbm -o run --output-format csv -- python3 $CMD &&
  run ${w}_flops 240 timeout -s KILL 230 rocprofv3 --pmc $FLOPS -d $O/$w/flops -o run --output-format csv -- python3 $CMD || { st=1; break; }
done
[ $st = 0 ] && python3 tools/pmc_kernels.py $O >&2
