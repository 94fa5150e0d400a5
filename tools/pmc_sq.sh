#!/bin/bash
# SQ instruction-mix / wait PMC passes (each its own run) over one command.
# Usage (GPU box): bash tools/pmc_sq.sh OUTDIR cmd args...
source tools/gpu_check.sh
O=$1; shift
run pmc_sq_a 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmca -o run --output-format csv -- "$@" &&
run pmc_sq_b 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $O/pmcb -o run --output-format csv -- "$@"
