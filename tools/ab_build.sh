#!/bin/bash
# Build a variant of libgmcmc.so whose hmc kernels come from another source
# tree (A/B timing of kernel changes in one GPU call; tools/ab_run.py).
#   tools/ab_build.sh <csrc-dir> <out-dir>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; OUT=$2
mkdir -p "$OUT"
FLAGS="$AB_DEFS --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -fno-slp-vectorize -fPIC -I/opt/rocm/include -I$SRC/../include"
/opt/rocm/bin/hipcc $FLAGS -c "$SRC/hmc_kernels.hip" -o "$OUT/hmc_kernels.hip.o"
B=$ROOT/general-mcmc_amd/build
OBJS=$(ls $B/*.o | grep -v hmc_kernels)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libgmcmc.so" "$OUT/hmc_kernels.hip.o" $OBJS \
  -L/opt/rocm/lib -lrccl -lhiprtc -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
rm -f "$OUT/hmc_kernels.hip.o"
