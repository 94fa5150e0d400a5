#!/bin/bash
# Variant of libgmcmc.so with the NUTS kernels built under extra defines
# (A/B of kernel knobs in one GPU call):  AB_DEFS="-DX=Y" tools/ab_build_nuts.sh <out-dir>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1
mkdir -p "$OUT"
SRC=$ROOT/general-mcmc_amd/csrc
FLAGS="$AB_DEFS --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -fno-slp-vectorize -fPIC -I/opt/rocm/include"
/opt/rocm/bin/hipcc $FLAGS -c "$SRC/nuts_kernels.hip" -o "$OUT/nuts_kernels.hip.o"
B=$ROOT/general-mcmc_amd/build
OBJS=$(ls $B/*.o | grep -v nuts_kernels)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libgmcmc.so" "$OUT/nuts_kernels.hip.o" $OBJS \
  -L/opt/rocm/lib -lrccl -lhiprtc -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
rm -f "$OUT/nuts_kernels.hip.o"
