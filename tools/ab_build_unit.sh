#!/bin/bash
# Variant of libgmcmc.so with ONE translation unit rebuilt from a source tree
# and/or under extra defines (A/B timing of kernel changes in one GPU call):
#   AB_DEFS="-DX=Y" tools/ab_build_unit.sh <unit, e.g. mh_kernels.hip> <csrc-dir> <out-dir>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
UNIT=$1; SRC=$2; OUT=$3
mkdir -p "$OUT"
FLAGS="$AB_DEFS --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -fno-slp-vectorize -fPIC -I/opt/rocm/include -I$SRC"
/opt/rocm/bin/hipcc $FLAGS -c "$SRC/$UNIT" -o "$OUT/$UNIT.o"
B=$ROOT/general-mcmc_amd/build
OBJS=$(ls $B/*.o | grep -v "/$UNIT.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libgmcmc.so" "$OUT/$UNIT.o" $OBJS \
  -L/opt/rocm/lib -lrccl -lhiprtc -ldl -Wl,-rpath,/opt/rocm/lib
rm -f "$OUT/$UNIT.o"
