#!/bin/bash
# A/B variant: libgmcmc.so with ONE translation unit compiled from the sources
# of a git revision (the other objects from the current build), e.g. the
# previous MH kernel against the current one:
#   tools/ab_build_rev.sh NAME REV mh_kernels.hip
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=$2; tu=$3
OUT=$ROOT/abtest/$name; SRC=$(mktemp -d)
mkdir -p "$OUT" "$SRC/csrc" "$SRC/include"
(cd "$ROOT" && git archive "$rev" general-mcmc_amd/csrc include | tar -x -C "$SRC")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -fno-slp-vectorize -fPIC -Wno-unused-result \
  -I/opt/rocm/include -c "$SRC/general-mcmc_amd/csrc/$tu" -o "$OUT/$tu.o"
B=$ROOT/general-mcmc_amd/build
OBJS=$(ls $B/*.o | grep -v "/$tu.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libgmcmc.so" "$OUT/$tu.o" $OBJS \
  -L/opt/rocm/lib -lrccl -lhiprtc -ldl -Wl,-rpath,/opt/rocm/lib
rm -rf "$OUT/$tu.o" "$SRC"
echo "built abtest/$name ($tu from $rev)"
