#!/bin/bash
# Build A/B variants of libgmcmc.so from the current sources with extra
# compile flags (measurement macros), each in its own build dir:
#   tools/ab_variants.sh NAME "FLAGS" [NAME "FLAGS" ...]  ->  abtest/NAME/libgmcmc.so
# then time them alternately in one GPU call with GMCMC_LIB=abtest/NAME/libgmcmc.so.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -C "$ROOT/general-mcmc_amd" -j8 BUILD="$ROOT/abtest/$name/build" LIB="$ROOT/abtest/$name/libgmcmc.so" \
       EXTRA_FLAGS="$flags" >/dev/null
  rm -rf "$ROOT/abtest/$name/build"
  echo "built abtest/$name ($flags)"
done
