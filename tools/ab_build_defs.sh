#!/bin/bash
# A/B variant: the whole libgmcmc.so built from the WORKING TREE's sources
# under extra defines, into abtest/NAME (its own build directory):
#   tools/ab_build_defs.sh NAME "-DGM_PACKED_BATCH=4"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; defs=$2
OUT=$ROOT/abtest/$name; SRC=$(mktemp -d)
mkdir -p "$OUT" "$SRC/tools"
cp -r "$ROOT/general-mcmc_amd" "$ROOT/include" "$SRC/"
cp "$ROOT/tools/embed_headers.py" "$ROOT/tools/source_digest.py" "$SRC/tools/"
rm -rf "$SRC/general-mcmc_amd/build" "$SRC/general-mcmc_amd/lib"
make -s -C "$SRC/general-mcmc_amd" -j${JOBS:-8} EXTRA_FLAGS="$defs" LIB="$OUT/libgmcmc.so" >/dev/null
rm -rf "$SRC"
echo "built abtest/$name with $defs"
