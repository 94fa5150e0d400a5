#!/bin/bash
# A/B baseline: the whole libgmcmc.so built from the sources of a git
# revision (e.g. the previous round's final tree) into abtest/NAME:
#   tools/ab_build_full.sh NAME REV
# then time it against the working tree's library in one GPU call
# (GMCMC_LIB=abtest/NAME/libgmcmc.so, tools/ab_run.py / ab_nuts.py).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=$2
OUT=$ROOT/abtest/$name; SRC=$(mktemp -d)
mkdir -p "$OUT"
(cd "$ROOT" && git archive "$rev" general-mcmc_amd include tools/embed_headers.py tools/source_digest.py | tar -x -C "$SRC")
make -s -C "$SRC/general-mcmc_amd" -j8 LIB="$OUT/libgmcmc.so" >/dev/null
rm -rf "$SRC"
echo "built abtest/$name from $rev"
