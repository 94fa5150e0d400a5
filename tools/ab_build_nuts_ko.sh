#!/bin/bash
# Measurement-only knock-out builds of the NUTS kernel (nuts_part0.hip holds
# layout 16x2): each variant removes one component's work (GM_KO_* macros in
# nuts_device.h / gm_device.h; results differ) so that its marginal cost can
# be read from the sampling-phase throughput (tools/ab_nuts.py).
#   tools/ab_build_nuts_ko.sh NAME "-DGM_KO_X" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/general-mcmc_amd/build
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  OUT=$ROOT/abtest/$name; mkdir -p "$OUT"
  /opt/rocm/bin/hipcc $flags --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -fno-slp-vectorize -fPIC \
    -Wno-unused-result -I/opt/rocm/include -c "$ROOT/general-mcmc_amd/csrc/nuts_part0.hip" -o "$OUT/nuts_part0.hip.o"
  OBJS=$(ls $B/*.o | grep -v nuts_part0)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libgmcmc.so" "$OUT/nuts_part0.hip.o" $OBJS \
    -L/opt/rocm/lib -lrccl -lhiprtc -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
  rm -f "$OUT/nuts_part0.hip.o"
  echo "built abtest/$name ($flags)"
done
