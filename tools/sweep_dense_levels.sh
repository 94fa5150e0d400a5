#!/bin/bash
# cfg3 with dense adaptation: full vs packed M^-1 in LDS, subtree-stack levels in LDS capped.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for cfg in "2 0" "2 1" "1 0" "1 1" "1 3" "1 6"; do
  set -- $cfg
  r=$(timeout -k 10 200 python tools/bench_configs.py --which 3 --nuts-mass dense --nuts-dense-forms $1,0 --nuts-lds-levels $2 | tail -1) || exit $?
  echo "minv_lds=$1 levels<=$2 $(echo "$r" | grep -o '"leapfrog_per_s": [0-9.e+]*')"
done
