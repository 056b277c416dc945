#!/bin/bash
# A/B of lb_rollout builds at the strong-scaling shard sizes (kbench --rollout, tpe layout)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
 for lib in gym-loadbalancing_amd/lbk8s/liblbk8s.so ${LIBS}; do
  echo "lib $lib"
  timeout -k 10 120 python3 tools/kbench.py --rollout --configs default --sizes ${SIZES:-17,20} --lib $lib || exit 1
 done
done
