#!/bin/bash
# persistent k_rollout_img experiment: bit-identity vs the product dispatch, then the A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/persist_check.py --envs 300001 --K 20 && \
timeout -k 10 120 python3 tools/persist_check.py --envs 1048576 --K 7 && \
REPS="1 2" LIBS="exp/liblbk8s_base.so gym-loadbalancing_amd/lbk8s/liblbk8s.so" ABARGS="--variants 0,11" bash tools/gpu_abroll.sh
