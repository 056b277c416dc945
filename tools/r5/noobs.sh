#!/bin/bash
# Diagnostic: k_rollout_lean without its obs stores (the env work and the reward / done stores
# only) against the product build, at 131,072 and 2^20 envs, K = 20 and 100.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/ab_libs.sh r05_ab_noobs.jsonl "131072 1048576" "20,100" exp/liblbk8s_cur.so exp/liblbk8s_noobs.so
