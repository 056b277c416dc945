#!/bin/bash
# Diagnostic: k_rollout_lean without its 4 per-step table loads (wrong values), against the
# product build, K = 20 (split layout) and 100 (single wave), 131,072 and 2^20 envs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/ab_libs.sh r05_ab_nogather.jsonl "131072 1048576" "20,100" exp/liblbk8s_cur.so exp/liblbk8s_nogather.so
