#!/bin/bash
# The round's last lean builds on one box: before the split layout (pre) and the product (cur),
# K = 20 (cur: split) and K = 100 (both single-wave), 131,072 and 2^20 envs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/ab_libs.sh r05_ab_pre_cur.jsonl "131072 1048576" "20,100" exp/liblbk8s_pre.so exp/liblbk8s_cur.so
