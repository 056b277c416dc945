#!/bin/bash
# The output stores' cache policy: nt (current) vs plain, sc1, nt sc1; K = 20 and 100.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/ab_libs.sh r05_ab_store_policy.jsonl "131072 1048576" "20,100" exp/liblbk8s_aux2.so exp/liblbk8s_aux0.so exp/liblbk8s_aux16.so exp/liblbk8s_aux18.so
