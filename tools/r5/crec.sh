#!/bin/bash
# Split layout with the next-episode records drawn by the copy wave: lean parity on it (the
# product build), then an A/B against the previous split build at the shard sizes, K = 20.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/gpu_tests_lean.sh || exit 1
bash tools/r5/ab_libs.sh r05_ab_crec.jsonl "131072 262144 1048576" 20 exp/liblbk8s_cur.so exp/liblbk8s_crec.so
