#!/bin/bash
# The split lean layout (env wave + copy wave per block): lean parity tests on it, then an A/B
# against the single-wave build at the shard sizes, K = 20 and 100.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-loadbalancing_amd/lbk8s/liblbk8s.so
cp exp/liblbk8s_split.so $L
bash tools/r5/gpu_tests_lean.sh || exit 1
cp exp/liblbk8s_cur.so $L
bash tools/r5/ab_libs.sh r05_ab_split.jsonl "131072 262144 1048576" "20,100" exp/liblbk8s_cur.so exp/liblbk8s_split.so
