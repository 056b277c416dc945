#!/bin/bash
# XCD-contiguous block -> env group mapping (LB_LEAN_XCD_MAP) against the product build: lean
# parity on it, then an A/B at the shard sizes, K = 20 and 100.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-loadbalancing_amd/lbk8s/liblbk8s.so
cp $L /tmp/prod.so
cp exp/liblbk8s_xcd.so $L
bash tools/r5/gpu_tests_lean.sh; rc=$?
cp /tmp/prod.so $L; [ $rc -eq 0 ] || exit $rc
bash tools/r5/ab_libs.sh r05_ab_xcd.jsonl "131072 262144 1048576" "20,100" exp/liblbk8s_cur.so exp/liblbk8s_xcd.so
