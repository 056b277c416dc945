#!/bin/bash
# Diagnostic: k_rollout_lean without the record prefetch (restarts load their records; correct)
# and without any loads in the step loop (+ constant table values; wrong values), K = 20 / 100.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-loadbalancing_amd/lbk8s/liblbk8s.so
cp $L /tmp/prod.so
cp exp/liblbk8s_nopref.so $L
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lean_oracle.py > gpurun_out/r05_nopref_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05_nopref_tests.log; cp /tmp/prod.so $L; [ $rc -eq 0 ] || exit $rc
bash tools/r5/ab_libs.sh r05_ab_noload.jsonl "131072 1048576" "20,100" exp/liblbk8s_cur.so exp/liblbk8s_nopref.so exp/liblbk8s_noload.so
