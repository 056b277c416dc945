#!/bin/bash
# Split layout with LDS flags: 1, 2 or 3 env waves per copy wave, against the barrier build
# (cur); lean parity on the 3-env-wave build first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-loadbalancing_amd/lbk8s/liblbk8s.so
cp $L /tmp/prod.so
cp exp/liblbk8s_fcw3.so $L
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lean_oracle.py tests/test_gpu_lean.py -k "not 40" > gpurun_out/r05_fcw_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_fcw_tests.log; cp /tmp/prod.so $L; [ $rc -eq 0 ] || exit $rc
bash tools/r5/ab_libs.sh r05_ab_fcw.jsonl "131072 1048576" 20 exp/liblbk8s_cur.so exp/liblbk8s_fcw1.so exp/liblbk8s_fcw2.so exp/liblbk8s_fcw3.so
