#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_api.py -k "vecmonitor or sb3" > gpurun_out/r05_monitor_tests.log 2>&1 || { tail -30 gpurun_out/r05_monitor_tests.log; exit 1; }
tail -3 gpurun_out/r05_monitor_tests.log
bash tools/r5/probe2.sh
