#!/bin/bash
# k_rollout_lean's parity tests: against the C oracle (new) and against lb_policy + lb_step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lean_oracle.py tests/test_gpu_lean.py "$@" > gpurun_out/r05_lean_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r05_lean_tests.log
exit $rc
