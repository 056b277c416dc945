#!/bin/bash
# the deep-sets forward GPU tests (new batch-size sweep included)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pt_fused.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_fused.log; exit 1; }
tail -2 gpurun_out/pt_fused.log
