#!/bin/bash
# Final check of the round's build: the whole GPU suite, smoke, and the driver's bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit 1
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1 || exit 1
tail -1 gpurun_out/bench_final.log | cut -c1-400
