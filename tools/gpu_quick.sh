#!/bin/bash
# Quick GPU iteration: parity tests, bench, kernel bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-q}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}.log 2>&1 \
 && timeout -k 10 300 python tools/kbench.py > gpurun_out/kbench_${TAG}.log 2>&1
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pytest_gpu_${TAG}.log; tail -1 gpurun_out/bench_${TAG}.log; cat gpurun_out/kbench_${TAG}.log
exit $rc
