#!/bin/bash
# The whole GPU suite, smoke() and the driver's bench line on the current build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05_full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -3 gpurun_out/smoke_${TAG}.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | cut -c1-400
