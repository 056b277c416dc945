#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile.
# Every GPU step has its own time limit; steps are chained with && (stop at first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
 && timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.log 2>&1 \
 && timeout -k 10 300 python tools/kbench.py > gpurun_out/kbench_${TAG}.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv \
      -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.log 2>&1
rc=$?
echo "exit $rc"
tail -5 gpurun_out/pytest_gpu_${TAG}.log
cat gpurun_out/bench_${TAG}.log 2>/dev/null | tail -3
cat gpurun_out/kbench_${TAG}.log 2>/dev/null
exit $rc
