#!/bin/bash
# Perf-investigation session: bandwidth calibration, PMC traffic passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 120 python tools/calib_bw.py > gpurun_out/calib_${TAG}.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_${TAG} -o run --output-format csv \
      -- python3 tools/pmc_probe.py > gpurun_out/pmc_fetch_${TAG}.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_${TAG} -o run --output-format csv \
      -- python3 tools/pmc_probe.py > gpurun_out/pmc_write_${TAG}.log 2>&1
rc=$?
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_${TAG}.txt 2>&1
echo "exit $rc"
cat gpurun_out/calib_${TAG}.log
exit $rc
