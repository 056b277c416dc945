#!/bin/bash
# Round-evidence session: parity tests, smoke, PMC traffic passes, bench (reads the
# traffic JSON), and the rocprofv3 kernel-trace summary of the same bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_${TAG} -o run --output-format csv \
      -- python3 tools/pmc_probe.py > gpurun_out/pmc_fetch_${TAG}.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_${TAG} -o run --output-format csv \
      -- python3 tools/pmc_probe.py > gpurun_out/pmc_write_${TAG}.log 2>&1 \
 && python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_${TAG}/run_counter_collection.csv \
      gpurun_out/pmc_write_${TAG}/run_counter_collection.csv --out gpurun_out/pmc_traffic_${TAG}.json \
 && cp gpurun_out/pmc_traffic_${TAG}.json profiles/pmc_traffic.json \
 && PMC_MODE=rollout timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcr_fetch_${TAG} -o run \
      --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmcr_fetch_${TAG}.log 2>&1 \
 && PMC_MODE=rollout timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcr_write_${TAG} -o run \
      --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmcr_write_${TAG}.log 2>&1 \
 && python3 tools/pmc_traffic.py gpurun_out/pmcr_fetch_${TAG}/run_counter_collection.csv \
      gpurun_out/pmcr_write_${TAG}/run_counter_collection.csv --steps-per-launch 100 --out gpurun_out/pmc_traffic_rollout_${TAG}.json \
 && cp gpurun_out/pmc_traffic_rollout_${TAG}.json profiles/pmc_traffic_rollout.json \
 && timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.log 2>&1
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pytest_gpu_${TAG}.log; tail -1 gpurun_out/smoke_${TAG}.log
cat gpurun_out/pmc_traffic_${TAG}.json; echo; cat gpurun_out/pmc_traffic_rollout_${TAG}.json; echo; tail -1 gpurun_out/bench_${TAG}.log; tail -1 gpurun_out/bench_prof_${TAG}.log
exit $rc
