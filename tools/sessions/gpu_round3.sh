#!/bin/bash
# Round-3 evidence session at the driver's bench shape (--steps 20 --warmup 5: one 20-step
# lb_rollout launch timed): parity tests, smoke, PMC passes of 20-step (and 100-step) rollout
# launches, the bench at both window lengths, and the rocprofv3 kernel summary of the
# driver's exact command.  Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
T="timeout -s KILL 90"
n=1048576
pmc_pair() {  # $1 = K: FETCH_SIZE and WRITE_SIZE passes of K-step launches -> traffic JSON
    PMC_MODE=rollout PMC_K=$1 $T rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_k$1_${TAG} -o run \
        --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmcf_k$1_${TAG}.log 2>&1 \
    && PMC_MODE=rollout PMC_K=$1 $T rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_k$1_${TAG} -o run \
        --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmcw_k$1_${TAG}.log 2>&1 \
    && python3 tools/pmc_traffic.py gpurun_out/pmcf_k$1_${TAG}/run_counter_collection.csv \
        gpurun_out/pmcw_k$1_${TAG}/run_counter_collection.csv --envs $n --steps-per-launch $1 \
        --out gpurun_out/pmc_traffic_rollout_k$1.json
}
sq_pass() {  # $1 = K: the SQ counters of K-step launches
    PMC_MODE=rollout PMC_K=$1 $T rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace -d gpurun_out/sq1_k$1_${TAG} -o run \
        --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/sq1_k$1_${TAG}.log 2>&1 \
    && PMC_MODE=rollout PMC_K=$1 $T rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM \
        SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM --kernel-trace -d gpurun_out/sq2_k$1_${TAG} -o run \
        --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/sq2_k$1_${TAG}.log 2>&1
}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || exit 1
fi
pmc_pair 20 && pmc_pair 100 && sq_pass 20 && sq_pass 100 \
 && timeout -k 10 400 python bench.py --steps 20 --warmup 5 --pmc-json gpurun_out/pmc_traffic.json \
      > gpurun_out/bench_k20_${TAG}.log 2>&1 \
 && timeout -k 10 400 python bench.py --pmc-json gpurun_out/pmc_traffic.json --no-cpu-baseline \
      > gpurun_out/bench_k100_${TAG}.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k20_${TAG} -o run --output-format csv \
      -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --pmc-json gpurun_out/pmc_traffic.json \
      > gpurun_out/bench_prof_k20_${TAG}.log 2>&1
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pytest_gpu_${TAG}.log 2>/dev/null; tail -1 gpurun_out/smoke_${TAG}.log 2>/dev/null
for k in 20 100; do cat gpurun_out/pmc_traffic_rollout_k$k.json 2>/dev/null; echo; done
for k in 20 100; do python3 tools/pmc_sum.py gpurun_out/sq1_k${k}_${TAG}/run_counter_collection.csv k_rollout 2>/dev/null; \
  python3 tools/pmc_sum.py gpurun_out/sq2_k${k}_${TAG}/run_counter_collection.csv k_rollout 2>/dev/null; done
tail -1 gpurun_out/bench_k20_${TAG}.log; tail -1 gpurun_out/bench_k100_${TAG}.log; tail -1 gpurun_out/bench_prof_k20_${TAG}.log
exit $rc
