#!/bin/bash
# Round-4 counter session for k_rollout_lean: FETCH/WRITE_SIZE traffic and the SQ passes of
# 20-step launches (the driver's window), product build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -s KILL 90"
K=${K:-20}
n=1048576
PMC_MODE=rollout PMC_K=$K $T rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_k$K -o run \
    --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmcf_k$K.log 2>&1 \
&& PMC_MODE=rollout PMC_K=$K $T rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_k$K -o run \
    --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmcw_k$K.log 2>&1 \
&& python3 tools/pmc_traffic.py gpurun_out/pmcf_k$K/run_counter_collection.csv \
    gpurun_out/pmcw_k$K/run_counter_collection.csv --envs $n --steps-per-launch $K \
    --out gpurun_out/pmc_traffic_rollout_k$K.json \
&& KS=$K EXTRA_PASS="${EXTRA_PASS:-SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH}" bash tools/gpu_sq.sh
rc=$?
cat gpurun_out/pmc_traffic_rollout_k$K.json; echo
exit $rc
