#!/bin/bash
# SQ counters of the DQN act kernel (k_deepsets_fwd<1,4,2>) at 4096 and 65,536 envs: VALU
# vs MFMA instruction counts and MFMA pipe busy cycles
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 4096 65536; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA \
      SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/actpmc_$n -o run \
      --output-format csv -- python3 tools/act_bench.py --envs $n --n 10 --reps 1 > gpurun_out/actpmc_$n.log 2>&1 || exit 1
  python3 tools/pmc_sum.py gpurun_out/actpmc_$n/run_counter_collection.csv k_deepsets_fwd || exit 1
done
