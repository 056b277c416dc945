#!/bin/bash
# Counters of k_rollout_tpe on bench.py's staggered workload (tools/pmc_probe.py,
# PMC_MODE=rollout, PMC_ENVS envs): SQ passes, then FETCH_SIZE / WRITE_SIZE -> traffic JSON.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -s KILL 90"
n=${PMC_ENVS:-1048576}
export PMC_MODE=rollout PMC_ENVS=$n PMC_K=${PMC_K:-100}
CMD="python3 tools/pmc_probe.py"
$T rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace -d gpurun_out/rp1_$n -o run --output-format csv -- $CMD > gpurun_out/rp1_$n.log 2>&1 || exit 1
$T rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM --kernel-trace -d gpurun_out/rp2_$n -o run --output-format csv -- $CMD > gpurun_out/rp2_$n.log 2>&1 || exit 1
$T rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace -d gpurun_out/rp3_$n -o run --output-format csv -- $CMD > gpurun_out/rp3_$n.log 2>&1 || echo "rp3 failed"
$T rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/rp4_$n -o run --output-format csv -- $CMD > gpurun_out/rp4_$n.log 2>&1 || exit 1
$T rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/rp5_$n -o run --output-format csv -- $CMD > gpurun_out/rp5_$n.log 2>&1 || exit 1
for z in rp1 rp2 rp3 rp4 rp5; do python3 tools/pmc_sum.py gpurun_out/${z}_$n/run_counter_collection.csv ${KNAME:-k_rollout} || true; done
python3 tools/pmc_traffic.py gpurun_out/rp4_$n/run_counter_collection.csv gpurun_out/rp5_$n/run_counter_collection.csv \
    --envs $n --steps-per-launch ${PMC_K:-100} --out gpurun_out/pmc_traffic_rollout_$n.json
