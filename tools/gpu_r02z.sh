# SQ counters of the step kernel at PMC_ENVS envs (bench's staggered workload)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -s KILL 120"
for n in ${SIZES}; do
 PMC_ENVS=$n $T rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace -d gpurun_out/z1_$n -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/z1_$n.log 2>&1 || exit 1
 PMC_ENVS=$n $T rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM --kernel-trace -d gpurun_out/z2_$n -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/z2_$n.log 2>&1 || exit 1
 PMC_ENVS=$n $T rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-trace -d gpurun_out/z3_$n -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/z3_$n.log 2>&1 || echo "z3 failed $n"
 for z in z1 z2 z3; do python3 tools/pmc_sum.py gpurun_out/${z}_$n/run_counter_collection.csv k_step_tpe || true; python3 tools/pmc_sum.py gpurun_out/${z}_$n/run_counter_collection.csv k_reset_listed || true; done
done
