# PMC passes over the backward (tools/train_bench.py R=65): cycle buckets and instruction mix
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
TAG=${TAG:-r}
$T 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_${TAG}1 -o run --output-format csv -- python3 tools/train_bench.py --R ${R:-65} --iters 3 > gpurun_out/pmc_${TAG}1.log 2>&1 || exit 1
$T 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM --kernel-trace -d gpurun_out/pmc_${TAG}2 -o run --output-format csv -- python3 tools/train_bench.py --R ${R:-65} --iters 3 > gpurun_out/pmc_${TAG}2.log 2>&1 || exit 1
$T 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_${TAG}3 -o run --output-format csv -- python3 tools/train_bench.py --R ${R:-65} --iters 3 > gpurun_out/pmc_${TAG}3.log 2>&1 || exit 1
for i in 1 2 3; do python3 tools/pmc_sum.py gpurun_out/pmc_${TAG}$i/run_counter_collection.csv train_bwd; done
