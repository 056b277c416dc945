set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
for l in bwd_il bwd_sgb3 bwd_sgb5; do $T 120 python tools/train_bench.py --lib exp/$l.so > gpurun_out/n_$l.json 2>&1 || exit 1; done
grep -h sets gpurun_out/n_*.json
$T 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_il1 -o run --output-format csv -- python3 tools/train_bench.py --R 65 --iters 3 --lib exp/bwd_il.so > gpurun_out/pmc_il1.log 2>&1 || exit 1
$T 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM --kernel-trace -d gpurun_out/pmc_il2 -o run --output-format csv -- python3 tools/train_bench.py --R 65 --iters 3 --lib exp/bwd_il.so > gpurun_out/pmc_il2.log 2>&1 || exit 1
for d in pmc_il1 pmc_il2; do python3 tools/pmc_sum.py gpurun_out/$d/run_counter_collection.csv train_bwd; done
