set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_train.py tests/test_nn_golden.py tests/test_gpu_learners.py > gpurun_out/o_tests.log 2>&1 || { tail -30 gpurun_out/o_tests.log; exit 1; }
tail -1 gpurun_out/o_tests.log
for l in ${LIBS:-bwd_old bwd_il2}; do $T 120 python tools/train_bench.py --lib exp/$l.so > gpurun_out/o_$l.json 2>&1 || exit 1; grep -h sets gpurun_out/o_$l.json; done
if [ -n "$PMC" ]; then
$T 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_o1 -o run --output-format csv -- python3 tools/train_bench.py --R 65 --iters 3 > gpurun_out/pmc_o1.log 2>&1 || exit 1
python3 tools/pmc_sum.py gpurun_out/pmc_o1/run_counter_collection.csv train_bwd
fi
