set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused_train.py tests/test_nn_golden.py > gpurun_out/l_tests.log 2>&1 && \
$T 120 python tools/train_bench.py --lib exp/bwd_old.so > gpurun_out/l_old.json 2>&1 && \
$T 120 python tools/train_bench.py > gpurun_out/l_new.json 2>&1
rc=$?
tail -3 gpurun_out/l_tests.log; cat gpurun_out/l_old.json gpurun_out/l_new.json
exit $rc
