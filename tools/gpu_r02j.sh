set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_train.py tests/test_nn_golden.py tests/test_gpu_learners.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_train_r02j.log 2>&1
rc=$?
tail -n 30 gpurun_out/pytest_train_r02j.log | grep -v "^$" | tail -25
for rep in 1 2; do
  timeout -k 10 200 python tools/train_bench.py --lib exp/liblbk8s_head.so > gpurun_out/tbj_head_$rep.log 2>&1 || exit 1
  timeout -k 10 200 python tools/train_bench.py --lib exp/liblbk8s_new.so > gpurun_out/tbj_new_$rep.log 2>&1 || exit 1
done
grep -h "^{" gpurun_out/tbj_*.log
exit $rc
