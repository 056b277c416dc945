set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_eval_golden.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02f.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --config2 > gpurun_out/kbench_c2_r02f.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --config1 > gpurun_out/kbench_c1_r02f.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --rollout --configs default,e64_multi --sizes 12,17,20 --ring 16 > gpurun_out/kbench_roll_r02f.log 2>&1
rc=$?
tail -n 3 gpurun_out/pytest_gpu_r02f.log
cat gpurun_out/kbench_c2_r02f.log gpurun_out/kbench_c1_r02f.log gpurun_out/kbench_roll_r02f.log | grep "^{"
exit $rc
