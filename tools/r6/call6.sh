set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_fused_train.py tests/test_gpu_learners.py tests/test_eval_golden.py tests/test_gpu_dqn_step.py > gpurun_out/r06_ds_tests.log 2>&1; rc=$?; tail -n 5 gpurun_out/r06_ds_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/train_bench.py --R 65,33,9 > gpurun_out/r06_train_bench_vg.jsonl 2>> gpurun_out/r06_ds.err || exit 1
timeout -k 10 300 python3 tools/rl_bench.py --algo ppo --updates 2 > gpurun_out/r06_rl_bench_ppo_vg.json 2>> gpurun_out/r06_ds.err || exit 1
cat gpurun_out/r06_train_bench_vg.jsonl gpurun_out/r06_rl_bench_ppo_vg.json
