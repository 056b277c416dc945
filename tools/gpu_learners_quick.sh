set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_learners.py tests/test_gpu_dist.py tests/test_gpu_fused_train.py tests/test_nn_golden.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_dqn2.log 2>&1; rc=$?; tail -4 gpurun_out/pt_dqn2.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 200 python tools/rl_bench.py --algo dqn --envs 4096 > gpurun_out/rl_dqn_n$r.json 2>gpurun_out/rl_dqn_err.log || exit 1; cat gpurun_out/rl_dqn_n$r.json; done
timeout -k 10 300 python tools/rl_bench.py --algo ppo --envs 4096 > gpurun_out/rl_ppo2.json 2> gpurun_out/rl_ppo_err.log || exit 1; cat gpurun_out/rl_ppo2.json
