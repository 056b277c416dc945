# PPO config-4 update time: fused vs foreach Adam
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nn_golden.py tests/test_gpu_learners.py > gpurun_out/t_tests.log 2>&1 || { tail -30 gpurun_out/t_tests.log; exit 1; }
tail -1 gpurun_out/t_tests.log
for f in 1; do LBK8S_FUSED_ADAM=$f $T 300 python tools/rl_bench.py --algo ppo --updates 3 > gpurun_out/t_ppo_$f.log 2>&1 || exit 1; grep -h "^{" gpurun_out/t_ppo_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused', $f, {k: d[k] for k in ('value','ms_per_update','rollout_ms','update_ms')})"; done
$T 300 python tools/rl_bench.py --algo dqn > gpurun_out/t_dqn.log 2>&1 && grep -h "^{" gpurun_out/t_dqn.log | cut -c1-300
