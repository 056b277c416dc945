#!/bin/bash
# DQN train-step launches cut (loss in the head's launch, unit-seed backward) and k_dqn_step with
# 2 envs per wave iteration vs 4: the DQN / PPO parity tests on the product build (P = 4) and the
# multi-step tests on the P = 2 build, then config 5 alternating the two builds, and PPO.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-loadbalancing_amd/lbk8s/liblbk8s.so
cp $L /tmp/lib_p4.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dqn_step.py \
    tests/test_gpu_learners.py tests/test_nn_golden.py > gpurun_out/r05_dqn_p4_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05_dqn_p4_tests.log; [ $rc -eq 0 ] || exit $rc
cp exp/liblbk8s_dqnp2.so $L
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dqn_step.py \
    "tests/test_gpu_learners.py::test_dqn_multi_step_periods_match_single_steps" > gpurun_out/r05_dqn_p2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05_dqn_p2_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r05_rl_dqn_p2.jsonl
for v in p4 p2 p4 p2; do
  if [ $v = p4 ]; then cp /tmp/lib_p4.so $L; else cp exp/liblbk8s_dqnp2.so $L; fi
  timeout -k 10 200 python tools/rl_bench.py --algo dqn --envs 4096 > /tmp/o.json 2>gpurun_out/rl_dqn_err.log || { tail -20 gpurun_out/rl_dqn_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('/tmp/o.json'));d['variant']='$v';print(json.dumps(d))" >> gpurun_out/r05_rl_dqn_p2.jsonl
  echo $v $(python3 -c "import json;print(json.load(open('/tmp/o.json'))['value'])")
done
cp /tmp/lib_p4.so $L
timeout -k 10 300 python tools/rl_bench.py --algo ppo --envs 4096 > gpurun_out/r05_rl_ppo.json 2> gpurun_out/rl_ppo_err.log || { tail -20 gpurun_out/rl_ppo_err.log; exit 1; }
cat gpurun_out/r05_rl_ppo.json
