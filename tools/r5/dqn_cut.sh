#!/bin/bash
# DQN train step with fewer launches (head loss in-launch, unit-seed backward, backward image packed
# with the forward's, target + trained forward paired) and P = 2: tests, config 5, kernel summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dqn_step.py \
    tests/test_gpu_learners.py tests/test_nn_golden.py tests/test_gpu_fused.py > gpurun_out/r05_dqn_cut_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05_dqn_cut_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r05_rl_dqn_cut.jsonl
for s in 2000 2000 6000 6000; do
  timeout -k 10 200 python tools/rl_bench.py --algo dqn --envs 4096 --steps $s >> gpurun_out/r05_rl_dqn_cut.jsonl 2>gpurun_out/rl_dqn_err.log || { tail -20 gpurun_out/rl_dqn_err.log; exit 1; }
  tail -1 gpurun_out/r05_rl_dqn_cut.jsonl | cut -c1-260
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dqn_cut -o run --output-format csv \
    -- python3 tools/rl_bench.py --algo dqn --envs 4096 --steps 1000 > gpurun_out/prof_dqn_cut.log 2>&1 || exit 1
head -20 gpurun_out/prof_dqn_cut/run_kernel_stats.csv | cut -c1-150
timeout -k 10 300 python tools/rl_bench.py --algo ppo --envs 4096 > gpurun_out/r05_rl_ppo_cut.json 2> gpurun_out/rl_ppo_err.log || { tail -20 gpurun_out/rl_ppo_err.log; exit 1; }
cat gpurun_out/r05_rl_ppo_cut.json
