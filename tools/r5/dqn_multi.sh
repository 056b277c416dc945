#!/bin/bash
# Multi-step DQN periods (lb_dqn_steps): parity tests, then config 5 with and without them,
# and the kernel summary of the multi-step run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dqn_step.py \
    "tests/test_gpu_learners.py::test_dqn_multi_step_periods_match_single_steps" \
    "tests/test_gpu_learners.py::test_dqn_graph_train_step_matches_eager" > gpurun_out/r05_dqn_multi_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r05_dqn_multi_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1 0 1; do
  LBK8S_DQN_MULTISTEP=$m timeout -k 10 200 python tools/rl_bench.py --algo dqn --envs 4096 \
      >> gpurun_out/r05_rl_dqn_multi.jsonl 2>gpurun_out/rl_dqn_err.log || { tail -20 gpurun_out/rl_dqn_err.log; exit 1; }
  tail -1 gpurun_out/r05_rl_dqn_multi.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dqn_multi -o run --output-format csv \
    -- python3 tools/rl_bench.py --algo dqn --envs 4096 --steps 500 > gpurun_out/prof_dqn_multi.log 2>&1 || exit 1
head -14 gpurun_out/prof_dqn_multi/run_kernel_stats.csv | cut -c1-160
