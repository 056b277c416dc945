#!/bin/bash
# DQN period launch with the env held in registers across its steps: parity tests, config 5,
# kernel summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dqn_step.py \
    tests/test_gpu_learners.py -k "dqn" > gpurun_out/r05_dqn_regs2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_dqn_regs2_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r05_rl_dqn_regs2.jsonl
for s in 2000 2000 2000 6000; do
  timeout -k 10 200 python tools/rl_bench.py --algo dqn --envs 4096 --steps $s >> gpurun_out/r05_rl_dqn_regs2.jsonl 2>gpurun_out/rl_dqn_err.log || { tail -20 gpurun_out/rl_dqn_err.log; exit 1; }
  tail -1 gpurun_out/r05_rl_dqn_regs2.jsonl | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['vector_steps'], d['value'], d['ms_per_vector_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dqn_regs2 -o run --output-format csv \
    -- python3 tools/rl_bench.py --algo dqn --envs 4096 --steps 1000 > gpurun_out/prof_dqn_regs2.log 2>&1 || exit 1
head -4 gpurun_out/prof_dqn_regs2/run_kernel_stats.csv | cut -c1-150
