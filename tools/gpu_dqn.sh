#!/bin/bash
# GPU suite + config-5 (DQN) A/B: period graphs with device RNG vs the round-2 host path,
# and the kernel summary of the period-graph run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_all.log 2>&1
rc=$?; tail -15 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
for m in "1 1" "0 0"; do
  set -- $m
  LBK8S_DQN_PERIOD_GRAPH=$1 LBK8S_DQN_DEVICE_RNG=$2 timeout -k 10 200 python tools/rl_bench.py --algo dqn --envs 4096 \
      > gpurun_out/rl_dqn_$1$2.json 2>gpurun_out/rl_dqn_err.log || { tail -20 gpurun_out/rl_dqn_err.log; exit 1; }
  cat gpurun_out/rl_dqn_$1$2.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dqn -o run --output-format csv \
    -- python3 tools/rl_bench.py --algo dqn --envs 4096 --steps 500 > gpurun_out/prof_dqn.log 2>&1 || exit 1
head -14 gpurun_out/prof_dqn/run_kernel_stats.csv | cut -c1-200
timeout -k 10 300 python tools/rl_bench.py --algo ppo --envs 4096 > gpurun_out/rl_ppo.json 2> gpurun_out/rl_ppo_err.log || { tail -20 gpurun_out/rl_ppo_err.log; exit 1; }
cat gpurun_out/rl_ppo.json
