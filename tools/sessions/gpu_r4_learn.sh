#!/bin/bash
# Learning curves at run.py's setup (tools/learn_curves.py): DQN (device RNG), DQN (host RNG),
# PPO, 200,000 learner steps each (or $STEPS), each step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${STEPS:-200000}
for run in ${RUNS:-dqn dqn_host ppo}; do
  case $run in
    dqn) a="--alg dqn";; dqn_host) a="--alg dqn --host-rng";; ppo) a="--alg ppo";;
  esac
  timeout -k 10 ${TL:-900} python3 -u tools/learn_curves.py $a --total-steps $S --out gpurun_out/learn_${run}.json \
      > gpurun_out/learn_${run}.log 2>&1 || { echo "$run failed"; tail -20 gpurun_out/learn_${run}.log; exit 1; }
  tail -1 gpurun_out/learn_${run}.log
done
