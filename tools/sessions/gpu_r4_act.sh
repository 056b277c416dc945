#!/bin/bash
# A/B of the deep-sets forward's wave-major spread (lb_dqn_act at config 5's shape, the
# training forward) between abx/liblbk8s_act_old.so and the product build: the DQN and
# deep-sets GPU tests first, then tools/act_bench.py and tools/train_bench.py per library,
# then config 5's rl_bench on the product build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fused or dqn or deepsets or argmax or learner or nn" > gpurun_out/pt_act.log 2>&1 \
  || { echo "pytest failed"; tail -30 gpurun_out/pt_act.log; exit 1; }
tail -2 gpurun_out/pt_act.log
for r in 1 2; do for lib in ${OLD:-abx/liblbk8s_act_old.so} gym-loadbalancing_amd/lbk8s/liblbk8s.so; do
  timeout -k 10 120 python tools/act_bench.py --lib $lib 2>>gpurun_out/act_err.log || exit 1
done; done > gpurun_out/act_ab.jsonl
cut -c1-200 gpurun_out/act_ab.jsonl
for lib in ${OLD:-abx/liblbk8s_act_old.so} gym-loadbalancing_amd/lbk8s/liblbk8s.so; do
  timeout -k 10 200 python tools/train_bench.py --R 65,9 --iters 20 --lib $lib 2>/dev/null | tail -2 || exit 1
done > gpurun_out/act_tb.jsonl
cut -c1-220 gpurun_out/act_tb.jsonl
timeout -k 10 300 python tools/rl_bench.py --algo dqn > gpurun_out/rl_dqn_act.json 2>gpurun_out/rl_dqn_act_err.log || exit 1
cut -c1-600 gpurun_out/rl_dqn_act.json
