#!/bin/bash
# A/B of the deep-sets forward's interleaved critic tail: deep-sets / learner GPU tests,
# tools/train_bench.py per library, then config 4's and config 5's rl_bench on the product build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fused or dqn or deepsets or argmax or learner or nn or ppo" > gpurun_out/pt_il.log 2>&1 \
  || { echo "pytest failed"; tail -30 gpurun_out/pt_il.log; exit 1; }
tail -2 gpurun_out/pt_il.log
for r in 1 2; do for lib in $OLD gym-loadbalancing_amd/lbk8s/liblbk8s.so; do
  timeout -k 10 200 python tools/train_bench.py --R 65,9 --iters 20 --lib $lib 2>/dev/null | tail -2 || exit 1
done; done > gpurun_out/il_tb.jsonl
cut -c1-220 gpurun_out/il_tb.jsonl
timeout -k 10 300 python tools/rl_bench.py --algo ppo > gpurun_out/rl_ppo_il.json 2>gpurun_out/rl_ppo_il_err.log || exit 1
cut -c1-700 gpurun_out/rl_ppo_il.json
timeout -k 10 300 python tools/rl_bench.py --algo dqn > gpurun_out/rl_dqn_il.json 2>gpurun_out/rl_dqn_il_err.log || exit 1
cut -c1-600 gpurun_out/rl_dqn_il.json
