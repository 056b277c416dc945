#!/bin/bash
# lb_dqn_act / lb_ds_q_argmax launch time against the batch size (R = 9): fixed latency
# chain vs work proportional to the envs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in 256 1024 2048 4096 8192 16384 65536; do
  timeout -k 10 120 python tools/act_bench.py --envs $n --reps 3 2>>gpurun_out/actsize_err.log || exit 1
done > gpurun_out/act_sizes.jsonl
cut -c1-150 gpurun_out/act_sizes.jsonl
