#!/bin/bash
# same-box A/B of config 5 (rl_bench --algo dqn): exp/head (the last commit) vs the tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do for t in exp/head/tools tools; do
  timeout -k 10 200 python $t/rl_bench.py --algo dqn 2>>gpurun_out/dqn_ab_err.log | tail -1 | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$t', round(d['value']/1e6,2), round(d['ms_per_vector_step']*1e3,2))" || exit 1
done; done | tee gpurun_out/dqn_ab.txt
