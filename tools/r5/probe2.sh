#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 exp/wbench_sizes > gpurun_out/r05_wbench_sizes.jsonl 2>&1 || exit 1
O=gpurun_out/r05_timeline2.jsonl
: > $O
for n in 131072 262144 1048576; do
  timeout -k 10 120 python3 tools/timeline_lean.py --lib exp/liblbk8s_timeline.so --envs $n --steps 20 >> $O 2>>gpurun_out/r05_probe.err || exit 1
done
cat gpurun_out/r05_wbench_sizes.jsonl $O
