#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r05_timeline_split.jsonl
: > $O
for n in 131072 1048576; do
  timeout -k 10 120 python3 tools/timeline_lean.py --lib exp/liblbk8s_timeline.so --envs $n --steps 20 --save gpurun_out/r05_tl_$n.npz >> $O 2>>gpurun_out/r05_probe.err || exit 1
done
cat $O
