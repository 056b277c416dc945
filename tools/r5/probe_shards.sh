#!/bin/bash
# Round 5, first probe: where the 131,072-env shard's K = 20 step goes (per-wave timeline),
# and K = 100 vs K = 20 at the strong-scaling shard sizes (product dispatch, k_rollout_lean).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r05_probe_shards.jsonl
: > $O
for n in 131072 262144; do
  timeout -k 10 120 python3 tools/timeline_lean.py --lib exp/liblbk8s_timeline.so --envs $n --steps 20 >> $O 2>>gpurun_out/r05_probe.err || exit 1
  timeout -k 10 120 python3 tools/roll_variants.py --envs $n --steps 100,20 --variants 0 --reps 3 --launches 1 >> $O 2>>gpurun_out/r05_probe.err || exit 1
done
timeout -k 10 120 python3 tools/timeline_lean.py --lib exp/liblbk8s_timeline.so --envs 1048576 --steps 20 >> $O 2>>gpurun_out/r05_probe.err || exit 1
cat $O
