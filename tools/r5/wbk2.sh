#!/bin/bash
# The store-only floor by where a 20-step launch writes, then the driver's bench line with its
# timed window on never-written slots (--warmup 5, the driver's) and on slots written one ring
# cycle before (--warmup 105).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 exp/wbench_k > gpurun_out/r05_wbench_k2.jsonl 2>&1 || { cat gpurun_out/r05_wbench_k2.jsonl; exit 1; }
cat gpurun_out/r05_wbench_k2.jsonl
: > gpurun_out/r05_bench_warm.jsonl
for w in 5 105 5 105; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup $w --no-cpu-baseline --no-step-line >> gpurun_out/r05_bench_warm.jsonl 2>gpurun_out/r05_bench_warm.err || exit 1
  tail -1 gpurun_out/r05_bench_warm.jsonl | python3 -c "import json,sys;d=json.load(sys.stdin);print('warmup', d['warmup'], round(d['roofline']['kernel_ms']*1e3,2), 'us/step frac', round(d['roofline']['frac'],3))"
done
