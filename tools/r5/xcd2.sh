#!/bin/bash
# The XCD-mapped product build: lean parity, a second A/B against the identity mapping at the
# small shards, the driver line and the shard sizes with rocprof summaries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/gpu_tests_lean.sh || exit 1
bash tools/r5/ab_libs.sh r05_ab_xcd2.jsonl "131072 131072 262144" 20 exp/liblbk8s_cur.so exp/liblbk8s_xcdprod.so || exit 1
: > gpurun_out/r05_xcd_lines.jsonl
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-step-line >> gpurun_out/r05_xcd_lines.jsonl 2>>gpurun_out/r05_bench.err || exit 1
for n in 131072 262144; do
  timeout -k 10 300 python3 bench.py --weak --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-step-line >> gpurun_out/r05_xcd_lines.jsonl 2>>gpurun_out/r05_bench.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_xcd_$n -o run --output-format csv -- \
      python3 bench.py --weak --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-step-line > gpurun_out/r05_xcd_${n}_under_rocprof.json 2>>gpurun_out/r05_bench.err || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r05_xcd_lines.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(d["config"].get("envs_per_gpu"), round(r["kernel_ms"] * 1e3, 2), "us/step frac", round(r["frac"], 3))
PY
