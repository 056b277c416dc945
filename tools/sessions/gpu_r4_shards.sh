#!/bin/bash
# Per-GPU time at the driver's window for the strong-scaling shard sizes of the 8-GPU node
# (one GPU, bench.py --weak --envs n --steps 20 --warmup 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r04_strong_sizes_k20.jsonl
: > $O
for n in 131072 262144 524288 1048576; do
  timeout -k 10 200 python3 bench.py --weak --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-step-line >> $O 2>>gpurun_out/r04_shards.err || exit 1
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r04_strong_sizes_k20.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(d["config"]["envs_per_gpu"], r["kernel"].split()[0], round(r["kernel_ms"] * 1e3, 2), "us/step", f'{d["value"]:.3e}', round(r["frac"], 3))
PY
