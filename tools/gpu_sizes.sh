#!/bin/bash
# bench.py at the strong-scaling shard sizes (1M envs over 1/2/4/8 GPUs), one GPU, both
# launch shapes per run -> gpurun_out/strong_sizes.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/strong_sizes.jsonl
for n in 131072 262144 524288 1048576; do
  timeout -k 10 200 python3 bench.py --weak --envs $n --no-cpu-baseline > gpurun_out/sizes_one.log 2>&1 || { cat gpurun_out/sizes_one.log; exit 1; }
  tail -1 gpurun_out/sizes_one.log >> gpurun_out/strong_sizes.jsonl
done
python3 - <<'PY'
import json
for l in open("gpurun_out/strong_sizes.jsonl"):
    d = json.loads(l)
    print(d["config"]["envs_per_gpu"], "rollout %.2f us (%.3e/s, frac %.3f)" % (d["roofline"]["kernel_ms"] * 1e3, d["value"], d["roofline"]["frac"]),
          "lb_step %.2f us (%.3e/s)" % (d["lb_step"]["kernel_ms"] * 1e3, d["lb_step"]["value"]))
PY
