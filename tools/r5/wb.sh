#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 200 exp/wbench_sizes > gpurun_out/r05_wbench_rot.jsonl 2>&1; rc=$?
python3 - <<'PY'
import json
for l in open("gpurun_out/r05_wbench_rot.jsonl"):
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d["envs"], d["K"], d["us_per_step"], d["mean_us_per_step"], d["shape"])
PY
exit $rc
