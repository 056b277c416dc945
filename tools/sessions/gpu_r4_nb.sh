#!/bin/bash
# lean kernel block size A/B: one-wave blocks (product, exp/liblbk8s_exp.so) vs 4-wave blocks
# (exp/liblbk8s_exp256.so), k_rollout_img as control; then the lean timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_lean.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lean2.log 2>&1 || { tail -60 gpurun_out/lean2.log; exit 1; }
tail -1 gpurun_out/lean2.log
: > gpurun_out/abnb.jsonl
for rep in 1 2 3; do
  timeout -k 10 150 python3 tools/roll_variants.py --lib exp/liblbk8s_exp.so --variants 0,1 --reps 1 --steps 20,100 >> gpurun_out/abnb.jsonl 2>gpurun_out/abnb_err.log || { cat gpurun_out/abnb_err.log; exit 1; }
  true
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/abnb.jsonl"):
    r = json.loads(l); agg[(r["lib"], r["variant"], r.get("kernel"), r["K"])].append(r["us_per_step"])
for k, v in sorted(agg.items(), key=str): print(k, v, "min", min(v))
PY
true
