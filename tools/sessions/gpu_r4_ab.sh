#!/bin/bash
# Round-4 A/B session: the store-pattern experiments (exp/wbench2, tools/wbench2.hip) and an
# interleaved lb_rollout A/B of library builds (tools/roll_variants.py) on bench.py's workload.
#   LIBS="exp/a.so exp/b.so" [WB=1] [STEPS=100,20] bash tools/gpu_r4_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$WB" ]; then
  timeout -k 10 240 ./exp/wbench2 > gpurun_out/wbench2.jsonl 2>&1 || { echo "wbench2 failed"; cat gpurun_out/wbench2.jsonl; exit 1; }
  cat gpurun_out/wbench2.jsonl
fi
OUT=gpurun_out/abroll.jsonl
: > $OUT
for rep in ${REPS:-1 2 3}; do
  for lib in ${LIBS}; do
    timeout -k 10 150 python3 tools/roll_variants.py --lib $lib --variants ${VARIANTS:-0} --reps 1 --steps ${STEPS:-100,20} ${ABARGS} \
        >> $OUT 2> gpurun_out/abroll_err.log || { cat gpurun_out/abroll_err.log; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/abroll.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["lib"], r["variant"], r["K"])].append(r["us_per_step"])
for k, v in sorted(agg.items()):
    print(k, v, "min", min(v))
PY
