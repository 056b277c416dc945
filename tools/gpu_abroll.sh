#!/bin/bash
# Interleaved A/B of lb_rollout builds on bench.py's staggered workload (tools/roll_variants.py,
# variant 0 = the product dispatch of each build), optionally after the GPU test suite.
#   LIBS="exp/liblbk8s_base.so gym-loadbalancing_amd/lbk8s/liblbk8s.so" [TESTS=1] bash tools/gpu_abroll.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/abroll.jsonl
: > $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu_ab.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_ab.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_ab.log
fi
for rep in ${REPS:-1 2 3}; do
  for lib in ${LIBS}; do
    timeout -k 10 150 python3 tools/roll_variants.py --lib $lib --variants 0 --reps 1 --steps ${STEPS:-100,20} ${ABARGS} \
        >> $OUT 2> gpurun_out/abroll_err.log || { cat gpurun_out/abroll_err.log; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/abroll.jsonl")]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["lib"], r["K"])].append(r["us_per_step"])
for k, v in sorted(agg.items()):
    print(k, v, "min", min(v))
PY
