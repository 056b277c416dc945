#!/bin/bash
# E = 64 rollout: its parity tests on the product build, then base / previous / product A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "e64 or slice or rollout or Rollout" > gpurun_out/r05_e64_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05_e64_tests.log
[ $rc -eq 0 ] || exit $rc
O=gpurun_out/r05_ab_e64b.jsonl
: > $O
for rep in 1 2; do
  for lib in "$@"; do
    timeout -k 10 200 python3 tools/roll_variants.py --lib $lib --config e64_multi --envs 1048576 --steps 100,20 --variants 0 --reps 1 --launches 1 >> $O 2>>$O.err || exit 1
  done
done
python3 - $O <<'PY'
import json,sys,collections
d=collections.defaultdict(list)
for l in open(sys.argv[1]):
    r=json.loads(l); d[(r["K"],r["lib"])].append(r["us_per_step"])
for k in sorted(d): print(k, d[k])
PY
