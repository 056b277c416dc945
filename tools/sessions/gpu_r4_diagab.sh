#!/bin/bash
# Interleaved A/B of diagnostic lean builds (exp/): the current build, without the episode-
# statistics row, without the row and the terminal observations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/diagab.jsonl
: > $O
for rep in 1 2 3; do
  for lib in ${LIBS:-exp/liblbk8s_cur.so exp/liblbk8s_nostats.so exp/liblbk8s_nostatsterm.so}; do
    timeout -k 10 150 python3 tools/roll_variants.py --lib $lib --variants 0 --reps 1 --steps ${STEPS:-20,100} >> $O 2>gpurun_out/diagab.err || { cat gpurun_out/diagab.err; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/diagab.jsonl"):
    r = json.loads(l); agg[(r["lib"], r["K"])].append(r["us_per_step"])
for k, v in sorted(agg.items(), key=str): print(k, v, "min", min(v))
PY
