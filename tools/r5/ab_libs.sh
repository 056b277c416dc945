#!/bin/bash
# Interleaved A/B across builds: each library in its own process, alternated, same box.
#   tools/r5/ab_libs.sh OUT "ENVS..." "K list" lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/$1; shift
ENVS=$1; shift
KS=$1; shift
: > $O
for rep in 1 2; do
  for n in $ENVS; do
    for lib in "$@"; do
      timeout -k 10 150 python3 tools/roll_variants.py --lib $lib --envs $n --steps $KS --variants 0 --reps 2 --launches 1 >> $O 2>>$O.err || exit 1
    done
  done
done
python3 - $O <<'PY'
import json,sys,collections
d=collections.defaultdict(list)
for l in open(sys.argv[1]):
    r=json.loads(l); d[(r["envs"],r["K"],r["lib"])].append(r["us_per_step"])
for k in sorted(d): print(k, [round(x,2) for x in d[k]], round(min(d[k]),2))
PY
