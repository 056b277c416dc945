#!/bin/bash
# Round-6 GPU session steps, one parameterised script (run under gpurun from the repo root).
#   tools/r6/session.sh STEP [args...]; steps chain with && in the gpurun command.
#   lean-tests LIB      k_rollout_lean parity (C oracle + lb_policy/lb_step) on a build
#   ab OUT "ENVS" "KS" LIB...   interleaved A/B of rollout builds (one process per build, alternated)
#   suite               the whole GPU test suite on the product build
#   smoke               __graft_entry__.smoke()
#   bench OUT [args]    bench.py line(s) into gpurun_out/OUT
#   prof OUT [args]     rocprofv3 --kernel-trace --stats of bench.py [args] into gpurun_out/OUT/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step=$1; shift
case $step in
  lean-tests)
    lib=$1; shift
    timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread --lib "$lib" \
      tests/test_gpu_lean_oracle.py tests/test_gpu_lean.py "$@" > gpurun_out/lean_tests_$(basename $lib .so).log 2>&1
    rc=$?; tail -n 5 gpurun_out/lean_tests_$(basename $lib .so).log; exit $rc ;;
  ab)
    O=gpurun_out/$1; ENVS=$2; KS=$3; shift 3
    : > $O
    for rep in 1 2; do for n in $ENVS; do for lib in "$@"; do
      timeout -k 10 150 python3 tools/roll_variants.py --lib $lib --envs $n --steps $KS --variants 0 --reps 2 \
        --launches 1 >> $O 2>>$O.err || exit 1
    done; done; done
    python3 - $O <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[(r["envs"], r["K"], r["lib"])].append(r["us_per_step"])
for k in sorted(d): print(k, [round(x, 2) for x in d[k]], "min", round(min(d[k]), 2), "med", round(sorted(d[k])[len(d[k]) // 2], 2))
PY
    ;;
  suite)
    timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests "$@" \
      > gpurun_out/gpu_suite.log 2>&1
    rc=$?; tail -n 15 gpurun_out/gpu_suite.log; exit $rc ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
  bench)
    O=gpurun_out/$1; shift
    timeout -k 10 300 python3 bench.py "$@" >> $O 2>>$O.err; rc=$?; tail -n 1 $O; exit $rc ;;
  prof)
    O=gpurun_out/$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run -- python3 bench.py "$@" > $O.log 2>&1
    rc=$?; tail -n 2 $O.log; exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
