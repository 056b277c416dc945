#!/bin/bash
# Parity of the round's kernel changes (slice rollout, fused DQN step, learners), then A/Bs
# and the config-5 learner rate.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dqn_step.py \
    tests/test_gpu_learners.py tests/test_gpu_api.py tests/test_gpu_parity.py > gpurun_out/r05_combo2_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05_combo2_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/rl_bench.py --algo dqn > gpurun_out/r05_rl_bench_dqn.json 2>gpurun_out/r05_rl_dqn.err || exit 1
cut -c1-400 gpurun_out/r05_rl_bench_dqn.json
O=gpurun_out/r05_ab_e64b.jsonl
: > $O
for rep in 1 2; do
  for lib in exp/liblbk8s_base.so exp/liblbk8s_d1.so exp/liblbk8s_s64.so; do
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
bash tools/r5/ab_libs.sh r05_ab_prio.jsonl "131072 1048576" "20" exp/liblbk8s_s64.so exp/liblbk8s_noprio.so
