#!/bin/bash
# config 5 with the period graphs captured before the timed learn() (rl_bench default now) and
# without (rounds 3-4's timing), on the current build; the learner parity tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learners.py \
    -k "dqn" > gpurun_out/r05_dqn_prep_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05_dqn_prep_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r05_rl_dqn_prep.jsonl
for p in 1 0 1 0 1 0; do
  LBK8S_BENCH_PREPARE=$p timeout -k 10 200 python tools/rl_bench.py --algo dqn --envs 4096 >> gpurun_out/r05_rl_dqn_prep.jsonl 2>gpurun_out/rl_dqn_err.log || { tail -20 gpurun_out/rl_dqn_err.log; exit 1; }
  echo prep=$p $(tail -1 gpurun_out/r05_rl_dqn_prep.jsonl | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['ms_per_vector_step'])")
done
