#!/bin/bash
# The whole GPU suite on the product build, then interleaved A/Bs of candidate builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05_gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r05_gpu_suite.log
[ $rc -eq 0 ] || exit $rc
O=gpurun_out/r05_ab_e64.jsonl
: > $O
for rep in 1 2; do
  for lib in exp/liblbk8s_base.so exp/liblbk8s_d1.so; do
    timeout -k 10 200 python3 tools/roll_variants.py --lib $lib --config e64_multi --envs 1048576 --steps 100,20 --variants 0 --reps 1 --launches 1 >> $O 2>>$O.err || exit 1
  done
done
cut -c1-200 $O
O=gpurun_out/r05_ab_act.jsonl
: > $O
for rep in 1 2; do
  for lib in exp/liblbk8s_d1.so exp/liblbk8s_ds2.so; do
    for n in 2048 4096 8192; do
      timeout -k 10 120 python3 tools/act_bench.py --lib $lib --envs $n --reps 3 >> $O 2>>$O.err || exit 1
    done
  done
done
cut -c1-160 $O
