#!/bin/bash
# Lean SALU cut (FAST-bound restart loops, paired request draws): parity tests, A/B vs the
# previous build, SQ counters at K = 20.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/gpu_tests_lean.sh && \
bash tools/r5/ab_libs.sh r05_ab_salu.jsonl "131072 1048576" 20 exp/liblbk8s_s64.so exp/liblbk8s_salu.so && \
LIBS="exp/liblbk8s_s64.so exp/liblbk8s_salu.so" KS=20 bash tools/gpu_sq.sh > gpurun_out/r05_sq_salu.txt 2>&1
rc=$?
cat gpurun_out/r05_sq_salu.txt
exit $rc
