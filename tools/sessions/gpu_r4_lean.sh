#!/bin/bash
# Round-4 lean-kernel session: its GPU tests, then an in-process A/B of k_rollout_lean
# (variant 0) against k_rollout_img (variant 1) on bench.py's workload (exp/liblbk8s_exp.so,
# a -DLB_EXPERIMENTS build of the same sources).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_lean.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lean2.log 2>&1 || { tail -60 gpurun_out/lean2.log; exit 1; }
tail -3 gpurun_out/lean2.log
LIBS="exp/liblbk8s_exp.so" VARIANTS=0,1 STEPS=20,100 bash tools/gpu_r4_ab.sh
