#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 200 exp/wbench_k > gpurun_out/r05_wbench_k.jsonl 2>&1; rc=$?
cat gpurun_out/r05_wbench_k.jsonl
exit $rc
