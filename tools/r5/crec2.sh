#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/ab_libs.sh r05_ab_crec2.jsonl "131072 131072 262144 1048576" 20 exp/liblbk8s_cur.so exp/liblbk8s_crec.so
