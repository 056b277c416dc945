#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/r5/e64_ab.sh exp/liblbk8s_base.so exp/liblbk8s_d1.so exp/liblbk8s_s64.so || exit 1
bash tools/r5/ab_libs.sh r05_ab_prio.jsonl "131072 1048576" "20" exp/liblbk8s_s64.so exp/liblbk8s_noprio.so
