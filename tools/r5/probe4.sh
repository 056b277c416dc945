#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/r5/probe_tl.sh > /dev/null || exit 1
bash tools/r5/ab_libs.sh r05_ab_rec.jsonl "131072 1048576" "20" exp/liblbk8s_base.so exp/liblbk8s_n4.so exp/liblbk8s_n3.so exp/liblbk8s_n2.so
