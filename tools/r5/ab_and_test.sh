#!/bin/bash
# A/B of candidate builds (interleaved processes) and the lean parity tests on the product build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=$1; shift
ENVS=$1; shift
KS=$1; shift
bash tools/r5/gpu_tests_lean.sh -k "oracle or staggered" || exit 1
bash tools/r5/ab_libs.sh $OUT "$ENVS" "$KS" "$@"
