#!/bin/bash
# A/B session: bench.py's workload on the product library and on exp/ variants,
# interleaved, at the sizes in SIZES (env counts per GPU).  Usage (on the box):
#   LIBS="exp/liblbk8s_X.so ..." SIZES="1048576 131072" bash tools/gpu_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/ab.jsonl
: > $OUT
for rep in 1 2; do
 for n in ${SIZES:-1048576}; do
  for lib in gym-loadbalancing_amd/lbk8s/liblbk8s.so ${LIBS}; do
   timeout -k 10 120 python3 tools/abtest.py --lib $lib --weak --envs $n ${ABARGS} > gpurun_out/ab_one.log 2>&1 || { cat gpurun_out/ab_one.log; exit 1; }
   python3 - "$lib" "$n" >> $OUT <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab_one.log") if l.startswith("{")][-1]
d = json.loads(line)
print(json.dumps({"lib": sys.argv[1], "envs": int(sys.argv[2]), "kernel_us": d["roofline"]["kernel_ms"] * 1e3,
                  "ms_per_step": d["ms_per_step"], "value": d["value"]}))
PY
   tail -1 $OUT
  done
 done
done
