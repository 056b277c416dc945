#!/bin/bash
# lb_ds_set_grads: the training/learner GPU tests, config 5's rl_bench and its kernel summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fused or dqn or learner or native or asan" > gpurun_out/pt_sg.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/pt_sg.log; exit 1; }
tail -2 gpurun_out/pt_sg.log
for r in 1 2; do
  timeout -k 10 300 python tools/rl_bench.py --algo dqn 2>>gpurun_out/rl_sg_err.log | tail -1 || exit 1
done > gpurun_out/rl_dqn_sg.jsonl
cut -c1-330 gpurun_out/rl_dqn_sg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dqn_sg -o run --output-format csv \
    -- python3 tools/rl_bench.py --algo dqn --steps 1000 > gpurun_out/prof_dqn_sg.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_dqn_sg/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/prof_dqn_sg/run_kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
for r in rows[:22]:
    print(r["Calls"].rjust(6), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(7), r["Name"][:100])
PY
