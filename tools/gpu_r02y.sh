# kernel-trace stats of bench.py at several per-GPU env counts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in ${SIZES}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/y_$n -o run --output-format csv \
    -- python3 bench.py --weak --envs $n --steps 300 --no-cpu-baseline ${ARGS} > gpurun_out/y_$n.log 2>&1 || exit 1
  echo "== $n"; tail -1 gpurun_out/y_$n.log | cut -c1-200
  head -5 gpurun_out/y_$n/run_kernel_stats.csv | cut -d, -f1-4
done
