# bench.py at the per-GPU env counts of config 3 strong-scaled to 1/2/4/8 GPUs (one GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r02}
: > gpurun_out/sizes_${TAG}.jsonl
for n in 131072 262144 524288 1048576; do
  timeout -k 10 200 python bench.py --weak --envs $n --no-cpu-baseline > gpurun_out/sizes_${TAG}_$n.log 2>&1 || exit 1
  grep -h '"metric"' gpurun_out/sizes_${TAG}_$n.log >> gpurun_out/sizes_${TAG}.jsonl
  tail -1 gpurun_out/sizes_${TAG}_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, round(d['ms_per_step']*1000,2), 'us', '%.3g' % d['value'])"
done
