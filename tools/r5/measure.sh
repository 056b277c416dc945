#!/bin/bash
# Round-5 measurement session of the product build: the driver's bench line (3 runs), its
# rocprofv3 kernel summary, the PMC traffic of 20- and 100-step launches, the strong-scaling
# shard sizes and the E = 64 config at the driver's window shape, smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 || { cat gpurun_out/r05_smoke.log; exit 1; }
tail -2 gpurun_out/r05_smoke.log
: > gpurun_out/r05_bench_k20.jsonl
for r in 1 2 3; do
  $T 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/r05_bench_k20.jsonl 2>>gpurun_out/r05_bench.err || exit 1
done
$T 400 python3 bench.py --steps 300 --warmup 100 --no-cpu-baseline > gpurun_out/r05_bench_k100.json 2>>gpurun_out/r05_bench.err || exit 1
$T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_bench -o run --output-format csv -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_bench_k20_under_rocprof.json 2>gpurun_out/r05_prof_bench.err || exit 1
for K in 20 100; do
  PMC_MODE=rollout PMC_K=$K timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r05_pmcf_k$K -o run \
      --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/r05_pmcf_k$K.log 2>&1 || exit 1
  PMC_MODE=rollout PMC_K=$K timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r05_pmcw_k$K -o run \
      --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/r05_pmcw_k$K.log 2>&1 || exit 1
  python3 tools/pmc_traffic.py gpurun_out/r05_pmcf_k$K/run_counter_collection.csv \
      gpurun_out/r05_pmcw_k$K/run_counter_collection.csv --envs 1048576 --steps-per-launch $K \
      --out gpurun_out/pmc_traffic_rollout_k$K.json || exit 1
done
: > gpurun_out/r05_strong_sizes_k20.jsonl
for n in 131072 262144 524288 1048576; do
  $T 300 python3 bench.py --weak --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-step-line >> gpurun_out/r05_strong_sizes_k20.jsonl 2>>gpurun_out/r05_bench.err || exit 1
done
for n in 131072 262144; do
  $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_shard_$n -o run --output-format csv -- \
      python3 bench.py --weak --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-step-line \
      > gpurun_out/r05_shard_${n}_under_rocprof.json 2>>gpurun_out/r05_bench.err || exit 1
done
$T 400 python3 bench.py --config e64_multi --steps 300 --warmup 100 --no-cpu-baseline > gpurun_out/r05_bench_e64.json 2>>gpurun_out/r05_bench.err || exit 1
python3 - <<'PY'
import json
def show(tag, d):
    r = d["roofline"]
    print(tag, d["config"].get("envs_per_gpu"), round(r["kernel_ms"] * 1e3, 2), "us/step", f'{d["value"]:.3e}', "frac", round(r["frac"], 3), r["kernel"].split()[0])
for l in open("gpurun_out/r05_bench_k20.jsonl"): show("k20", json.loads(l))
show("k100", json.load(open("gpurun_out/r05_bench_k100.json")))
for l in open("gpurun_out/r05_strong_sizes_k20.jsonl"): show("shard", json.loads(l))
show("e64", json.load(open("gpurun_out/r05_bench_e64.json")))
for K in (20, 100): print("pmc", K, open(f"gpurun_out/pmc_traffic_rollout_k{K}.json").read()[:300])
PY
