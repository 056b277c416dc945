#!/bin/bash
# GPU session steps (run under gpurun from the repo root; chain steps with &&):
#   tools/gpu_session.sh STEP [args...]
#
#   suite                      the whole GPU test suite (product build)      -> gpurun_out/gpu_suite.log
#   smoke                      __graft_entry__.smoke()
#   lean-tests [LIB]           k_rollout_lean parity (C oracle; lb_policy + lb_step) on a build
#   ab OUT "ENVS" "KS" LIB...  interleaved A/B of rollout builds: one process per (build, size),
#                              alternated twice, us per step                  -> gpurun_out/OUT
#   bench OUT [ARGS]           bench.py lines (default: the driver's command) -> gpurun_out/OUT
#   prof OUT [ARGS]            rocprofv3 --kernel-trace --stats of bench.py   -> gpurun_out/OUT/
#   pmc TAG K                  HBM traffic of K-step launches: FETCH_SIZE and WRITE_SIZE passes of
#                              tools/pmc_probe.py, corrected by tools/pmc_traffic.py
#                                                                             -> gpurun_out/pmc_traffic_rollout_kK.json
#   sizes TAG                  the strong-scaling shard sizes at the driver's window, and rocprof
#                              summaries at 131,072 / 262,144                  -> gpurun_out/TAG_strong_sizes_k20.jsonl
#   learners TAG               config 4 (PPO) and config 5 (DQN) learner benches, training-step bench
#   sq TAG K [LIB]             SQ counters (two passes) of K-step lb_rollout launches, per wave-step
#   measure TAG                the round's measurement of the product build: smoke, the driver's
#                              line x3, K = 100, rocprof of the driver command, PMC at K = 20 / 100,
#                              shard sizes, the E = 64 config
#
# Every GPU step runs under its own time limit; a failed step ends the session (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
step=$1; shift
case $step in
  suite)
    $T 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests "$@" \
      > gpurun_out/gpu_suite.log 2>&1
    rc=$?; tail -n 15 gpurun_out/gpu_suite.log; exit $rc ;;
  smoke)
    $T 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
  lean-tests)
    lib=${1:-gym-loadbalancing_amd/lbk8s/liblbk8s.so}; shift || true
    log=gpurun_out/lean_tests_$(basename $lib .so).log
    $T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread --lib "$lib" \
      tests/test_gpu_lean_oracle.py tests/test_gpu_lean.py "$@" > $log 2>&1
    rc=$?; tail -n 5 $log; exit $rc ;;
  ab)
    O=gpurun_out/$1; ENVS=$2; KS=$3; shift 3
    : > $O
    for rep in 1 2; do for n in $ENVS; do for lib in "$@"; do
      $T 150 python3 tools/roll_variants.py --lib $lib --envs $n --steps $KS --variants 0 --reps 2 \
        --launches 1 >> $O 2>>$O.err || exit 1
    done; done; done
    python3 - $O <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[(r["envs"], r["K"], r["lib"])].append(r["us_per_step"])
for k in sorted(d): print(k, [round(x, 2) for x in d[k]], "min", round(min(d[k]), 2), "med", round(sorted(d[k])[len(d[k]) // 2], 2))
PY
    ;;
  bench)
    O=gpurun_out/$1; shift
    [ $# -eq 0 ] && set -- --gpus 1 --steps 20 --warmup 5
    $T 400 python3 bench.py "$@" >> $O 2>>$O.err; rc=$?; tail -n 1 $O | cut -c1-300; exit $rc ;;
  prof)
    O=gpurun_out/$1; shift
    [ $# -eq 0 ] && set -- --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
    $T 400 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 bench.py "$@" \
      > $O.json 2>$O.err
    rc=$?; tail -n 1 $O.json | cut -c1-300; exit $rc ;;
  pmc)
    TAG=$1; K=$2
    PMC_MODE=rollout PMC_K=$K timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_pmcf_k$K \
      -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/${TAG}_pmcf_k$K.log 2>&1 || exit 1
    PMC_MODE=rollout PMC_K=$K timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_pmcw_k$K \
      -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/${TAG}_pmcw_k$K.log 2>&1 || exit 1
    python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmcf_k$K/run_counter_collection.csv \
      gpurun_out/${TAG}_pmcw_k$K/run_counter_collection.csv --envs 1048576 --steps-per-launch $K \
      --out gpurun_out/pmc_traffic_rollout_k$K.json ;;
  sizes)
    TAG=$1
    : > gpurun_out/${TAG}_strong_sizes_k20.jsonl
    for n in 131072 262144 524288 1048576; do
      $T 300 python3 bench.py --weak --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-step-line \
        >> gpurun_out/${TAG}_strong_sizes_k20.jsonl 2>>gpurun_out/${TAG}_sizes.err || exit 1
    done
    for n in 131072 262144; do
      $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_shard_$n -o run --output-format csv -- \
        python3 bench.py --weak --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-step-line \
        > gpurun_out/${TAG}_shard_${n}_under_rocprof.json 2>>gpurun_out/${TAG}_sizes.err || exit 1
    done ;;
  learners)
    TAG=$1
    $T 300 python3 tools/rl_bench.py --algo ppo --updates 2 > gpurun_out/${TAG}_rl_bench_ppo.json 2>>gpurun_out/${TAG}_rl.err || exit 1
    $T 300 python3 tools/rl_bench.py --algo dqn > gpurun_out/${TAG}_rl_bench_dqn.json 2>>gpurun_out/${TAG}_rl.err || exit 1
    $T 300 python3 tools/train_bench.py --R 65,9 > gpurun_out/${TAG}_train_bench.jsonl 2>>gpurun_out/${TAG}_rl.err || exit 1
    tail -n 1 gpurun_out/${TAG}_rl_bench_ppo.json gpurun_out/${TAG}_rl_bench_dqn.json | cut -c1-300 ;;
  sq)
    TAG=$1; K=$2; lib=${3:-gym-loadbalancing_amd/lbk8s/liblbk8s.so}
    PMC_LIB=$lib PMC_MODE=rollout PMC_K=$K timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace \
      -d gpurun_out/${TAG}_sqa_k$K -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/${TAG}_sqa_k$K.log 2>&1 || exit 1
    PMC_LIB=$lib PMC_MODE=rollout PMC_K=$K timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM --kernel-trace \
      -d gpurun_out/${TAG}_sqb_k$K -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/${TAG}_sqb_k$K.log 2>&1 || exit 1
    for z in sqa sqb; do python3 tools/pmc_sum.py gpurun_out/${TAG}_${z}_k$K/run_counter_collection.csv k_rollout; done ;;
  measure)
    TAG=$1
    $T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
    tail -n 3 gpurun_out/${TAG}_smoke.log
    : > gpurun_out/${TAG}_bench_k20.jsonl
    for r in 1 2 3; do
      $T 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/${TAG}_bench_k20.jsonl 2>>gpurun_out/${TAG}_bench.err || exit 1
    done
    $T 400 python3 bench.py --steps 300 --warmup 100 --no-cpu-baseline > gpurun_out/${TAG}_bench_k100.json 2>>gpurun_out/${TAG}_bench.err || exit 1
    $T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_bench -o run --output-format csv -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_k20_under_rocprof.json \
      2>gpurun_out/${TAG}_prof_bench.err || exit 1
    bash "$0" pmc $TAG 20 && bash "$0" pmc $TAG 100 && bash "$0" sizes $TAG || exit 1
    $T 400 python3 bench.py --config e64_multi --steps 300 --warmup 100 --no-cpu-baseline > gpurun_out/${TAG}_bench_e64.json 2>>gpurun_out/${TAG}_bench.err || exit 1
    python3 - $TAG <<'PY'
import json, sys
tag = sys.argv[1]
def show(t, d):
    r = d["roofline"]
    print(t, d["config"].get("envs_per_gpu"), round(r["kernel_ms"] * 1e3, 2), "us/step", f'{d["value"]:.3e}', "frac", round(r["frac"], 3), r["kernel"].split()[0])
for l in open(f"gpurun_out/{tag}_bench_k20.jsonl"): show("k20", json.loads(l))
show("k100", json.load(open(f"gpurun_out/{tag}_bench_k100.json")))
for l in open(f"gpurun_out/{tag}_strong_sizes_k20.jsonl"): show("shard", json.loads(l))
show("e64", json.load(open(f"gpurun_out/{tag}_bench_e64.json")))
for K in (20, 100): print("pmc", K, open(f"gpurun_out/pmc_traffic_rollout_k{K}.json").read()[:300])
PY
    ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
