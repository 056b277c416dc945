#!/bin/bash
# k_dqn_step P = 4 vs P = 2: kernel summaries of the config-5 learner, then longer alternating runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-loadbalancing_amd/lbk8s/liblbk8s.so
cp $L /tmp/lib_p4.so
for v in p4 p2; do
  if [ $v = p4 ]; then cp /tmp/lib_p4.so $L; else cp exp/liblbk8s_dqnp2.so $L; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dqn_$v -o run --output-format csv \
      -- python3 tools/rl_bench.py --algo dqn --envs 4096 --steps 1000 > gpurun_out/prof_dqn_$v.log 2>&1 || exit 1
  echo "== $v"; head -4 gpurun_out/prof_dqn_$v/run_kernel_stats.csv | cut -c1-150
done
: > gpurun_out/r05_rl_dqn_p2b.jsonl
for v in p4 p2 p4 p2 p4 p2; do
  if [ $v = p4 ]; then cp /tmp/lib_p4.so $L; else cp exp/liblbk8s_dqnp2.so $L; fi
  timeout -k 10 200 python tools/rl_bench.py --algo dqn --envs 4096 --steps 6000 > /tmp/o.json 2>gpurun_out/rl_dqn_err.log || { tail -20 gpurun_out/rl_dqn_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('/tmp/o.json'));d['variant']='$v';print(json.dumps(d))" >> gpurun_out/r05_rl_dqn_p2b.jsonl
  echo $v $(python3 -c "import json;print(json.load(open('/tmp/o.json'))['value'])")
done
cp /tmp/lib_p4.so $L
