#!/bin/bash
# The DQN vector step's launches (fused vs three), the config-5 kernel summary, and the lean
# kernel's SQ counters at the driver's K = 20 (round-start build vs this build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/act_bench.py --vector-step --envs 4096 --reps 5 > gpurun_out/r05_dqn_vstep.jsonl 2>gpurun_out/r05_dqn_vstep.err || exit 1
cut -c1-200 gpurun_out/r05_dqn_vstep.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_dqn -o run --output-format csv -- python3 tools/rl_bench.py --algo dqn --steps 1000 --warmup 200 > gpurun_out/r05_prof_dqn.log 2>&1 || exit 1
tail -2 gpurun_out/r05_prof_dqn.log | cut -c1-300
LIBS="exp/liblbk8s_base.so gym-loadbalancing_amd/lbk8s/liblbk8s.so" KS=20 timeout -k 10 400 bash tools/gpu_sq.sh > gpurun_out/r05_sq.txt 2>&1
rc=$?
cat gpurun_out/r05_sq.txt | cut -c1-600
exit $rc
