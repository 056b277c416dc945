#!/bin/bash
# Round-4 re-timing of the other BASELINE configs on the current build: config 2 (4096 envs),
# config 1 (run_baselines workload), lb_step per scenario and size (E=64 slice included), and
# bench.py's rollout line for the cfg1 / e64_multi scenarios.  Each GPU step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r04_configs.jsonl
: > $O
timeout -k 10 200 python3 tools/kbench.py --config2 >> $O 2> gpurun_out/r04_configs.err \
&& timeout -k 10 200 python3 tools/kbench.py --config1 >> $O 2>> gpurun_out/r04_configs.err \
&& timeout -k 10 300 python3 tools/kbench.py --configs default,cfg1,e64_multi --sizes 16,18,20 >> $O 2>> gpurun_out/r04_configs.err \
&& timeout -k 10 300 python3 bench.py --config cfg1 --no-cpu-baseline >> $O 2>> gpurun_out/r04_configs.err \
&& timeout -k 10 300 python3 bench.py --config e64_multi --no-cpu-baseline >> $O 2>> gpurun_out/r04_configs.err
rc=$?
cut -c1-300 $O
exit $rc
