#!/bin/bash
# end of round 3: the whole GPU suite and smoke on the final build, config 5 A/B against the
# previous commit (exp/head) on this box, config 5's kernel summary, config 4's line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit 1
tail -1 gpurun_out/smoke_final.log
bash tools/gpu_dqn_ab.sh || exit 1
timeout -k 10 300 python tools/rl_bench.py --algo dqn > gpurun_out/rl_dqn_final.json 2>>gpurun_out/rl_err.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dqn_final -o run --output-format csv \
    -- python3 tools/rl_bench.py --algo dqn --steps 1000 > gpurun_out/prof_dqn_final.log 2>&1 || exit 1
timeout -k 10 400 python tools/rl_bench.py --algo ppo --config e64_multi > gpurun_out/rl_ppo_final.json 2>>gpurun_out/rl_err.log || exit 1
cut -c1-300 gpurun_out/rl_dqn_final.json gpurun_out/rl_ppo_final.json
