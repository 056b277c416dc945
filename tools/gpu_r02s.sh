# Learner benchmarks (configs 4 and 5) + a kernel-trace summary of the PPO run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
TAG=${TAG:-r02}
$T 300 python tools/rl_bench.py --algo ppo --updates 2 > gpurun_out/rl_ppo_${TAG}.log 2>&1 || { tail -20 gpurun_out/rl_ppo_${TAG}.log; exit 1; }
$T 300 python tools/rl_bench.py --algo dqn > gpurun_out/rl_dqn_${TAG}.log 2>&1 || { tail -20 gpurun_out/rl_dqn_${TAG}.log; exit 1; }
$T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ppo_${TAG} -o run --output-format csv -- python3 tools/rl_bench.py --algo ppo --updates 1 > gpurun_out/rl_ppo_prof_${TAG}.log 2>&1 || exit 1
grep -h "^{" gpurun_out/rl_ppo_${TAG}.log gpurun_out/rl_dqn_${TAG}.log | cut -c1-600
head -12 gpurun_out/prof_ppo_${TAG}/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
