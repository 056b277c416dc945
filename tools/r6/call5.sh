set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_prof_ppo -o run --output-format csv -- python3 tools/rl_bench.py --algo ppo --updates 2 > gpurun_out/r06_rl_bench_ppo.json 2> gpurun_out/r06_prof_ppo.err || exit 1
$T 300 python3 tools/train_bench.py --R 65,9 > gpurun_out/r06_train_bench.jsonl 2>> gpurun_out/r06_prof_ppo.err || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_prof_dqn -o run --output-format csv -- python3 tools/rl_bench.py --algo dqn > gpurun_out/r06_rl_bench_dqn.json 2> gpurun_out/r06_prof_dqn.err || exit 1
tail -n 2 gpurun_out/r06_rl_bench_ppo.json gpurun_out/r06_rl_bench_dqn.json gpurun_out/r06_train_bench.jsonl
