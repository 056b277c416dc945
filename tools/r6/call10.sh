set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dqn_step.py tests/test_gpu_learners.py tests/test_gpu_fused.py > gpurun_out/r06_dqn_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r06_dqn_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/r06_dqn_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in exp/liblbk8s_split128.so gym-loadbalancing_amd/lbk8s/liblbk8s.so; do
    timeout -k 10 300 python3 tools/act_bench.py --vector-step --lib $lib >> $O 2>> gpurun_out/r06_dqn_ab.err || exit 1
    timeout -k 10 300 python3 tools/rl_bench.py --algo dqn --lib $lib >> $O 2>> gpurun_out/r06_dqn_ab.err || exit 1
  done
done
cat $O | cut -c1-400
