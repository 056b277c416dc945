set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_fused_train.py tests/test_gpu_learners.py tests/test_eval_golden.py tests/test_gpu_dist.py > gpurun_out/r06_ds_tests2.log 2>&1; rc=$?; tail -n 5 gpurun_out/r06_ds_tests2.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/r06_ppo_ab.jsonl
: > $O
for rep in 1 2; do
  timeout -k 10 300 python3 tools/rl_bench.py --algo ppo --updates 2 --torch-set-sums >> $O 2>> gpurun_out/r06_ppo_ab.err || exit 1
  timeout -k 10 300 python3 tools/rl_bench.py --algo ppo --updates 2 >> $O 2>> gpurun_out/r06_ppo_ab.err || exit 1
done
python3 -c "
import json
for l in open('$O'): r=json.loads(l); print(r['set_sums'], round(r['value']), round(r['update_ms'],2), round(r['rollout_ms'],2))"
