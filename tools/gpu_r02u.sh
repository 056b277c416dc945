# DQN config 5: fused vs foreach Adam, alternating, twice
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for i in 1 2; do for f in 0 1; do LBK8S_FUSED_ADAM=$f $T 300 python tools/rl_bench.py --algo dqn > gpurun_out/u_dqn_$f$i.log 2>&1 || exit 1; grep -h "^{" gpurun_out/u_dqn_$f$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused', $f, d['value'], d['ms_per_vector_step'])"; done; done
