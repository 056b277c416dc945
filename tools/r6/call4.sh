set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gym-loadbalancing_amd/lbk8s/liblbk8s.so
bash tools/gpu_session.sh ab r06_ab_diag.jsonl "131072 1048576" "20" $P exp/liblbk8s_mr.so exp/liblbk8s_noepi.so exp/liblbk8s_norec.so exp/liblbk8s_allthree.so || exit 1
for n in 131072 1048576; do timeout -k 10 150 python3 tools/roll_variants.py --envs $n --steps 20 --variants 0 --reps 3 --launches 1 --lockstep >> gpurun_out/r06_ab_diag_lockstep.jsonl 2>>gpurun_out/r06_ab_diag.jsonl.err || exit 1; done
python3 -c "
import json
for l in open('gpurun_out/r06_ab_diag_lockstep.jsonl'): r=json.loads(l); print('lockstep', r['envs'], r['us_per_step'])"
