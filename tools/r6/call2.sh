set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/timeline_lean.py --lib exp/liblbk8s_tl.so --envs 131072 --steps 20 > gpurun_out/r06_timeline_split_131072.jsonl 2>gpurun_out/r06_tl.err &&
timeout -k 10 200 python3 tools/timeline_lean.py --lib exp/liblbk8s_tl.so --envs 1048576 --steps 20 > gpurun_out/r06_timeline_split_1m.jsonl 2>>gpurun_out/r06_tl.err &&
for n in 131072 1048576; do for m in "" "--lockstep"; do timeout -k 10 150 python3 tools/roll_variants.py --envs $n --steps 20 --variants 0 --reps 3 --launches 1 $m >> gpurun_out/r06_lockstep.jsonl 2>>gpurun_out/r06_lockstep.err || exit 1; done; done &&
bash tools/gpu_session.sh suite && bash tools/gpu_session.sh smoke
