set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 131072 1048576; do for m in "" "--lockstep"; do
  timeout -k 10 200 python3 tools/timeline_lean.py --lib exp/liblbk8s_tl.so --envs $n --steps 20 $m >> gpurun_out/r06_timeline_lockstep_vs_stagger.jsonl 2>>gpurun_out/r06_tl3.err || exit 1
done; done
bash tools/gpu_session.sh suite && bash tools/gpu_session.sh smoke
