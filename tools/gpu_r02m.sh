set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for l in bwd_old bwd_lat; do $T 120 python tools/train_bench.py --lib exp/$l.so > gpurun_out/m_$l.json 2>&1 || exit 1; done
cat gpurun_out/m_*.json | grep sets
