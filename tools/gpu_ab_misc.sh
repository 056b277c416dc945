set -o pipefail
for r in 1 2; do for lib in exp/liblbk8s_c4.so gym-loadbalancing_amd/lbk8s/liblbk8s.so; do timeout -k 10 200 python tools/train_bench.py --R 65,9 --iters 20 --lib $lib 2>/dev/null | tail -2; done; done > gpurun_out/tb2.jsonl; cut -c1-150 gpurun_out/tb2.jsonl
REPS="1 2" LIBS="gym-loadbalancing_amd/lbk8s/liblbk8s.so exp/liblbk8s_ntrd.so" bash tools/gpu_abroll.sh
