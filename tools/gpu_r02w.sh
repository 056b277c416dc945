# A/B of step-kernel variants on bench.py's workload (alternating, twice)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for i in 1 2; do for l in ${LIBS}; do $T 200 python tools/abtest.py --lib exp/$l.so ${ARGS} > gpurun_out/w_${l}_$i.log 2>&1 || exit 1; grep -h '"metric"' gpurun_out/w_${l}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l', $i, round(d['ms_per_step']*1000,2), 'us', d['roofline']['kernel_ms'])"; done; done
