# A/B of step-kernel variants on bench.py's workload at several per-GPU env counts
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for n in ${SIZES}; do for i in 1 2; do for l in ${LIBS}; do
  $T 200 python tools/abtest.py --lib exp/$l.so --weak --envs $n ${ARGS} > gpurun_out/x_${l}_${n}_$i.log 2>&1 || exit 1
  grep -h '"metric"' gpurun_out/x_${l}_${n}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l', $n, $i, round(d['ms_per_step']*1000,2), 'us', round(d['roofline']['kernel_ms']*1000,2))"
done; done; done
