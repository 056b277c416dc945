set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/k20probe.txt
: > $O
for i in 1 2; do timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-step-line 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench k20', d['roofline']['kernel_ms']*1e3, d['roofline']['frac'])" >> $O; done
timeout -k 10 200 python3 tools/roll_variants.py --variants 0 --reps 2 --steps 20 --launches 1 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('roll launches=1', d['us_per_step'])" >> $O
timeout -k 10 200 python3 tools/roll_variants.py --variants 0 --reps 2 --steps 20 --launches 3 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('roll launches=3', d['us_per_step'])" >> $O
timeout -k 10 200 python3 tools/roll_variants.py --variants 0 --reps 2 --steps 100 --launches 3 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('roll k100 launches=3', d['us_per_step'])" >> $O
cat $O
