set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/k20probe3.txt
: > $O
P='import json,sys
for l in sys.stdin: d=json.loads(l); print(sys.argv[1], d["us_per_step"])'
B='import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["roofline"]["kernel_ms"]*1e3,2), round(d["roofline"]["frac"],4), d["config"]["resets_in_window"])'
for r in 1 2 3; do
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-step-line 2>/dev/null | python3 -c "$B" "bench k20 graph" >> $O || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-step-line --no-graph 2>/dev/null | python3 -c "$B" "bench k20 nograph" >> $O || exit 1
done
timeout -k 10 200 python3 tools/roll_variants.py --variants 0 --reps 3 --steps 20 --launches 1 2>>gpurun_out/k20probe3.err | python3 -c "$P" "roll1" >> $O || exit 1
cat $O
