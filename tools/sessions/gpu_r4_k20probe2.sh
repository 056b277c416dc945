set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/k20probe2.txt
: > $O
P='import json,sys
for l in sys.stdin: d=json.loads(l); print(sys.argv[1], d["us_per_step"])'
for mode in "" "--graph" "--stats-before" "--graph --stats-before"; do
  timeout -k 10 200 python3 tools/roll_variants.py --variants 0 --reps 3 --steps 20 --launches 1 $mode 2>>gpurun_out/k20probe2.err | python3 -c "$P" "roll1 [$mode]" >> $O || exit 1
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-step-line 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench k20', d['roofline']['kernel_ms']*1e3)" >> $O
cat $O
