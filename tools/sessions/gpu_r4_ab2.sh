set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab2.jsonl
for rep in 1 2 3; do
  timeout -k 10 150 python3 tools/roll_variants.py --lib exp/liblbk8s_base.so --variants 0 --reps 1 --steps 20,100 >> gpurun_out/ab2.jsonl 2>gpurun_out/ab2_err.log || { cat gpurun_out/ab2_err.log; exit 1; }
  timeout -k 10 150 python3 tools/roll_variants.py --lib exp/liblbk8s_exp.so --variants 0,1 --reps 1 --steps 20,100 >> gpurun_out/ab2.jsonl 2>gpurun_out/ab2_err.log || { cat gpurun_out/ab2_err.log; exit 1; }
done
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab2.jsonl"):
    r = json.loads(l); agg[(r["lib"], r["variant"], r.get("kernel"), r["K"])].append(r["us_per_step"])
for k, v in sorted(agg.items(), key=str): print(k, v, "min", min(v))
PY
