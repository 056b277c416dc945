set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r06_train_ab.jsonl
: > $O
for rep in 1 2 3; do
  for lib in exp/liblbk8s_ds0.so gym-loadbalancing_amd/lbk8s/liblbk8s.so; do
    timeout -k 10 300 python3 tools/train_bench.py --R 65,9 --lib $lib >> $O 2>> gpurun_out/r06_train_ab.err || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r06_train_ab.jsonl"):
    r = json.loads(l); d[(r["R"], r["lib"])].append((r["fwd_ms"], r["bwd_ms"]))
for k in sorted(d): print(k, d[k])
PY
