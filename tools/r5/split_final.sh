#!/bin/bash
# The product build with the split layout for short launches: lean parity (both layouts), the
# driver's bench line x2, and the shard sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r5/gpu_tests_lean.sh || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-step-line > /tmp/b.json 2>>gpurun_out/r05_bench.err || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print('k20', round(d['roofline']['kernel_ms']*1e3,2), 'frac', round(d['roofline']['frac'],3), d['roofline']['kernel'][:40])"
done
for n in 131072 262144; do
  timeout -k 10 300 python3 bench.py --weak --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-step-line > /tmp/b.json 2>>gpurun_out/r05_bench.err || exit 1
  python3 -c "import json;d=json.load(open('/tmp/b.json'));print($n, round(d['roofline']['kernel_ms']*1e3,2), 'frac', round(d['roofline']['frac'],3))"
done
