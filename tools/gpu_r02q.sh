# Wave-contiguous obs stores in the slice step: parity, E=64 write bytes, step time A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_api.py > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
$T 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/q_w_obs -o run --output-format csv -- python3 tools/pmc_probe.py e64_multi > gpurun_out/q_w_obs.log 2>&1 || exit 1
python3 - gpurun_out/q_w_obs/run_counter_collection.csv <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_step" in r["Kernel_Name"]]
v = [float(r["Counter_Value"]) * 1024 for r in rows][-13:]
print("obs-wave write B/env-step", statistics.median(v) / (1 << 20))
PY
for i in 1 2; do
$T 200 python tools/kbench.py --configs e64_multi,cfg1 --sizes 12,15,17,20 --lib exp/bwd_il5.so > gpurun_out/q_kb_base$i.log 2>&1 || exit 1
$T 200 python tools/kbench.py --configs e64_multi,cfg1 --sizes 12,15,17,20 > gpurun_out/q_kb_obs$i.log 2>&1 || exit 1
done
grep -h "^{" gpurun_out/q_kb_*.log | cut -c1-200
