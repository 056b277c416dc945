# E=64 write-excess probe: WRITE_SIZE of the slice step, stock build vs no edyn stores
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/p_w_base -o run --output-format csv -- python3 tools/pmc_probe.py e64_multi > gpurun_out/p_w_base.log 2>&1 || exit 1
PMC_LIB=exp/e64_noed.so $T 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/p_w_noed -o run --output-format csv -- python3 tools/pmc_probe.py e64_multi > gpurun_out/p_w_noed.log 2>&1 || exit 1
for d in p_w_base p_w_noed; do python3 - gpurun_out/$d/run_counter_collection.csv <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_step" in r["Kernel_Name"]]
v = [float(r["Counter_Value"]) * 1024 for r in rows][-13:]
print(sys.argv[1], rows[0]["Kernel_Name"][:40], "write B/env-step", statistics.median(v) / (1 << 20))
PY
done
