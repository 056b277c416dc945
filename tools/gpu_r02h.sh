set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_r02.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_bwd1 -o run --output-format csv -- python3 tools/train_bench.py --R 65 --iters 3 > gpurun_out/pmc_bwd1.log 2>&1
rc1=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc_bwd2 -o run --output-format csv -- python3 tools/train_bench.py --R 65 --iters 3 > gpurun_out/pmc_bwd2.log 2>&1
rc2=$?
echo "rc $rc1 $rc2"
grep -c . gpurun_out/counters_r02.txt
for d in pmc_bwd1 pmc_bwd2; do f=gpurun_out/$d/run_counter_collection.csv; [ -f $f ] && python3 - $f <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", ""))[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if "train" in k or "deepsets" in k:
        print(k, dict(v))
PY
done
exit 0
