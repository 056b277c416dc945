set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_bwdn1 -o run --output-format csv -- python3 tools/train_bench.py --R 65 --iters 3 > gpurun_out/pmc_bwdn1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc_bwdn2 -o run --output-format csv -- python3 tools/train_bench.py --R 65 --iters 3 > gpurun_out/pmc_bwdn2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_MFMA SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES --kernel-trace -d gpurun_out/pmc_bwdn3 -o run --output-format csv -- python3 tools/train_bench.py --R 65 --iters 3 > gpurun_out/pmc_bwdn3.log 2>&1
for d in pmc_bwdn1 pmc_bwdn2 pmc_bwdn3; do f=gpurun_out/$d/run_counter_collection.csv; [ -f $f ] && python3 - $f <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r.get("Kernel_Name", "")[:50]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if "train_bwd" in k or "deepsets_fwd" in k:
        print(k, {a: f"{b:.4g}" for a, b in v.items()})
PY
done
tail -3 gpurun_out/pmc_bwdn3.log
exit 0
