# PMC cycle buckets of the bench's step kernel (tools/pmc_probe.py workload)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d gpurun_out/v1 -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/v1.log 2>&1 || exit 1
$T 180 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/v2 -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/v2.log 2>&1 || exit 1
$T 180 rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TD_BUSY_avr --kernel-trace -d gpurun_out/v3 -o run --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/v3.log 2>&1 || true
for i in 1 2 3; do [ -f gpurun_out/v$i/run_counter_collection.csv ] && python3 tools/pmc_sum.py gpurun_out/v$i/run_counter_collection.csv k_step; done
exit 0
