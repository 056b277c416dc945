#!/bin/bash
# SQ counter passes of lb_rollout launches (tools/pmc_probe.py, PMC_MODE=rollout) for the
# libraries in LIBS (default: the product build), K in KS; summaries per wave-step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -s KILL 90"
for lib in ${LIBS:-gym-loadbalancing_amd/lbk8s/liblbk8s.so}; do
 for K in ${KS:-100}; do
  tag=$(basename $lib .so)_k$K
  PMC_LIB=$lib PMC_MODE=rollout PMC_K=$K $T rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace -d gpurun_out/sqa_$tag -o run \
      --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/sqa_$tag.log 2>&1 || exit 1
  PMC_LIB=$lib PMC_MODE=rollout PMC_K=$K $T rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM \
      SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM --kernel-trace -d gpurun_out/sqb_$tag -o run \
      --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/sqb_$tag.log 2>&1 || exit 1
  if [ -n "$EXTRA_PASS" ]; then
    PMC_LIB=$lib PMC_MODE=rollout PMC_K=$K $T rocprofv3 --pmc $EXTRA_PASS --kernel-trace -d gpurun_out/sqc_$tag -o run \
        --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/sqc_$tag.log 2>&1 || exit 1
  fi
  echo "== $tag"
  for z in sqa sqb sqc; do [ -f gpurun_out/${z}_$tag/run_counter_collection.csv ] && python3 tools/pmc_sum.py gpurun_out/${z}_$tag/run_counter_collection.csv k_rollout; done
 done
done
