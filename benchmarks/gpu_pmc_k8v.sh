#!/bin/bash
# LDS / wait counters of the standalone K8 harness variants (csrc/bench/k8_variants.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  rm -rf /tmp/pmc_k8v_$v
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d /tmp/pmc_k8v_$v -o k8v -- "$GRAFT_REPO_ROOT/csrc/bench/k8v_$v" > "$GRAFT_REPO_ROOT/gpurun_out/pmc/k8v_$v.log" 2>&1 || exit 1
  find /tmp/pmc_k8v_$v -name "*counter_collection.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pmc/k8v_$v.csv" \;
done
