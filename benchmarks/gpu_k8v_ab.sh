#!/bin/bash
# K8 harness A/B: split-bf16 (default) vs FP32 MFMA (TORCHEVAL_AMD_K8_EXACT=1), with and
# without the per-stage global loads; then SQ + TCC counter passes of the default build.
set -e
mkdir -p gpurun_out/pmc
for v in base noload; do
  echo "== $v x3"; timeout -k 10 60 csrc/bench/k8v_$v
  echo "== $v exact"; TORCHEVAL_AMD_K8_EXACT=1 timeout -k 10 60 csrc/bench/k8v_$v
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d /tmp/pmc_a -o k8v -- "$R/csrc/bench/k8v_base" > "$R/gpurun_out/pmc/k8x_sq.log" 2>&1
find /tmp/pmc_a -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc/k8x_sq.csv" \;
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum \
  --kernel-trace --output-format csv -d /tmp/pmc_b -o k8v -- "$R/csrc/bench/k8v_base" > "$R/gpurun_out/pmc/k8x_tcc.log" 2>&1
find /tmp/pmc_b -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc/k8x_tcc.csv" \;
timeout -s KILL 90 rocprofv3 --pmc TCC_MISS_sum TCC_EA0_RDREQ_sum \
  --kernel-trace --output-format csv -d /tmp/pmc_c -o k8v -- "$R/csrc/bench/k8v_base" > "$R/gpurun_out/pmc/k8x_tcc2.log" 2>&1
find /tmp/pmc_c -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc/k8x_tcc2.csv" \;
echo done
