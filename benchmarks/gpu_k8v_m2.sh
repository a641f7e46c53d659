#!/bin/bash
# K8 kMode 2 harness: default, without the per-stage loads, without the interleave pins; SQ counters.
set -e
mkdir -p gpurun_out/pmc
for v in base noload nosched; do echo "== $v"; timeout -k 10 60 csrc/bench/k8v_$v; done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
  --kernel-trace --output-format csv -d /tmp/pmc_m2 -o k8v -- "$R/csrc/bench/k8v_base" > "$R/gpurun_out/pmc/k8m2_sq.log" 2>&1
find /tmp/pmc_m2 -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc/k8m2_sq.csv" \;
echo done
