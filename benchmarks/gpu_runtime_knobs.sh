#!/bin/bash
# HIP runtime knobs vs the K1 floor harness (per-launch cost, empty dispatch, host cost, the
# bench region driven from C++).  One line per knob setting.  (ROC_SYSTEM_SCOPE_SIGNAL=0 hangs
# the harness: removed, profiles/hip_runtime_knobs_r4.txt.)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for knob in "NONE=1" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0" "DEBUG_HIP_KERNARG_COPY_OPT=0" "DEBUG_HIP_KERNARG_COPY_OPT=1" \
            "ROC_USE_FGS_KERNARG=0" "ROC_USE_FGS_KERNARG=1" "ROC_CPU_WAIT_FOR_SIGNAL=0" \
            "ROC_CPU_WAIT_FOR_SIGNAL=1" "DEBUG_CLR_BLIT_KERNARG_OPT=0" "GPU_FLUSH_ON_EXECUTION=1" "ROC_AQL_QUEUE_SIZE=65536"; do
  out=$(env $knob timeout -k 10 60 ./csrc/bench/k1_floor.bin 8 200 2>&1)
  rc=$?
  [ $rc -ne 0 ] && { echo "$knob rc=$rc"; echo "$out" | tail -3; exit $rc; }
  prod=$(echo "$out" | grep '"prod (' | sed 's/.*us_per_launch": \([0-9.]*\).*/\1/')
  empty=$(echo "$out" | grep '"empty (2048' | sed 's/.*us_per_launch": \([0-9.]*\).*/\1/')
  host=$(echo "$out" | grep host_us_per_launch)
  echo "{\"knob\": \"$knob\", \"prod_us\": $prod, \"empty_us\": $empty, \"host\": $host}"
done
