#!/bin/bash
# PMC counter passes (kernel-trace + counters only; no sys/runtime trace) over pmc_targets.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = tag, rest = counters
  local tag=$1; shift
  rm -rf /tmp/pmc_$tag
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d /tmp/pmc_$tag -o $tag -- \
    python3 "$GRAFT_REPO_ROOT/benchmarks/pmc_targets.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log"; return 1; }
  find /tmp/pmc_$tag -name "*counter_collection.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.csv" \;
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU && \
run fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
run write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
ls -la "$GRAFT_REPO_ROOT/gpurun_out/pmc/"
