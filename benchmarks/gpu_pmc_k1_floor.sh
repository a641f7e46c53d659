#!/bin/bash
# SQ / TCC counter passes over the K1 floor harness (prod vs pure-read vs variants), one pass
# per run as rocprofv3 requires; per-kernel means printed and kept under gpurun_out/pmc.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
BIN="$GRAFT_REPO_ROOT/csrc/bench/k1_floor.bin"
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = tag, rest = counters
  local tag=$1; shift
  rm -rf /tmp/pmc_$tag
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d /tmp/pmc_$tag -o $tag -- \
    "$BIN" 8 30 > "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log"; return 1; }
  find /tmp/pmc_$tag -name "*counter_collection.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.csv" \;
  python3 - "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.csv" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, "  " + "  ".join(f"{c}={sum(v)/len(v):.0f}" for c, v in sorted(d.items())))
PY
}
run k1sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM && \
run k1fetch FETCH_SIZE TCC_HIT_sum && \
run k1write WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE
