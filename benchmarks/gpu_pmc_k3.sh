#!/bin/bash
# PMC passes over multiclass_auroc 100k x 100 (K3a radix passes + K3 scan at 10M keys)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
run() {
  tag=$1; shift
  rm -rf /tmp/pmc_$tag
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d /tmp/pmc_$tag -o $tag -- \
    python3 "$GRAFT_REPO_ROOT/benchmarks/profile_mc_auroc.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log"; return 1; }
  find /tmp/pmc_$tag -name "*counter_collection.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.csv" \;
  python3 - "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.csv" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if "tea::" not in name:
        continue
    agg[name[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):14.1f}  (n={len(v)})")
PY
}
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS && \
run mem FETCH_SIZE WRITE_SIZE TCP_TCC_READ_REQ_sum
