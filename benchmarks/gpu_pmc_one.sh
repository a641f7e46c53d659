#!/bin/bash
# One SQ counter pass over the PMC_ONLY-filtered pmc_targets workload: $1 = tag, rest = counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
tag=$1; shift
rm -rf /tmp/pmc_$tag
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d /tmp/pmc_$tag -o $tag -- \
  python3 "$GRAFT_REPO_ROOT/benchmarks/pmc_targets.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log"; exit 1; }
find /tmp/pmc_$tag -name "*counter_collection.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.csv" \;
python3 - "$GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.csv" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):14.1f}  (n={len(v)})")
PY
