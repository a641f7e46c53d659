#!/bin/bash
# One SQ counter pass over the K3b 1M binary_auroc workload (profile_auroc_1m.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pmc_k3b
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d /tmp/pmc_k3b -o k3b -- \
  python3 "$GRAFT_REPO_ROOT/benchmarks/profile_auroc_1m.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc/k3b.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc/k3b.log"; exit 1; }
find /tmp/pmc_k3b -name "*counter_collection.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pmc/k3b.csv" \;
python3 - "$GRAFT_REPO_ROOT/gpurun_out/pmc/k3b.csv" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if "bk_" not in r["Kernel_Name"]:
        continue
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):14.1f}  (n={len(v)})")
PY
