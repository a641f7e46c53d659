#!/bin/bash
# rocprofv3 counter passes over the final K9b kernels at D = 2048 (plain launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_k9b
export TMPDIR=/tmp
export TORCHEVAL_AMD_SYMEIG_COOP=0
pass() {
  tag=$1; shift
  rm -rf /tmp/pmck9_$tag
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d /tmp/pmck9_$tag -o $tag -- python3 "$GRAFT_REPO_ROOT/benchmarks/k9b_pmc_probe.py") > "$GRAFT_REPO_ROOT/gpurun_out/pmc_k9b/$tag.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc_k9b/$tag.log"; return 1; }
  find /tmp/pmck9_$tag -name "*counter_collection.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pmc_k9b/$tag.csv" \;
  find /tmp/pmck9_$tag -name "*kernel_trace.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pmc_k9b/${tag}_trace.csv" \;
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
pass lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVES || exit 1
pass mem FETCH_SIZE || exit 1
python3 - <<'PY'
import csv, collections, glob, os
root = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/pmc_k9b/"
for f in sorted(glob.glob(root + "*.csv")):
    if f.endswith("_trace.csv"):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(f))
    for k, d in agg.items():
        print(" ", k)
        for c, v in sorted(d.items()):
            print(f"     {c:24s} {sum(v)/len(v):16.1f} (n={len(v)})")
PY
