#!/bin/bash
# K9b multisection lanes per eigenvalue A/B with the product-form Sturm count (D = 2048)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r6_sturmL
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in 16 32 64; do
  rm -rf /tmp/pf
  TORCHEVAL_AMD_SYMEIG_L=$L TORCHEVAL_AMD_SYMEIG_COOP=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/pf -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/fid_compute_probe.py" > "$O/prof_$L.log" 2>&1 || { echo "L=$L failed"; tail -3 "$O/prof_$L.log"; exit 1; }
  f=$(find /tmp/pf -name "*kernel_trace.csv" | head -1)
  cp "$f" "$O/trace_$L.csv"
done
echo done
