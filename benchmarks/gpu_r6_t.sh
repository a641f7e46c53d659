#!/bin/bash
# round 6, call T: kernel stats of binary_auroc 1M, bucket mode vs the four onesweep passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for b in 1 0; do
  rm -rf /tmp/pb$b
  TORCHEVAL_AMD_K3_BUCKET=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pb$b -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/k3_bucket_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/r6t_$b.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r6t_$b.log"; exit 1; }
  f=$(find /tmp/pb$b -name "*kernel_stats.csv" | head -1)
  cp "$f" "$GRAFT_REPO_ROOT/gpurun_out/r6t_kstats_bucket$b.csv"
  echo "== bucket=$b"; cut -d, -f1-4 "$f" | head -14
done
