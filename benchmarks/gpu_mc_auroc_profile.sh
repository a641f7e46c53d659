#!/bin/bash
# Kernel stats of multiclass_auroc N=100k C=100 (K3a segmented radix sort + K3 scan)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_mc
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_mc -o mc -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_mc_auroc.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_mc.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_mc.log"; exit 1; }
find /tmp/prof_mc -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/mc_auroc_kernel_stats.csv" \;
cut -d, -f1-4 "$GRAFT_REPO_ROOT/gpurun_out/mc_auroc_kernel_stats.csv" | cut -c1-150
