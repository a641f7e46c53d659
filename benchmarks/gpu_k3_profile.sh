#!/bin/bash
# Kernel trace of binary_auroc / binary_auprc at N=1M (K3a radix sort + K3 scan)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_k3
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_k3 -o k3 -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_auroc_1m.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_k3.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_k3.log"; exit 1; }
find /tmp/prof_k3 -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k3_kernel_stats.csv" \;
find /tmp/prof_k3 -name "*kernel_trace.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k3_kernel_trace.csv" \;
cut -d, -f1-4 "$GRAFT_REPO_ROOT/gpurun_out/k3_kernel_stats.csv" | cut -c1-150
