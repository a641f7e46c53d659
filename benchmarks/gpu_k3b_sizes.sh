#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for n in 32768 1000000; do
rm -rf /tmp/p$n
AUROC_N=$n timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p$n -o k -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_auroc_1m.py" > "$GRAFT_REPO_ROOT/gpurun_out/p$n.log" 2>&1 || exit 1
find /tmp/p$n -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k3b_stats_$n.csv" \;
find /tmp/p$n -name "*kernel_trace.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k3b_trace_$n.csv" \;
cut -d, -f1-4 "$GRAFT_REPO_ROOT/gpurun_out/k3b_stats_$n.csv" | grep bk_
done
