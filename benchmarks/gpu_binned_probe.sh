#!/bin/bash
# Probe: where does the time of the binned / AUROC functionals go (torch.profiler host+device,
# and per-kernel rocprofv3 stats for just those cases).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/profile_ops.py binned_auroc binned_precision_recall "binary_auroc N" BinnedAUPRC > gpurun_out/profile_ops.log 2>&1 || { tail -30 gpurun_out/profile_ops.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_binned
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_binned -o binned -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_suite.py" --no-aten --min-time 0.2 --only binned > "$GRAFT_REPO_ROOT/gpurun_out/prof_binned.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_binned.log"; exit 1; }
find /tmp/prof_binned -name "*_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/binned_" \; 
find /tmp/prof_binned -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/binned_kernel_stats.csv" \;
echo ok
