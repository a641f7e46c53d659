#!/bin/bash
# binary_auroc 1M kernel timeline (GPU-bound or host-bound?)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u benchmarks/k3_timeline_probe.py || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pf
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/pf -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/k3_timeline_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/k3tl_prof.log" 2>&1
echo "rocprof rc=$?"
f=$(find /tmp/pf -name "*kernel_trace.csv" | head -1)
cp "$f" "$GRAFT_REPO_ROOT/gpurun_out/k3tl_kernel_trace.csv"
