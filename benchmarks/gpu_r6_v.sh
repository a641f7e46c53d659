#!/bin/bash
# round 6, call V: FID compute kernel timeline; K3 bucket-mode phase trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./csrc/bench/k3_bucket_trace.bin > gpurun_out/r6v_bucket_trace.txt 2>&1 || { cat gpurun_out/r6v_bucket_trace.txt; exit 1; }
tail -14 gpurun_out/r6v_bucket_trace.txt
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pf
TORCHEVAL_AMD_SYMEIG_COOP=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/pf -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/fid_compute_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/r6v_prof.log" 2>&1
echo "rocprof rc=$?"
f=$(find /tmp/pf -name "*kernel_trace.csv" | head -1)
cp "$f" "$GRAFT_REPO_ROOT/gpurun_out/r6v_fid_kernel_trace.csv"
