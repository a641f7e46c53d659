#!/bin/bash
# async sync overlap: wall-clock A/B, then a kernel trace and its overlap analysis
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 180 python3 benchmarks/rccl_overlap_device.py --reps 10 --out gpurun_out/overlap_ms.json > gpurun_out/overlap_ms.log 2>&1 || { tail -30 gpurun_out/overlap_ms.log; exit 1; }
cat gpurun_out/overlap_ms.json
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_ov
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/prof_ov -o ov -- python3 "$GRAFT_REPO_ROOT/benchmarks/rccl_overlap_device.py" --reps 3 > "$GRAFT_REPO_ROOT/gpurun_out/overlap_prof.log" 2>&1 || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/overlap_prof.log"; exit 1; }
find /tmp/prof_ov -name "*kernel_trace.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/overlap_kernel_trace.csv" \;
find /tmp/prof_ov -name "*memory_copy_trace.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/overlap_memcpy_trace.csv" \;
cd "$GRAFT_REPO_ROOT" && python3 benchmarks/rccl_overlap_device.py --trace gpurun_out/overlap_kernel_trace.csv --out gpurun_out/overlap_trace.json
