#!/bin/bash
# K9b: GPU tests, timing and rocprofv3 kernel stats of the symmetric eigenvalue path
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/gpu/test_k9b_symeig.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k9b_tests.log 2>&1 || { tail -30 gpurun_out/k9b_tests.log; exit 1; }
tail -2 gpurun_out/k9b_tests.log
timeout -k 10 180 python benchmarks/symeig_timing.py > gpurun_out/k9b_timing.json 2>&1 || { tail -20 gpurun_out/k9b_timing.json; exit 1; }
cat gpurun_out/k9b_timing.json
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_k9b
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_k9b -o k9b -- \
  python3 "$GRAFT_REPO_ROOT/benchmarks/symeig_timing.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_k9b.log" 2>&1
# rocprofv3 has crashed at process exit after writing its output on this image; keep the files
echo "rocprofv3 rc=$?"
find /tmp/prof_k9b -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k9b_kernel_stats.csv" \;
find /tmp/prof_k9b -name "*kernel_trace.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k9b_kernel_trace.csv" \;
head -6 "$GRAFT_REPO_ROOT/gpurun_out/k9b_kernel_stats.csv" | cut -c1-160
