#!/bin/bash
# K3b parity tests, then the K3b vs K3a+K3 sweep and a kernel trace of the 1M workload
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/gpu/test_k3b_bucket_auc.py > gpurun_out/t_k3b.log 2>&1 || { tail -40 gpurun_out/t_k3b.log; exit 1; }
tail -3 gpurun_out/t_k3b.log
timeout -k 10 300 python -u benchmarks/k3b_sweep.py > gpurun_out/k3b_sweep.log 2>&1 || { tail -20 gpurun_out/k3b_sweep.log; exit 1; }
tail -1 gpurun_out/k3b_sweep.log > gpurun_out/k3b_sweep.json
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_k3b
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_k3b -o k3b -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_auroc_1m.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_k3b.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_k3b.log"; exit 1; }
find /tmp/prof_k3b -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k3b_kernel_stats.csv" \;
head -12 "$GRAFT_REPO_ROOT/gpurun_out/k3b_kernel_stats.csv"
