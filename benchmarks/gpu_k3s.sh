#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/gpu/test_k3s_samplesort.py > gpurun_out/t_k3s.log 2>&1 || { tail -40 gpurun_out/t_k3s.log; exit 1; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k3_k4_k6.py tests/gpu/test_dist_auc_gpu.py tests/gpu/test_k3c_curves.py tests/gpu/test_classification_gpu.py > gpurun_out/t_k3_rest.log 2>&1 || { tail -40 gpurun_out/t_k3_rest.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_k3s
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_k3s -o k3s -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_auroc_1m.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_k3s.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_k3s.log"; exit 1; }
find /tmp/prof_k3s -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k3s_kernel_stats.csv" \;
tail -3 "$GRAFT_REPO_ROOT/gpurun_out/t_k3s.log"; tail -2 "$GRAFT_REPO_ROOT/gpurun_out/t_k3_rest.log"
