#!/bin/bash
# K5 GPU tests, then the torch.profiler breakdown of the regression cases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k5_k7_k8.py tests/gpu/test_k5b_rowsums.py > gpurun_out/t_k5.log 2>&1 || { tail -30 gpurun_out/t_k5.log; exit 1; }
tail -1 gpurun_out/t_k5.log
timeout -k 10 300 python3 -u benchmarks/profile_ops.py "mean_squared_error" "r2_score" > gpurun_out/profile_k5.txt 2>&1 || { tail -30 gpurun_out/profile_k5.txt; exit 1; }
grep -E "^#####|Self CUDA time total|_kernel" gpurun_out/profile_k5.txt | cut -c1-70,150-175
