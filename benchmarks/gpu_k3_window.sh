#!/bin/bash
# K3 straddling-tie window: parity tests, bench rows, kernel stats at 1M.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/gpu/test_k3_k4_k6.py tests/gpu/test_k3c_curves.py tests/gpu/test_k3m_merge.py tests/gpu/test_dist_auc_gpu.py > gpurun_out/k3w_tests.log 2>&1 || { tail -40 gpurun_out/k3w_tests.log; exit 1; }
tail -2 gpurun_out/k3w_tests.log
timeout -k 10 240 python -u benchmarks/bench_suite.py --only "auroc|auprc|precision_recall_curve N=1M|recall_at_fixed" --no-aten --out gpurun_out/k3w_suite.json > gpurun_out/k3w_suite.log 2>&1
cat gpurun_out/k3w_suite.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k3w -o k3w -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_auroc_1m.py" > "$GRAFT_REPO_ROOT/gpurun_out/k3w_prof.log" 2>&1
find /tmp/k3w -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/k3w_kernel_stats.csv" \;
cut -c1-150 "$GRAFT_REPO_ROOT/gpurun_out/k3w_kernel_stats.csv" | head -8
