#!/bin/bash
# Fused-flag CM sync (tests + floors) and the K8 small-D split sweep vs the library update.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/gpu/test_accuracy_gpu.py tests/gpu/test_rccl_single_rank.py > gpurun_out/pytest_r3g.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r3g.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 benchmarks/sync_breakdown.py > gpurun_out/sync_breakdown.json 2> gpurun_out/sync_breakdown.err || { tail -20 gpurun_out/sync_breakdown.err; exit 1; }
cat gpurun_out/sync_breakdown.json
timeout -k 10 200 python3 benchmarks/rccl_sync_floor.py --out gpurun_out/sync_floor.json > /dev/null 2> gpurun_out/sync_floor.err || { tail -20 gpurun_out/sync_floor.err; exit 1; }
cat gpurun_out/sync_floor.json
timeout -k 10 300 python3 benchmarks/k8_sweep.py --d 512 768 1024 --k 1000 4096 --splits 0 1 2 4 8 16 --out gpurun_out/k8_sweep_small_d_r3.json > gpurun_out/k8_sweep.log 2>&1 || { tail -20 gpurun_out/k8_sweep.log; exit 1; }
cat gpurun_out/k8_sweep.log
