#!/bin/bash
# Direct RCCL communicators: tests, then the sync floors and breakdown with and without them
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_rccl_direct.py tests/gpu/test_rccl_single_rank.py tests/gpu/test_accuracy_gpu.py > gpurun_out/t_rccl_direct.log 2>&1 || { tail -40 gpurun_out/t_rccl_direct.log; exit 1; }
tail -2 gpurun_out/t_rccl_direct.log
timeout -k 10 200 python3 benchmarks/sync_breakdown.py > gpurun_out/sync_breakdown_direct.json 2> gpurun_out/sbd.err || { tail -20 gpurun_out/sbd.err; exit 1; }
cat gpurun_out/sync_breakdown_direct.json
timeout -k 10 200 python3 benchmarks/rccl_sync_floor.py --out gpurun_out/sync_floor_direct.json > /dev/null 2> gpurun_out/sf.err || { tail -20 gpurun_out/sf.err; exit 1; }
cat gpurun_out/sync_floor_direct.json
TORCHEVAL_AMD_DIRECT_RCCL=0 timeout -k 10 200 python3 benchmarks/rccl_sync_floor.py --out gpurun_out/sync_floor_torchdist.json > /dev/null 2> gpurun_out/sf0.err || { tail -20 gpurun_out/sf0.err; exit 1; }
cat gpurun_out/sync_floor_torchdist.json
bash benchmarks/gpu_overlap.sh
