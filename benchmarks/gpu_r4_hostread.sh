#!/bin/bash
# Host-read fast path: its GPU tests, the flag-reading GPU suites, the latency probe, the sync floors.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_hostread.py \
  tests/gpu/test_accuracy_gpu.py tests/gpu/test_rccl_direct.py tests/gpu/test_k5_k7_k8.py > gpurun_out/hostread_tests.log 2>&1
rc=$?; tail -3 gpurun_out/hostread_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/hostread_tests.log | head; exit $rc; }
timeout -k 10 60 ./csrc/bench/host_poll_latency.bin > gpurun_out/host_poll_latency.txt && cat gpurun_out/host_poll_latency.txt || exit 1
timeout -k 10 300 python benchmarks/rccl_sync_floor.py > gpurun_out/sync_floor_hostread.json 2> gpurun_out/sync_floor_hostread.err
rc=$?; cat gpurun_out/sync_floor_hostread.json; tail -3 gpurun_out/sync_floor_hostread.err; exit $rc
