#!/bin/bash
# Round 3: K1 isolation A/B, RCCL primitive + sync floors, host cost, new GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./csrc/bench/k1_v3.bin 8 0 > gpurun_out/k1_v3_pool8_rand.txt 2>&1 || { cat gpurun_out/k1_v3_pool8_rand.txt; exit 1; }
timeout -k 10 120 ./csrc/bench/k1_v3.bin 16 2 > gpurun_out/k1_v3_pool16_c50.txt 2>&1 || { cat gpurun_out/k1_v3_pool16_c50.txt; exit 1; }
timeout -k 10 200 python3 benchmarks/rccl_primitive_latency.py > gpurun_out/rccl_prim.json 2> gpurun_out/rccl_prim.err || { tail gpurun_out/rccl_prim.err; exit 1; }
timeout -k 10 200 python3 benchmarks/rccl_sync_floor.py --out gpurun_out/sync_floor.json > /dev/null 2> gpurun_out/sync_floor.err || { tail gpurun_out/sync_floor.err; exit 1; }
timeout -k 10 200 python3 benchmarks/host_overhead.py > gpurun_out/host_overhead.json 2> gpurun_out/host_overhead.err || { tail gpurun_out/host_overhead.err; exit 1; }
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/gpu/test_accuracy_gpu.py tests/gpu/test_compile_gpu.py tests/gpu/test_torch_ops_gpu.py > gpurun_out/pytest_r3b.log 2>&1; echo "pytest rc=$?"
tail -5 gpurun_out/pytest_r3b.log
cat gpurun_out/k1_v3_pool8_rand.txt gpurun_out/rccl_prim.json gpurun_out/sync_floor.json gpurun_out/host_overhead.json
