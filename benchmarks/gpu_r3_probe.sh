#!/bin/bash
# Round-3 probe: K1 A/B harness (random targets and 1-in-5 correct rows; 8- and 16-batch
# pools), host cost per update, the driver's bench command and the 1-rank RCCL sync floors.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./csrc/bench/k1_v3.bin 8 0 > gpurun_out/k1_v3_pool8_rand.txt 2>&1 || { cat gpurun_out/k1_v3_pool8_rand.txt; exit 1; }
cat gpurun_out/k1_v3_pool8_rand.txt
timeout -k 10 120 ./csrc/bench/k1_v3.bin 8 5 > gpurun_out/k1_v3_pool8_c20.txt 2>&1 || { cat gpurun_out/k1_v3_pool8_c20.txt; exit 1; }
timeout -k 10 120 ./csrc/bench/k1_v3.bin 16 0 > gpurun_out/k1_v3_pool16_rand.txt 2>&1 || { cat gpurun_out/k1_v3_pool16_rand.txt; exit 1; }
timeout -k 10 180 python3 benchmarks/host_overhead.py > gpurun_out/host_overhead.json 2> gpurun_out/host_overhead.err || { tail -20 gpurun_out/host_overhead.err; exit 1; }
cat gpurun_out/host_overhead.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
timeout -k 10 300 python3 benchmarks/rccl_sync_floor.py --out gpurun_out/sync_floor.json > /dev/null 2> gpurun_out/sync_floor.err || { tail -20 gpurun_out/sync_floor.err; exit 1; }
cat gpurun_out/sync_floor.json
echo ok
