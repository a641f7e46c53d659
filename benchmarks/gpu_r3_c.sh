#!/bin/bash
# Round 3: K1 micro kernel - GPU tests, the driver's bench command, harness A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/gpu/test_k1_classification.py tests/gpu/test_accuracy_gpu.py tests/gpu/test_compile_gpu.py tests/gpu/test_classification_gpu.py > gpurun_out/pytest_r3c.log 2>&1; echo "pytest rc=$?"
tail -4 gpurun_out/pytest_r3c.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 2000 --warmup 200 --no-reference > gpurun_out/bench_2k.json 2> gpurun_out/bench_2k.err || { tail -20 gpurun_out/bench_2k.err; exit 1; }
cat gpurun_out/bench_2k.json
timeout -k 10 120 ./csrc/bench/k1_v3.bin 8 0 > gpurun_out/k1_v3_pool8_rand.txt 2>&1 || { cat gpurun_out/k1_v3_pool8_rand.txt; exit 1; }
cat gpurun_out/k1_v3_pool8_rand.txt
timeout -k 10 120 ./csrc/bench/k1_v3.bin 16 2 > gpurun_out/k1_v3_pool16_c50.txt 2>&1 || { cat gpurun_out/k1_v3_pool16_c50.txt; exit 1; }
cat gpurun_out/k1_v3_pool16_c50.txt
