#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./csrc/bench/k1_v3.bin 8 0 > gpurun_out/k1_v3_pool8_rand.txt 2>&1 || { cat gpurun_out/k1_v3_pool8_rand.txt; exit 1; }
cat gpurun_out/k1_v3_pool8_rand.txt
timeout -k 10 120 ./csrc/bench/k1_v3.bin 16 2 > gpurun_out/k1_v3_pool16_c50.txt 2>&1 || { cat gpurun_out/k1_v3_pool16_c50.txt; exit 1; }
cat gpurun_out/k1_v3_pool16_c50.txt
