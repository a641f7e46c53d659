#!/bin/bash
# K8 bf16 three-way-split path: parity tests, then the sweep in both modes.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/gpu/test_k5_k7_k8.py > gpurun_out/k8x_tests.log 2>&1 || { tail -40 gpurun_out/k8x_tests.log; exit 1; }
tail -3 gpurun_out/k8x_tests.log
timeout -k 10 300 python -u benchmarks/k8_sweep.py --d 2048 512 1024 --k 1000 8192 50000 --out gpurun_out/k8x_sweep.json > gpurun_out/k8x_sweep.log 2>&1
cat gpurun_out/k8x_sweep.log
