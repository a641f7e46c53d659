#!/bin/bash
# K8 quick loop: GPU tests of K8/FID, the harness variants, the x3 sweep rows.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/gpu/test_k5_k7_k8.py > gpurun_out/k8q_tests.log 2>&1 || { tail -40 gpurun_out/k8q_tests.log; exit 1; }
tail -2 gpurun_out/k8q_tests.log
for v in base noload nosched; do echo "== $v"; timeout -k 10 60 csrc/bench/k8v_$v; done
timeout -k 10 300 python -u benchmarks/k8_sweep.py --d 2048 --k 1000 8192 50000 --modes x3 --out gpurun_out/k8q_sweep.json > gpurun_out/k8q_sweep.log 2>&1
cut -c1-200 gpurun_out/k8q_sweep.log
