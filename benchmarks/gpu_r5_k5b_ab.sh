#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k4b_sample_binned_auroc.py \
  tests/gpu/test_k5_pending.py tests/gpu/test_k5b_rowsums.py tests/gpu/test_k5_v2_odd.py \
  > gpurun_out/r5_k5b_tests.log 2>&1 || { tail -40 gpurun_out/r5_k5b_tests.log; exit 1; }
tail -1 gpurun_out/r5_k5b_tests.log
timeout -k 10 120 python -u benchmarks/k5b_pend_ab.py > gpurun_out/r5_k5b_ab_vpt8.json 2>&1 || { tail -20 gpurun_out/r5_k5b_ab_vpt8.json; exit 1; }
cat gpurun_out/r5_k5b_ab_vpt8.json
timeout -k 10 120 python -u benchmarks/odd_width_cliff.py > gpurun_out/r5_odd_width_2.json 2>&1 || { tail -20 gpurun_out/r5_odd_width_2.json; exit 1; }
cat gpurun_out/r5_odd_width_2.json
