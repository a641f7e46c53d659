#!/bin/bash
# Round 5: K1 / K5 / K5b tests, the odd-width cliff benchmark, the K5b deferred-mode A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/gpu/test_k5_pending.py tests/gpu/test_k5b_rowsums.py tests/gpu/test_k5_k7_k8.py tests/gpu/test_k1_unal.py tests/gpu/test_k1_classification.py tests/gpu/test_classification_gpu.py tests/gpu/test_accuracy_gpu.py tests/gpu/test_k1_micro.py \
  > gpurun_out/r5_k5b_tests.log 2>&1 || { tail -40 gpurun_out/r5_k5b_tests.log; exit 1; }
tail -3 gpurun_out/r5_k5b_tests.log
timeout -k 10 120 python -u benchmarks/odd_width_cliff.py > gpurun_out/r5_odd_width_1.json 2>&1 || { tail -20 gpurun_out/r5_odd_width_1.json; exit 1; }
cat gpurun_out/r5_odd_width_1.json
timeout -k 10 120 python -u benchmarks/k5b_pend_ab.py > gpurun_out/r5_k5b_ab_vpt8.json 2>&1 || { tail -20 gpurun_out/r5_k5b_ab_vpt8.json; exit 1; }
cat gpurun_out/r5_k5b_ab_vpt8.json
TORCHEVAL_AMD_K5B_PEND_VPT=4 timeout -k 10 120 python -u benchmarks/k5b_pend_ab.py > gpurun_out/r5_k5b_ab_vpt4.json 2>&1 || { tail -20 gpurun_out/r5_k5b_ab_vpt4.json; exit 1; }
cat gpurun_out/r5_k5b_ab_vpt4.json
