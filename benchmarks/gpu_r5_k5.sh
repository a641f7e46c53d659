#!/bin/bash
# Round 5: K5 v2 correctness (new odd-width / geometry tests + the existing K5 tests), then
# the v1 / v2 geometry A/B and the odd-width cliff benchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/gpu/test_k5_pending.py tests/gpu/test_k5_v2_odd.py tests/gpu/test_k5_k7_k8.py tests/gpu/test_k5b_rowsums.py tests/gpu/test_k1_unal.py tests/gpu/test_k1_micro.py tests/gpu/test_k1_classification.py \
  > gpurun_out/r5_k5_tests.log 2>&1 || { tail -30 gpurun_out/r5_k5_tests.log; exit 1; }
tail -3 gpurun_out/r5_k5_tests.log
timeout -k 10 200 python -u benchmarks/k5_v2_ab.py > gpurun_out/r5_k5_ab.jsonl 2>&1 || { tail -20 gpurun_out/r5_k5_ab.jsonl; exit 1; }
cat gpurun_out/r5_k5_ab.jsonl
if [ "${K5_ODD:-0}" = 1 ]; then
timeout -k 10 120 python -u benchmarks/odd_width_cliff.py > gpurun_out/r5_odd_width.json 2>&1 || { tail -20 gpurun_out/r5_odd_width.json; exit 1; }
cat gpurun_out/r5_odd_width.json
fi
