#!/bin/bash
# Round 5: the whole GPU suite (K4b per-sample binned AUROC, K5 / K5b deferred mode, K1 unaligned
# rows, direct-RCCL engine), then the K5b deferred A/B and the odd-width cliff benchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5_c_tests.log 2>&1 || { tail -40 gpurun_out/r5_c_tests.log; exit 1; }
tail -1 gpurun_out/r5_c_tests.log
timeout -k 10 120 python -u benchmarks/k5b_pend_ab.py > gpurun_out/r5_k5b_ab_vpt8.json 2>&1 || { tail -20 gpurun_out/r5_k5b_ab_vpt8.json; exit 1; }
cat gpurun_out/r5_k5b_ab_vpt8.json
timeout -k 10 120 python -u benchmarks/odd_width_cliff.py > gpurun_out/r5_odd_width_3.json 2>&1 || { tail -20 gpurun_out/r5_odd_width_3.json; exit 1; }
cat gpurun_out/r5_odd_width_3.json
