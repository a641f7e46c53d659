#!/bin/bash
# Staged FID updates: GPU parity tests + bench rows with staging on (default) and off.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/gpu/test_k5_k7_k8.py tests/gpu/test_rccl_direct.py > gpurun_out/fid_stage_tests.log 2>&1
timeout -k 10 240 python -u benchmarks/bench_suite.py --only FID --no-aten --out gpurun_out/fid_stage_on.json > gpurun_out/fid_stage_on.log 2>&1
TORCHEVAL_AMD_FID_STAGE_ROWS=0 timeout -k 10 240 python -u benchmarks/bench_suite.py --only FID --no-aten --out gpurun_out/fid_stage_off.json > gpurun_out/fid_stage_off.log 2>&1
tail -3 gpurun_out/fid_stage_tests.log; cat gpurun_out/fid_stage_on.log gpurun_out/fid_stage_off.log
