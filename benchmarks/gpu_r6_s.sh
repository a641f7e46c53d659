#!/bin/bash
# round 6, call S: K3a splitter-bucket mode - tests, then the binary_auroc A/B against 4 passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/gpu/test_k3_bucket.py \
  > gpurun_out/r6s_tests.log 2>&1 || { tail -60 gpurun_out/r6s_tests.log; exit 1; }
tail -3 gpurun_out/r6s_tests.log
K3_AB_BUCKET=1 timeout -k 10 400 python -u benchmarks/k3_onesweep_ab.py > gpurun_out/r6s_ab.jsonl 2> gpurun_out/r6s.err || { tail -20 gpurun_out/r6s.err; exit 1; }
cat gpurun_out/r6s_ab.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/gpu/test_k3_onesweep.py \
  tests/gpu/test_k3_k4_k6.py tests/gpu/test_k3c_curves.py tests/gpu/test_k3t_auc.py tests/gpu/test_k3_onesweep_timeout.py \
  > gpurun_out/r6s_k3.log 2>&1 || { tail -40 gpurun_out/r6s_k3.log; exit 1; }
tail -1 gpurun_out/r6s_k3.log
