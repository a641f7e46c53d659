#!/bin/bash
# round 6, call B: graph-replay fix re-test, K9d Cholesky / sandwich / covariance tests, FID
# component timing, then the existing FID / eigenvalue tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/gpu/test_k5_pending.py \
  > gpurun_out/r6b_pending.log 2>&1 || { tail -40 gpurun_out/r6b_pending.log; exit 1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/gpu/test_k9d_cholesky.py \
  > gpurun_out/r6b_k9d.log 2>&1 || { tail -60 gpurun_out/r6b_k9d.log; exit 1; }
timeout -k 10 240 python -u benchmarks/fid_compute_timing.py > gpurun_out/r6b_fid_timing.json 2> gpurun_out/r6b_fid_timing.err \
  || { tail -20 gpurun_out/r6b_fid_timing.err; exit 1; }
cat gpurun_out/r6b_fid_timing.json
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py \
  tests/gpu -k "fid or frechet or image" > gpurun_out/r6b_fid_tests.log 2>&1 || { tail -40 gpurun_out/r6b_fid_tests.log; exit 1; }
tail -2 gpurun_out/r6b_fid_tests.log
