#!/bin/bash
# round 6, call G: pipelined K9d potrf - tests + trace + FID timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9d_cholesky.py \
  > gpurun_out/r6g_tests.log 2>&1 || { tail -60 gpurun_out/r6g_tests.log; exit 1; }
tail -1 gpurun_out/r6g_tests.log
timeout -k 10 120 python -u benchmarks/k9d_trace.py 2048 > gpurun_out/r6g_k9d_trace.json 2> gpurun_out/r6g.err || { tail -20 gpurun_out/r6g.err; exit 1; }
cat gpurun_out/r6g_k9d_trace.json
