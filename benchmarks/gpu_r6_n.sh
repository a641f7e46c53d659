#!/bin/bash
# round 6, call N: 4-column potrf, unrolled phases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9d_cholesky.py \
  tests/gpu/test_k5_pending.py > gpurun_out/r6n_tests.log 2>&1 || { tail -60 gpurun_out/r6n_tests.log; exit 1; }
tail -1 gpurun_out/r6n_tests.log
timeout -k 10 120 python -u benchmarks/k9d_trace.py 2048 > gpurun_out/r6n_k9d_trace.json 2> gpurun_out/r6n.err || { tail -20 gpurun_out/r6n.err; exit 1; }
cat gpurun_out/r6n_k9d_trace.json
timeout -k 10 120 python -u benchmarks/k5b_probe.py > gpurun_out/r6n_k5b_probe.json 2>> gpurun_out/r6n.err || { tail -20 gpurun_out/r6n.err; exit 1; }
cat gpurun_out/r6n_k5b_probe.json
