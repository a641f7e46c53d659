#!/bin/bash
# round 6, call X: K9d 4-wave diagonal factorisation - tests, trace, FID timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/gpu/test_k9d_cholesky.py \
  tests/gpu/test_k9p_pivchol.py > gpurun_out/r6x_tests.log 2>&1 || { tail -40 gpurun_out/r6x_tests.log; exit 1; }
tail -1 gpurun_out/r6x_tests.log
timeout -k 10 120 python -u benchmarks/k9d_trace.py 2048 > gpurun_out/r6x_k9d_trace.json 2> gpurun_out/r6x.err || { tail -20 gpurun_out/r6x.err; exit 1; }
cat gpurun_out/r6x_k9d_trace.json
timeout -k 10 300 python -u benchmarks/bench_suite.py --only FID --out gpurun_out/r6x_fid.json > gpurun_out/r6x_fid.log 2>&1 || { tail -20 gpurun_out/r6x_fid.log; exit 1; }
grep "FID compute" gpurun_out/r6x_fid.log
