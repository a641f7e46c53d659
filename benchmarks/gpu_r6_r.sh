#!/bin/bash
# round 6, call R: K9p (LDS-resident) tests, phase trace, rank-deficient FID timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 python -u benchmarks/k9p_trace.py > gpurun_out/r6r_trace.json 2> gpurun_out/r6r.err || { tail -20 gpurun_out/r6r.err; exit 1; }
cat gpurun_out/r6r_trace.json
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/gpu/test_k9p_pivchol.py \
  > gpurun_out/r6r_tests.log 2>&1 || { tail -60 gpurun_out/r6r_tests.log; exit 1; }
tail -3 gpurun_out/r6r_tests.log
timeout -k 10 200 python -u benchmarks/fid_singular_probe.py > gpurun_out/r6r_probe.json 2>> gpurun_out/r6r.err || { tail -20 gpurun_out/r6r.err; exit 1; }
cat gpurun_out/r6r_probe.json
