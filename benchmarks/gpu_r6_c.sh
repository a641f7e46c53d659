#!/bin/bash
# round 6, call C: K9d batched re-poll; FID component timing incl. sandwich block counts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9d_cholesky.py \
  > gpurun_out/r6c_k9d.log 2>&1 || { tail -60 gpurun_out/r6c_k9d.log; exit 1; }
tail -1 gpurun_out/r6c_k9d.log
timeout -k 10 240 python -u benchmarks/fid_compute_timing.py > gpurun_out/r6c_fid_timing.json 2> gpurun_out/r6c_fid_timing.err \
  || { tail -20 gpurun_out/r6c_fid_timing.err; exit 1; }
cat gpurun_out/r6c_fid_timing.json
