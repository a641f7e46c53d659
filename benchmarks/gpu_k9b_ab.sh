#!/bin/bash
# K9b: GPU tests of the eigenvalue path, then the timing / hand-off A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py tests/gpu/test_k5_k7_k8.py > gpurun_out/t_k9b.log 2>&1 || { tail -30 gpurun_out/t_k9b.log; exit 1; }
tail -2 gpurun_out/t_k9b.log
timeout -k 10 300 python3 benchmarks/symeig_timing.py > gpurun_out/symeig_timing_r3b.json 2> gpurun_out/symeig_timing.err || { tail -20 gpurun_out/symeig_timing.err; exit 1; }
cat gpurun_out/symeig_timing_r3b.json
