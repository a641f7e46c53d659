#!/bin/bash
# K9b with the 512-thread default at D=2048: eigenvalue + FID GPU tests, timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu -k "fid or symeig or k9 or frechet or eig" > gpurun_out/r5_k9def_tests.log 2>&1 || { tail -30 gpurun_out/r5_k9def_tests.log; exit 1; }
tail -1 gpurun_out/r5_k9def_tests.log
timeout -k 10 240 python3 benchmarks/symeig_timing.py > gpurun_out/symeig_timing_nt512_default_r5.json 2> gpurun_out/symeig_def.err || { tail -20 gpurun_out/symeig_def.err; exit 1; }
cat gpurun_out/symeig_timing_nt512_default_r5.json
