#!/bin/bash
# K9b v2 (rows per wave): eigenvalue tests with the wave kernel, then the timing A/B against
# tridiag_kernel (TORCHEVAL_AMD_SYMEIG_WAVE=0); plus the K4b large-threshold test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py > gpurun_out/r5_k9w_tests.log 2>&1 || { tail -30 gpurun_out/r5_k9w_tests.log; exit 1; }
tail -2 gpurun_out/r5_k9w_tests.log
timeout -k 10 240 python3 benchmarks/symeig_timing.py > gpurun_out/symeig_timing_wave_r5.json 2> gpurun_out/symeig_timing_wave.err || { tail -20 gpurun_out/symeig_timing_wave.err; exit 1; }
cat gpurun_out/symeig_timing_wave_r5.json
TORCHEVAL_AMD_SYMEIG_WAVE=0 timeout -k 10 240 python3 benchmarks/symeig_timing.py > gpurun_out/symeig_timing_block_r5.json 2> gpurun_out/symeig_timing_block.err || { tail -20 gpurun_out/symeig_timing_block.err; exit 1; }
cat gpurun_out/symeig_timing_block_r5.json
timeout -k 10 240 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k4b_sample_binned_auroc.py > gpurun_out/r5_k4b_tests.log 2>&1 || { tail -30 gpurun_out/r5_k4b_tests.log; exit 1; }
tail -2 gpurun_out/r5_k4b_tests.log
