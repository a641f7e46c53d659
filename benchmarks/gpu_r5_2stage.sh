#!/bin/bash
# two-stage K9b costing: stage 1 (dense -> band) on rocSOLVER geqrf + FP64 GEMMs, timings and a
# kernel-stats profile; plus the opt-in wave-kernel test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py -k wave > gpurun_out/r5_wave_test.log 2>&1 || { tail -30 gpurun_out/r5_wave_test.log; exit 1; }
tail -1 gpurun_out/r5_wave_test.log
timeout -k 10 400 python3 -u benchmarks/fid_two_stage_probe.py --b 16 32 64 > gpurun_out/fid_two_stage_r5.jsonl 2> gpurun_out/fid_two_stage.err || { tail -20 gpurun_out/fid_two_stage.err; exit 1; }
cat gpurun_out/fid_two_stage_r5.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2s -o run -- python3 benchmarks/fid_two_stage_probe.py --b 32 > gpurun_out/prof2s.log 2>&1 || { tail -20 gpurun_out/prof2s.log; exit 1; }
f=$(find gpurun_out/prof2s -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/fid_two_stage_kernel_stats_b32.csv; head -15 gpurun_out/fid_two_stage_kernel_stats_b32.csv | cut -c1-200
