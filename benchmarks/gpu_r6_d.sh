#!/bin/bash
# round 6, call D: K9d phase trace; K5b per-statistic costs (PSNR / CTR vs Sum / MSE / WC)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u benchmarks/k9d_trace.py 2048 > gpurun_out/r6d_k9d_trace.json 2> gpurun_out/r6d.err || { tail -20 gpurun_out/r6d.err; exit 1; }
cat gpurun_out/r6d_k9d_trace.json
timeout -k 10 120 python -u benchmarks/k9d_trace.py 128 >> gpurun_out/r6d_k9d_trace.json 2>> gpurun_out/r6d.err || { tail -20 gpurun_out/r6d.err; exit 1; }
tail -1 gpurun_out/r6d_k9d_trace.json
timeout -k 10 120 python -u benchmarks/k5b_probe.py > gpurun_out/r6d_k5b_probe.json 2>> gpurun_out/r6d.err || { tail -20 gpurun_out/r6d.err; exit 1; }
cat gpurun_out/r6d_k5b_probe.json
