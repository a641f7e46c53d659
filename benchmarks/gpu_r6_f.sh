#!/bin/bash
# round 6, call F: K9d trace with the wave-0 stamp
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u benchmarks/k9d_trace.py 2048 > gpurun_out/r6f_k9d_trace.json 2> gpurun_out/r6f.err || { tail -20 gpurun_out/r6f.err; exit 1; }
cat gpurun_out/r6f_k9d_trace.json
timeout -k 10 120 python -u benchmarks/k9d_trace.py 64 >> gpurun_out/r6f_k9d_trace.json 2>> gpurun_out/r6f.err || { tail -20 gpurun_out/r6f.err; exit 1; }
tail -1 gpurun_out/r6f_k9d_trace.json
