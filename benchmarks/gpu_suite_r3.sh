#!/bin/bash
# Round-3 refresh of the BASELINE.md suite (native vs eager ATen on the same GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u benchmarks/bench_suite.py --out gpurun_out/bench_suite_r3.json > gpurun_out/bench_suite_r3.log 2>&1 || { tail -30 gpurun_out/bench_suite_r3.log; exit 1; }
tail -45 gpurun_out/bench_suite_r3.log
