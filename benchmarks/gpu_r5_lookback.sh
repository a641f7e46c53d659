#!/bin/bash
# K3a onesweep look-back with batched re-polls: tests, per-phase trace, wall-time A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k3_onesweep.py > gpurun_out/r5_lb_tests.log 2>&1 || { tail -40 gpurun_out/r5_lb_tests.log; exit 1; }
tail -1 gpurun_out/r5_lb_tests.log
timeout -k 10 120 ./csrc/bench/k3_pass_trace.bin > gpurun_out/k3_pass_trace_batched_r5.txt 2>&1 || { cat gpurun_out/k3_pass_trace_batched_r5.txt; exit 1; }
cat gpurun_out/k3_pass_trace_batched_r5.txt
timeout -k 10 400 python3 benchmarks/k3_onesweep_ab.py > gpurun_out/k3_lb_ab_r5.jsonl 2> gpurun_out/k3_lb_ab.err || { tail -20 gpurun_out/k3_lb_ab.err; exit 1; }
cut -c1-140 gpurun_out/k3_lb_ab_r5.jsonl
