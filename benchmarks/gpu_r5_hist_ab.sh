#!/bin/bash
# K3a onesweep histogram geometry A/B: 4096 x h keys per block
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k3_onesweep.py > gpurun_out/r5_hist_tests.log 2>&1 || { tail -40 gpurun_out/r5_hist_tests.log; exit 1; }
tail -1 gpurun_out/r5_hist_tests.log
K3_AB_HIST_ROUNDS=1,2,4,8,1 timeout -k 10 500 python3 benchmarks/k3_onesweep_ab.py > gpurun_out/k3_hist_ab_r5.jsonl 2> gpurun_out/k3_hist_ab.err || { tail -20 gpurun_out/k3_hist_ab.err; exit 1; }
cut -c1-120 gpurun_out/k3_hist_ab_r5.jsonl
