#!/bin/bash
# Round 5: K3a onesweep with spread digit totals (tests, A/B, kernel trace) + K5b VPT 16 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash benchmarks/gpu_r5_k3.sh || exit 1
TORCHEVAL_AMD_K5B_PEND_VPT=16 timeout -k 10 120 python -u benchmarks/k5b_pend_ab.py > gpurun_out/r5_k5b_ab_vpt16.json 2>&1 || { tail -20 gpurun_out/r5_k5b_ab_vpt16.json; exit 1; }
cat gpurun_out/r5_k5b_ab_vpt16.json
