#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu -k "auroc or auprc or curve or sortscan or k3" > gpurun_out/t_k3.log 2>&1 || { tail -30 gpurun_out/t_k3.log; exit 1; }
tail -2 gpurun_out/t_k3.log
bash benchmarks/gpu_k3_profile.sh > gpurun_out/k3_prof_out.txt 2>&1 || { tail -20 gpurun_out/k3_prof_out.txt; exit 1; }
bash benchmarks/gpu_overlap.sh
