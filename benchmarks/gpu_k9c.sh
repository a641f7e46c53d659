#!/bin/bash
# K9 GPU tests, the symeig timing JSON and the Cholesky host/device probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash benchmarks/gpu_k9b_ab.sh || exit 1
timeout -k 10 200 python3 benchmarks/fid_chol_host_probe.py 2>/dev/null | tail -1
