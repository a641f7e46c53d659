#!/bin/bash
# The opt-in / A-B arms against the GPU tests that exercise them (each arm's variable is read once
# per process): the legacy K3a sort, the K3 tile-sum fold, the rows-per-wave K9b reduction
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K3SEL="auroc or auprc or curve or k3 or retrieval or recall_at or precision_at"
TORCHEVAL_AMD_K3_ONESWEEP=0 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu -k "$K3SEL" > gpurun_out/arm_legacy_sort.log 2>&1 || { tail -30 gpurun_out/arm_legacy_sort.log; exit 1; }
echo "legacy sort: $(tail -1 gpurun_out/arm_legacy_sort.log)"
TORCHEVAL_AMD_K3_FOLD=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu -k "$K3SEL" > gpurun_out/arm_k3_fold.log 2>&1 || { tail -30 gpurun_out/arm_k3_fold.log; exit 1; }
echo "k3 fold: $(tail -1 gpurun_out/arm_k3_fold.log)"
TORCHEVAL_AMD_SYMEIG_WAVE=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu -k "fid or symeig or k9 or frechet or eig" > gpurun_out/arm_symeig_wave.log 2>&1 || { tail -30 gpurun_out/arm_symeig_wave.log; exit 1; }
echo "symeig wave: $(tail -1 gpurun_out/arm_symeig_wave.log)"
