#!/bin/bash
# K3 tile-sum fold into the last onesweep pass: its tests and every AUROC / AUPRC GPU test,
# then the wall-time A/B (fold on / off / legacy sort) and a kernel-stats profile (launch count)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k3_onesweep.py > gpurun_out/r5_fold_tests.log 2>&1 || { tail -40 gpurun_out/r5_fold_tests.log; exit 1; }
tail -1 gpurun_out/r5_fold_tests.log
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu -k "auroc or auprc or curve or k3 or retrieval or recall_at" > gpurun_out/r5_fold_tests2.log 2>&1 || { tail -40 gpurun_out/r5_fold_tests2.log; exit 1; }
tail -1 gpurun_out/r5_fold_tests2.log
timeout -k 10 400 python3 benchmarks/k3_onesweep_ab.py > gpurun_out/k3_fold_ab_r5.jsonl 2> gpurun_out/k3_fold_ab.err || { tail -20 gpurun_out/k3_fold_ab.err; exit 1; }
cat gpurun_out/k3_fold_ab_r5.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fold -o run -- python3 benchmarks/profile_auroc_1m.py > gpurun_out/prof_fold.log 2>&1 || { tail -20 gpurun_out/prof_fold.log; exit 1; }
f=$(find gpurun_out/prof_fold -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/k3_fold_kernel_stats.csv
cut -c1-150 gpurun_out/k3_fold_kernel_stats.csv | head -12
