#!/bin/bash
# torch.profiler host + device breakdown of selected suite cases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u benchmarks/profile_ops.py "mean_squared_error" "r2_score" "Sum.update" "perplexity" "multilabel_precision_recall_curve" "binary_binned_auroc" "multiclass_precision_recall_curve" > gpurun_out/profile_ops.txt 2>&1 || { tail -30 gpurun_out/profile_ops.txt; exit 1; }
grep -E "^#####|Self CUDA time total|Self CPU time total" gpurun_out/profile_ops.txt
