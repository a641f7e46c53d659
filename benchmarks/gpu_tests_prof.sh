#!/bin/bash
# whole GPU test suite, then the torch.profiler breakdown of selected suite cases
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_full.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_full.log | head -20; exit 1; }
bash benchmarks/gpu_profile_ops.sh
