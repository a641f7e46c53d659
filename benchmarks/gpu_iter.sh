#!/bin/bash
# Kernel iteration loop: gpu tests matching $1 (pytest -k expr), then profile_ops cases $2...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K="$1"; shift
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "$K" > gpurun_out/iter_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/iter_pytest.log
[ $rc -ne 0 ] && exit $rc
if [ $# -gt 0 ]; then
  timeout -k 10 300 python benchmarks/profile_ops.py "$@" > gpurun_out/iter_profile.log 2>&1 || { tail -30 gpurun_out/iter_profile.log; exit 1; }
  grep -E "#####|tea::|Self CUDA" gpurun_out/iter_profile.log | cut -c1-60,140-175
fi
