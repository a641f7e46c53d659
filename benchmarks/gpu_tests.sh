#!/bin/bash
# GPU test session: the gpu-marked kernel tests, then the whole CPU suite with the ROCm device
# visible (MetricClassTester then runs every class metric on cpu AND cuda).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=25 "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m "not gpu" -q -x -p no:cacheprovider > gpurun_out/pytest_cpu_on_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_cpu_on_gpu.log
exit $rc
