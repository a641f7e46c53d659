#!/bin/bash
# Order-dependence check: the GPU suite with its files in reverse order (one process), after the
# test-order-dependent race found in the direct-RCCL host wait this round.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
files=$(ls tests/gpu/test_*.py | sort -r | tr '\n' ' ')
timeout -k 10 900 python3 -u -m pytest $files -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_reverse.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_reverse.log; [ $rc -ne 0 ] && grep -E "FAILED|Error" gpurun_out/pytest_reverse.log | head -10
exit $rc
