#!/bin/bash
# K9b early exit of finished workgroups: numerics, then the timing A/B in separate processes.
# (The switch was removed after this A/B, profiles/k9b_early_exit_ab_r4.json: both arms now run the same kernel.)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/gpu/test_k9b_symeig.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k9b_tests.log 2>&1
rc=$?; tail -2 gpurun_out/k9b_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/k9b_tests.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 180 python benchmarks/symeig_timing.py > gpurun_out/k9b_exit_on_$i.json 2>&1 || { tail -5 gpurun_out/k9b_exit_on_$i.json; exit 1; }
  TORCHEVAL_AMD_SYMEIG_EARLY_EXIT=0 timeout -k 10 180 python benchmarks/symeig_timing.py > gpurun_out/k9b_exit_off_$i.json 2>&1 || { tail -5 gpurun_out/k9b_exit_off_$i.json; exit 1; }
  echo "on:  $(cat gpurun_out/k9b_exit_on_$i.json | tail -1)"
  echo "off: $(cat gpurun_out/k9b_exit_off_$i.json | tail -1)"
done
