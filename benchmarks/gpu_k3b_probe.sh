#!/bin/bash
# K3b per-block phase stamps (csrc/bench/k3b_probe.bin) at a few sizes, then the parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/k3b_probe.txt
for args in "32768" "1000000" "1000000 normal" "2097152"; do
  timeout -k 10 60 ./csrc/bench/k3b_probe.bin $args >> gpurun_out/k3b_probe.txt 2>&1 || { cat gpurun_out/k3b_probe.txt; exit 1; }
done
if [ -x ./csrc/bench/k3b_probe_linear.bin ]; then
  echo "--- linear (coalesced, wrong-place) scatter stores: timing experiment" >> gpurun_out/k3b_probe.txt
  timeout -k 10 60 ./csrc/bench/k3b_probe_linear.bin 1000000 >> gpurun_out/k3b_probe.txt 2>&1 || { cat gpurun_out/k3b_probe.txt; exit 1; }
fi
cat gpurun_out/k3b_probe.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/gpu/test_k3b_bucket_auc.py > gpurun_out/t_k3b.log 2>&1 || { tail -40 gpurun_out/t_k3b.log; exit 1; }
tail -3 gpurun_out/t_k3b.log
