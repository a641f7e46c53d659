#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/k3b_probe.txt
for args in "32768" "1000000"; do
  timeout -k 10 60 ./csrc/bench/k3b_probe.bin $args >> gpurun_out/k3b_probe.txt 2>&1 || { cat gpurun_out/k3b_probe.txt; exit 1; }
done
cat gpurun_out/k3b_probe.txt
