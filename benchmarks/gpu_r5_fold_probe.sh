#!/bin/bash
# K3 fold cost split: full fold / fold without atomics / fold instantiation without fold work / no fold
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K3_AB_FOLD_PROBE=1 timeout -k 10 400 python3 benchmarks/k3_onesweep_ab.py > gpurun_out/k3_fold_probe_r5.jsonl 2> gpurun_out/k3_fold_probe.err || { tail -20 gpurun_out/k3_fold_probe.err; exit 1; }
cut -c1-200 gpurun_out/k3_fold_probe_r5.jsonl
