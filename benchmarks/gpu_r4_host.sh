#!/bin/bash
# Host-cost anatomy of the north-star update: Python layers, and the same region from C++.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python benchmarks/host_cost_anatomy.py > gpurun_out/host_anatomy.json 2> gpurun_out/host_anatomy.err
rc=$?; cat gpurun_out/host_anatomy.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/host_anatomy.err; exit $rc; }
timeout -k 10 120 ./csrc/bench/k1_floor.bin 8 400 > gpurun_out/k1_floor_host.txt 2>&1
rc=$?; tail -2 gpurun_out/k1_floor_host.txt; exit $rc
