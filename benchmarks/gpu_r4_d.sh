#!/bin/bash
# Round 4: K1 floor variants, sync host breakdown (direct plans), sync floor.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./csrc/bench/k1_floor.bin 8 400 > gpurun_out/k1_floor_r4c.txt 2>&1
rc=$?; cat gpurun_out/k1_floor_r4c.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python benchmarks/sync_breakdown.py > gpurun_out/sync_breakdown_r4.json 2> gpurun_out/sb.err
rc=$?; cat gpurun_out/sync_breakdown_r4.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/sb.err; exit $rc; }
timeout -k 10 300 python benchmarks/rccl_sync_floor.py > gpurun_out/sync_floor_r4.json 2> gpurun_out/sync_floor_r4.err
rc=$?; cat gpurun_out/sync_floor_r4.json; exit $rc
