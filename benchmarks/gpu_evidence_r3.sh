#!/bin/bash
# End-of-round evidence: steady-state bench, the timed region's fixed cost, 1-rank sync floors
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --gpus 1 --steps 5000 --warmup 200 --no-reference > gpurun_out/bench_5k_final.json 2> gpurun_out/b5k.err || { tail -20 gpurun_out/b5k.err; exit 1; }
cat gpurun_out/bench_5k_final.json
timeout -k 10 300 python3 benchmarks/bench_fixed_cost.py > gpurun_out/fixed_cost_final.json 2> gpurun_out/fc.err || { tail -20 gpurun_out/fc.err; exit 1; }
cat gpurun_out/fixed_cost_final.json
timeout -k 10 200 python3 benchmarks/rccl_sync_floor.py --out gpurun_out/sync_floor_final.json > /dev/null 2> gpurun_out/sf.err || { tail -20 gpurun_out/sf.err; exit 1; }
cat gpurun_out/sync_floor_final.json
