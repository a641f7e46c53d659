#!/bin/bash
# The driver command repeated on one (shared, loaded) box, plus the in-process region series
# (benchmarks/bench_region_series.py) for the same box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
uptime
v() { python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])"; }
for i in 1 2 3 4 5 6; do
  echo "bench $(timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | v)"
done
timeout -k 10 120 python benchmarks/bench_region_series.py 2>/dev/null
uptime
