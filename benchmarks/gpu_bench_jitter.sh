#!/bin/bash
# bench.py's single ~140 us timed region on a loaded host: the driver command repeated, plain /
# with a 2 ms sleep before the region / with the HIP runtime spinning longer before it blocks
# in a synchronize (interleaved), then the median of 100 regions for reference.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
uptime
v() { python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])"; }
for i in 1 2 3 4 5; do
  a=$(timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | v)
  b=$(BENCH_PRESLEEP_MS=2 timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | v)
  c=$(ROC_ACTIVE_WAIT_TIMEOUT=2000 timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | v)
  echo "plain $a presleep $b activewait $c"
done
timeout -k 10 120 python benchmarks/host_cost_anatomy.py 2>/dev/null
uptime
