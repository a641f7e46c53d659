#!/bin/bash
# The driver's exact bench command (--steps 20 --warmup 5), a 20k-step steady-state run for
# comparison, and rocprofv3 kernel stats of the exact driver command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20000 --warmup 1000 --no-reference > gpurun_out/bench_20k.json 2> gpurun_out/bench_20k.err || { tail -20 gpurun_out/bench_20k.err; exit 1; }
cat gpurun_out/bench_20k.json
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_driver
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_driver -o drv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_driver.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_driver.log"; exit 1; }
find /tmp/prof_driver -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/driver_kernel_stats.csv" \;
find /tmp/prof_driver -name "*kernel_trace.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/driver_kernel_trace.csv" \;
grep '"metric"' "$GRAFT_REPO_ROOT/gpurun_out/prof_driver.log"
echo ok
