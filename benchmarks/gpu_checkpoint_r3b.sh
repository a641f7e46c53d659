#!/bin/bash
# Checkpoint: GPU suite + smoke + driver bench, rocprof kernel stats of the driver command,
# then the BASELINE.md suite refresh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash benchmarks/gpu_full.sh || exit 1
export TMPDIR=/tmp
rm -rf /tmp/prof_drv
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_drv -o drv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_drv.log" 2>&1) || { tail -20 gpurun_out/prof_drv.log; exit 1; }
find /tmp/prof_drv -name "*kernel_stats.csv" -exec cp {} gpurun_out/drv_kernel_stats.csv \;
head -3 gpurun_out/drv_kernel_stats.csv | cut -c1-160
timeout -k 10 1000 python3 -u benchmarks/bench_suite.py --out gpurun_out/bench_suite_r3b.json > gpurun_out/bench_suite_r3b.log 2>&1 || { tail -30 gpurun_out/bench_suite_r3b.log; exit 1; }
tail -42 gpurun_out/bench_suite_r3b.log
