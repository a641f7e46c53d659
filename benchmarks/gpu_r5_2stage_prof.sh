#!/bin/bash
# kernel stats of the two-stage stage-1 probe (b = 32, 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 32 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2s_b$b -o run -- python3 benchmarks/fid_two_stage_probe.py --b $b > gpurun_out/prof2s_b$b.log 2>&1 || { tail -20 gpurun_out/prof2s_b$b.log; exit 1; }
  f=$(find gpurun_out/prof2s_b$b -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] || { find gpurun_out/prof2s_b$b | head; exit 1; }
  cp "$f" gpurun_out/fid_two_stage_kernel_stats_b$b.csv
  cut -c1-160 gpurun_out/fid_two_stage_kernel_stats_b$b.csv | head -12
done
