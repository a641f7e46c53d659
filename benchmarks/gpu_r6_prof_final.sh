#!/bin/bash
# round 6 final profiles: bench.py kernel stats, a FETCH_SIZE pass over the headline kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6_prof
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pb /tmp/pm
[ -f "$R/gpurun_out/r6_prof/bench_kernel_stats.csv" ] || timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pb -o run -- python3 "$R/bench.py" --steps 2000 --warmup 200 > "$R/gpurun_out/r6_prof/bench_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/r6_prof/bench_prof.log"; exit 1; }
f=$(find /tmp/pb -name "*kernel_stats.csv" 2>/dev/null | head -1)
[ -n "$f" ] && cp "$f" "$R/gpurun_out/r6_prof/bench_kernel_stats.csv"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pm -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/r6_prof/bench_pmc.log" 2>&1 || { tail -5 "$R/gpurun_out/r6_prof/bench_pmc.log"; exit 1; }
f=$(find /tmp/pm -name "*counter_collection.csv" | head -1)
cp "$f" "$R/gpurun_out/r6_prof/bench_pmc.csv"
echo done
