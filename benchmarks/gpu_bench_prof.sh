#!/bin/bash
# rocprofv3 kernel stats of the north-star bench.py (K1 pred-free path) + one FETCH_SIZE pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_bench /tmp/pmc_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -o bench -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5000 --warmup 200 --no-reference > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log"; exit 1; }
find /tmp/prof_bench -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/bench_kernel_stats.csv" \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc_bench -o pmc -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-reference > "$GRAFT_REPO_ROOT/gpurun_out/pmc_bench.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc_bench.log"; exit 1; }
find /tmp/pmc_bench -name "*counter_collection.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/bench_pmc.csv" \;
head -4 "$GRAFT_REPO_ROOT/gpurun_out/bench_kernel_stats.csv" | cut -c1-200
