#!/bin/bash
# Benchmark session: BASELINE-table suite (native vs eager ATen on the same GPU), the
# north-star bench.py, and a rocprofv3 kernel-stats capture of the suite's native path.
# Only the *_stats.csv summaries are kept (gpurun copies back at most 64 MiB).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python benchmarks/bench_suite.py --out gpurun_out/bench_suite.json "$@" > gpurun_out/bench_suite.log 2>&1 || { tail -20 gpurun_out/bench_suite.log; exit 1; }
tail -25 gpurun_out/bench_suite.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_suite
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_suite -o suite -- python3 "$GRAFT_REPO_ROOT/benchmarks/bench_suite.py" --no-aten --min-time 0.2 "$@" > "$GRAFT_REPO_ROOT/gpurun_out/prof_suite.log" 2>&1
# rocprofv3 has crashed at process exit after writing its output on this image; keep the files
echo "rocprofv3 rc=$?"
find /tmp/prof_suite -name "*_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/" \;
ls "$GRAFT_REPO_ROOT/gpurun_out/"
