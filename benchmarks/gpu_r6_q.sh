#!/bin/bash
# round 6, call Q: K9p pivoted Cholesky tests + rank-deficient FID timing + kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/gpu/test_k9p_pivchol.py \
  > gpurun_out/r6q_tests.log 2>&1 || { tail -60 gpurun_out/r6q_tests.log; exit 1; }
tail -3 gpurun_out/r6q_tests.log
timeout -k 10 200 python -u benchmarks/fid_singular_probe.py > gpurun_out/r6q_probe.json 2> gpurun_out/r6q.err || { tail -20 gpurun_out/r6q.err; exit 1; }
cat gpurun_out/r6q_probe.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r6q_prof" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/fid_singular_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/r6q_prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/r6q_prof.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/r6q_prof" -name "*kernel_stats.csv" | head -1 | xargs head -25
