#!/bin/bash
# round 6, call O: K9d potrf probes (results invalid in probe modes: timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for pr in 0 1 2 3 8; do
  TORCHEVAL_AMD_K9D_PROBE=$pr timeout -k 10 120 python -u benchmarks/k9d_trace.py 2048 > gpurun_out/r6o_probe$pr.json 2> gpurun_out/r6o.err || { tail -20 gpurun_out/r6o.err; exit 1; }
  echo "probe $pr: $(python3 -c "import json;d=json.load(open('gpurun_out/r6o_probe$pr.json'));print(d['total_us_first_stamp_to_last'], d['median_us_per_column'])")"
done
