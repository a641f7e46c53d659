#!/bin/bash
# Kernel stats of FID compute at D = 2048
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/prof_fid
# (under rocprofv3 this process has segfaulted in teardown AFTER the tool wrote its results: a
# non-zero exit is accepted when the stats file exists and the workload printed "done")
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_fid -o fid -- \
  python3 "$GRAFT_REPO_ROOT/benchmarks/profile_fid_compute.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_fid.log" 2>&1)
grep -q "^done" gpurun_out/prof_fid.log || { tail -20 gpurun_out/prof_fid.log; exit 1; }
find /tmp/prof_fid -name "*kernel_stats.csv" -exec cp {} gpurun_out/fid_compute_kernel_stats.csv \;
python3 - <<'PY'
import csv
for r in list(csv.reader(open("gpurun_out/fid_compute_kernel_stats.csv")))[:12]:
    print(r[0][:70], r[1], r[2], r[3])
PY
