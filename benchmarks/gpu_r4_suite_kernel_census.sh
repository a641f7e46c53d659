#!/bin/bash
# Kernel census of the GPU test suite: rocprofv3 kernel stats over `pytest tests/gpu -m gpu`
# (K9b's plain launch: rocprofv3 crashes at exit after any cooperative launch, exit_bisect_r4/).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/prof_suite
(cd /tmp && TORCHEVAL_AMD_SYMEIG_COOP=0 timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
  -d /tmp/prof_suite -o suite -- python3 -m pytest "$GRAFT_REPO_ROOT/tests/gpu" -m gpu -q -x \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$GRAFT_REPO_ROOT/gpurun_out/prof_suite.log" 2>&1)
rc=$?
echo "rocprofv3 suite rc=$rc"; tail -3 gpurun_out/prof_suite.log
find /tmp/prof_suite -name "*kernel_stats.csv" -exec cp {} gpurun_out/suite_kernel_stats.csv \;
python3 - <<'PY'
import csv
rows = list(csv.reader(open("gpurun_out/suite_kernel_stats.csv")))
tea = [r for r in rows[1:] if "tea::" in r[0]]
print("kernels total", len(rows) - 1, "tea kernels", len(tea), "tea dispatches", sum(int(r[1]) for r in tea))
PY
exit $rc
