#!/bin/bash
# Which stage of the FID compute leaves the process to segfault in exit under rocprofv3?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/exit_bisect
export TMPDIR=/tmp
for st in import k1 chol eig fid; do
  rm -rf /tmp/pb_$st
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pb_$st -o $st -- \
    python3 "$GRAFT_REPO_ROOT/benchmarks/exit_bisect.py" $st > "$GRAFT_REPO_ROOT/gpurun_out/exit_bisect/$st.log" 2>&1)
  rc=$?
  echo "stage $st rc=$rc done=$(grep -c '^done' gpurun_out/exit_bisect/$st.log)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
done
exit 0
