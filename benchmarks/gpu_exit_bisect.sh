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
for mode in coop plain; do
  rm -rf /tmp/pc_$mode
  (cd /tmp && timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pc_$mode -o $mode -- \
    "$GRAFT_REPO_ROOT/csrc/bench/coop_exit_probe.bin" $mode > "$GRAFT_REPO_ROOT/gpurun_out/exit_bisect/probe_$mode.log" 2>&1)
  echo "bare HIP $mode launch rc=$?"
done
rm -rf /tmp/pb_eig_plain
(cd /tmp && TORCHEVAL_AMD_SYMEIG_COOP=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pb_eig_plain -o eigp -- \
  python3 "$GRAFT_REPO_ROOT/benchmarks/exit_bisect.py" eig > "$GRAFT_REPO_ROOT/gpurun_out/exit_bisect/eig_plain.log" 2>&1)
echo "stage eig with a plain launch rc=$?"
exit 0
