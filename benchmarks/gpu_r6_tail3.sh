#!/bin/bash
# K9b tail tile-height A/B: kernel timelines of FID compute at TR = 8 / 4 / 2, then tests at the default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r6_tail3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for tr in 8 4 2; do
  rm -rf /tmp/pf
  TORCHEVAL_AMD_SYMEIG_TAIL_TR=$tr TORCHEVAL_AMD_SYMEIG_COOP=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/pf -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/fid_compute_probe.py" > "$O/prof_$tr.log" 2>&1 || { echo "rocprof TR=$tr failed"; tail -5 $O/prof_$tr.log; exit 1; }
  f=$(find /tmp/pf -name "*kernel_trace.csv" | head -1)
  cp "$f" "$O/trace_$tr.csv"
  tail -1 "$O/prof_$tr.log"
done
cd "$GRAFT_REPO_ROOT"
for tr in 8 4 2; do
  TORCHEVAL_AMD_SYMEIG_TAIL_TR=$tr timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py > $O/tests_$tr.log 2>&1 || { tail -30 $O/tests_$tr.log; exit 1; }
  tail -1 $O/tests_$tr.log
done
