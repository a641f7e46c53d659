#!/bin/bash
# K9b register-resident tail: tests, A/B (tail on / off / on), FID compute kernel timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6_tail2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py tests/gpu/test_k9p_pivchol.py tests/metrics/image > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_on.json 2>$O/ab_on.err &&
TORCHEVAL_AMD_SYMEIG_TAIL=0 timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_off.json 2>$O/ab_off.err &&
timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab_on2.json 2>$O/ab_on2.err || { cat $O/ab_*.err | tail; exit 1; }
cat $O/ab_*.json
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pf
TORCHEVAL_AMD_SYMEIG_COOP=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/pf -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/fid_compute_probe.py" > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1
echo "rocprof rc=$?"
f=$(find /tmp/pf -name "*kernel_trace.csv" | head -1)
cp "$f" "$GRAFT_REPO_ROOT/$O/fid_kernel_trace.csv"
