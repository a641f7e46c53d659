#!/bin/bash
# K9b product-form Sturm counts: eigenvalue / FID tests, accuracy + FID compute probe, kernel timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6_sturm
mkdir -p $O

timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/gpu/test_k9b_symeig.py tests/gpu/test_k9p_pivchol.py tests/gpu/test_k9d_cholesky.py tests/metrics/image > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u benchmarks/k9b_tail_ab.py > $O/ab.json 2>$O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab.json
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pf
TORCHEVAL_AMD_SYMEIG_COOP=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/pf -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/fid_compute_probe.py" > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1
echo "rocprof rc=$?"
f=$(find /tmp/pf -name "*kernel_trace.csv" | head -1)
cp "$f" "$GRAFT_REPO_ROOT/$O/fid_kernel_trace.csv"
